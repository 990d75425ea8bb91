"""Committed golden vectors (tests/golden/golden.npz, oracle-generated; see
tests/golden/make_golden.py) against the oracle (CPU) and the HIP path (GPU)."""
import os

import numpy as np
import pytest

from tests.golden.make_golden import CASES, CONFIGS, inputs, sha

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN, allow_pickle=False)


def _same(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8),
                                                                        b.view(np.uint8))


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_inputs_unchanged(golden, case):
    name, n, H, W, dt, mode, gen = case
    L, R = inputs(n, H, W, dt, gen)
    assert str(golden[name + "/inputs_sha256"]) == sha(L) + sha(R)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_reproduces_golden(oracle, golden, case):
    name, n, H, W, dt, mode, gen = case
    L, R = inputs(n, H, W, dt, gen)
    for cname, cfg in CONFIGS:
        d, corr = oracle.match(L, R, oracle.OracleConfig(mode=mode, **cfg))
        assert _same(d, golden["%s/%s/disparity" % (name, cname)]), (name, cname)
        if corr is not None:
            assert _same(corr, golden["%s/%s/corrmap" % (name, cname)]), (name, cname)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_gpu_reproduces_golden(gpu, golden, case):
    import torch
    from libbicos_amd.device import MatchConfig
    name, n, H, W, dt, mode, gen = case
    L, R = inputs(n, H, W, dt, gen)

    def dev(a):
        a = np.ascontiguousarray(a)
        return torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a).cuda()

    for cname, cfg in CONFIGS:
        d, corr = gpu.match(dev(L), dev(R), MatchConfig(mode=mode, **cfg))
        assert _same(d.cpu().numpy(), golden["%s/%s/disparity" % (name, cname)]), (name, cname)
        if corr is not None:
            assert _same(corr.cpu().numpy(), golden["%s/%s/corrmap" % (name, cname)]), (name, cname)


# ------------------------------------------ whole-frame fixtures (tests/golden/frames.json)
def _frames():
    import json
    return json.load(open(os.path.join(os.path.dirname(GOLDEN), "frames.json")))


def test_frames_cover_every_config():
    from tests.golden.make_frames import (FRAMES, SEARCH_FLAGS, SEARCH_FRAMES, SEARCH_INPUTS,
                                          SEARCH_SHAPE)
    db = _frames()
    assert sorted(db) == sorted(list(FRAMES) + list(SEARCH_FRAMES))
    for name, spec in FRAMES.items():
        n, H, W, cfg = spec[:4]
        gen = spec[4] if len(spec) > 4 else {}
        r = db[name]
        assert (r["n"], r["H"], r["W"], r["config"]) == (n, H, W, cfg), name
        assert (r["dtype"], r.get("maxval")) == (gen.get("dtype", "u8"), gen.get("maxval")), name
        assert len(r["disparity_bands"]) == -(-H // r["band_rows"])
    for name, (kind, fl) in SEARCH_FRAMES.items():
        r = db[name]
        assert (r["H"], r["W"], r["words"]) == SEARCH_SHAPE + (SEARCH_INPUTS[kind],)
        assert (r["input"], r["flags"], r["max_lr_diff"]) == (kind,) + SEARCH_FLAGS[fl]
        assert len(r["disparity_bands"]) == -(-r["H"] // r["band_rows"])


# Band 0 (the first 64 rows) of every round-4 fixture regenerates from the committed
# generators + the oracle to the committed band hash (rows are independent: SURVEY.md s8 e).
# The whole frames take minutes each; make_frames.py rebuilds them.
@pytest.mark.parametrize("name", ["full_n6", "full_n8", "full_n12", "full_n16", "full_n8_s25",
                                  "full_n16_s10", "cfg2_u16", "cfg3_u16"])
def test_oracle_reproduces_frame_band0(oracle, name):
    from tests.golden.make_frames import FRAMES, band_hashes, frame_stacks
    rec = _frames()[name]
    rows = rec["band_rows"]
    L, R = frame_stacks(FRAMES[name], 0, rows)
    d, c = oracle.match(L, R, oracle.OracleConfig(**rec["config"]))
    assert band_hashes(d, rows)[0] == rec["disparity_bands"][0]
    assert band_hashes(c, rows)[0] == rec["corrmap_bands"][0]


@pytest.mark.parametrize("kind", ["random", "periodic64", "lowtex", "random_u32", "random_u64"])
def test_oracle_reproduces_search_band0(oracle, kind):
    from tests.golden.make_frames import SEARCH_FLAGS, band_hashes, search_inputs
    db = _frames()
    rows = db["search_%s_nodupes" % kind]["band_rows"]
    d0, d1, bits = search_inputs(kind, oracle, 0, rows)
    for fl, (flags, lr) in SEARCH_FLAGS.items():
        rec = db["search_%s_%s" % (kind, fl)]
        assert rec["bits"] == bits
        d = oracle.search(d0, d1, flags, lr)
        assert band_hashes(d, rows)[0] == rec["disparity_bands"][0], fl


def test_oracle_reproduces_frame_cfg1(oracle):
    """The cheapest whole frame (BASELINE cfg1) regenerates from the committed generator +
    oracle to the same hashes (the others take minutes; make_frames.py rebuilds them)."""
    from libbicos_amd.synthetic import stereo_stack
    from tests.golden.make_frames import frame_record
    rec = _frames()["cfg1"]
    L, R = stereo_stack(rec["n"], rec["H"], rec["W"])
    d, c = oracle.match(L, R, oracle.OracleConfig(**rec["config"]))
    assert frame_record(rec["n"], rec["H"], rec["W"], rec["config"], L, R, d, c) == rec
