"""GPU parity: the gfx950 HIP path vs the CPU oracle, through the C-ABI.

Bar (north star): integer disparities bit-exact; nxcorr / subpixel floats within
1e-4 -- the kernels are written to be bit-exact there too, and these tests
demand exact equality (the tolerance is only used for Precision::DOUBLE, which
has no CPU oracle: |corr - float64 numpy| <= 1e-12).
"""
import contextlib
import numpy as np
import pytest

from libbicos_amd import _lib
from libbicos_amd.synthetic import random_stack, stereo_stack
from oracle import ref_numpy as N

pytestmark = pytest.mark.gpu

FLOAT_TOL = 1e-4  # north-star tolerance for nxcorr/subpixel floats (we assert exact below)


def dev(a):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    return torch.from_numpy(a).cuda()


def host(t):
    return t.cpu().numpy()


def same(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    assert a.dtype == b.dtype, (a.dtype, b.dtype)
    if not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
        if a.dtype.kind == "f":
            both = np.isnan(a) & np.isnan(b)
            diff = np.abs(a.astype(np.float64) - b.astype(np.float64))
            diff[both] = 0
            bad = np.argwhere(~(diff == 0))
            raise AssertionError("%d float mismatches, max |d| %g, first %s: %r vs %r" % (
                len(bad), np.nanmax(diff), bad[0], a[tuple(bad[0])], b[tuple(bad[0])]))
        bad = np.argwhere(a != b)
        raise AssertionError("%d mismatches, first %s: %r vs %r" % (
            len(bad), bad[0], a[tuple(bad[0])], b[tuple(bad[0])]))


def cfg_of(O, **kw):
    return O.OracleConfig(**kw)


def gpu_match(eng, L, R, **kw):
    from libbicos_amd.device import MatchConfig
    d, c = eng.match(dev(L), dev(R), MatchConfig(**kw))
    return host(d), (host(c) if c is not None else None)


# ----------------------------------------------------------------- transform
@pytest.mark.parametrize("n,mode,dt", [
    (2, 0, np.uint8), (3, 0, np.uint8), (4, 0, np.uint8), (8, 0, np.uint8), (9, 0, np.uint16),
    (10, 0, np.uint8), (17, 0, np.uint8), (33, 0, np.uint8), (33, 0, np.uint16),
    (40, 0, np.uint8), (45, 0, np.uint8), (65, 0, np.uint16),
    (2, 1, np.uint8), (3, 1, np.uint8), (4, 1, np.uint8), (8, 1, np.uint16), (10, 1, np.uint8),
    (16, 1, np.uint8),
])
def test_transform_bit_exact(gpu, oracle, n, mode, dt):
    s = random_stack(n, 13, 301, dt, seed=n * 7 + mode)
    words = oracle.desc_words(n, mode)
    ref = oracle.transform(s, mode, words)
    out = host(gpu.transform(dev(s), mode, words)).view(np.uint32)
    same(out[:, : 301 * words].reshape(13, 301, words), ref)


# FULL transform, every n it supports (2..16: each its own static kernel), u8 and u16,
# extreme values present; and a wider descriptor than the match would pick (the generic
# kernel)
@pytest.mark.parametrize("n", list(range(2, 17)))
@pytest.mark.parametrize("dt", [np.uint8, np.uint16])
def test_transform_full_every_n(gpu, oracle, n, dt):
    s = random_stack(n, 6, 257, dt, seed=900 + n)
    s[:, 0, :5] = 0
    s[:, 1, :5] = np.iinfo(dt).max
    words = oracle.desc_words(n, 1)
    ref = oracle.transform(s, 1, words)
    out = host(gpu.transform(dev(s), 1, words)).view(np.uint32)
    same(out[:, : 257 * words].reshape(6, 257, words), ref)
    if words < 8:
        wide = 2 * words
        ref2 = oracle.transform(s, 1, wide)
        out2 = host(gpu.transform(dev(s), 1, wide)).view(np.uint32)
        same(out2[:, : 257 * wide].reshape(6, 257, wide), ref2)


# u8 LIMITED transform over every n bucket, exact and padded, on random stacks with the
# extreme values 0 / 255 present, and on a plane-pitch-padded view (a 4-pixels-per-lane
# form of the transform was measured slower in round 3: profiles/quad_px_r03.jsonl)
@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 9, 10, 12, 16, 17, 23, 24, 25, 32, 33, 34, 40,
                               41, 47, 48, 49, 64, 65])
def test_transform_limited_u8_buckets(gpu, oracle, n):
    mode = 0
    s = random_stack(n, 9, 324, np.uint8, seed=500 + n)
    s[:, 0, :8] = 0
    s[:, 1, :8] = 255
    s[n // 2, 2, 4:12] = 255
    words = oracle.desc_words(n, mode)
    ref = oracle.transform(s, mode, words)
    out = host(gpu.transform(dev(s), mode, words)).view(np.uint32)
    same(out[:, : 324 * words].reshape(9, 324, words), ref)


@pytest.mark.parametrize("n,mode,dt,W,P", [
    (33, 0, np.uint8, 200, 256),    # dword-aligned rows
    (33, 0, np.uint8, 201, 257),    # odd byte pitch
    (17, 0, np.uint16, 301, 302),   # u16, 604-byte rows
    (17, 0, np.uint16, 301, 303),   # u16, 606-byte rows
    (12, 1, np.uint8, 259, 260),    # FULL (static-n kernel)
    (12, 1, np.uint8, 259, 261),
    (9, 0, np.uint8, 5, 8),         # one partial tile
])
def test_transform_padded_pitches(gpu, oracle, n, mode, dt, W, P):
    """Padded row pitches / plane strides (aligned and odd), u8 / u16, LIMITED / FULL,
    against the oracle."""
    import torch
    H = 11
    s = random_stack(n, H, W, dt, seed=77 + W)
    tdt = torch.uint8 if dt == np.uint8 else torch.int16
    buf = torch.zeros((n, H + 3, P), dtype=tdt, device="cuda")
    buf[:, :H, :W] = dev(s)
    words = oracle.desc_words(n, mode)
    out = host(gpu.transform(buf[:, :H, :W], mode, words)).view(np.uint32)
    same(out[:, : W * words].reshape(H, W, words), oracle.transform(s, mode, words))


# -------------------------------------------------------------------- search
def _low_entropy_desc(H, W, words, seed, bits=6):
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    mask = np.uint32((1 << bits) - 1)
    d[..., 1:] = 0
    d[..., 0] &= mask     # forces many exact duplicate minima
    return d


def _pack(desc):
    H, W, words = desc.shape
    from libbicos_amd import _lib
    pitch = _lib.lib().bicos_desc_pitch(W, words)
    out = np.zeros((H, pitch), np.uint32)
    out[:, : W * words] = desc.reshape(H, W * words)
    return out.view(np.int32)


@pytest.mark.parametrize("words", [1, 2, 4, 8])
@pytest.mark.parametrize("flags,lr", [(1, -1), (2, 1), (3, 1), (2, 0), (3, 5)])
@pytest.mark.parametrize("W", [1, 7, 64, 333, 1030])
def test_search_bit_exact(gpu, oracle, words, flags, lr, W):
    H = 5
    rng = np.random.default_rng(words * 1000 + W)
    d0 = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    d1 = d0[:, np.roll(np.arange(W), 3)] ^ (rng.random((H, W, words)) < 0.02).astype(np.uint32)
    for a, b in ((d0, d1), (_low_entropy_desc(H, W, words, 1), _low_entropy_desc(H, W, words, 2))):
        ref = oracle.search(a, b, flags, lr)
        out = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, flags, lr))
        same(out, ref)


def test_search_multi_chunk(gpu, oracle):
    # W * 32 B > 64 KiB LDS stage -> the right row is streamed in chunks
    H, W, words = 2, 3001, 8
    rng = np.random.default_rng(9)
    a = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    b = a[:, ::-1].copy()
    b[..., 0] ^= 1
    for flags, lr in ((1, -1), (3, 2)):
        same(host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, flags, lr)),
             oracle.search(a, b, flags, lr))


# --------------------------------------------------------------------- agree
@pytest.mark.parametrize("n,dt", [(2, np.uint8), (8, np.uint8), (33, np.uint8), (17, np.uint16),
                                  (40, np.uint8), (65, np.uint8)])
@pytest.mark.parametrize("minvar", [None, 2.0])
@pytest.mark.parametrize("W", [200, 203, 600])  # 4-byte aligned pitches: LDS-staged kernel
def test_agree_bit_exact(gpu, oracle, n, dt, minvar, W):
    H = 9
    L, R = stereo_stack(n, H, W, dt, dmin=3, drange=20, seed=n)
    rng = np.random.default_rng(n)
    raw = rng.integers(-5, 30, size=(H, W)).astype(np.int16)
    raw[rng.random((H, W)) < 0.2] = -32768
    R[:, 0, 40] = 9  # constant right pixel -> NaN correlation
    raw[0, 45] = 5
    mv = None if minvar is None else np.float32(minvar) * np.float32(n)
    rd, rc = oracle.agree(raw, L, R, 0.5, mv)
    out, corr = gpu.agree(dev(raw), dev(L), dev(R), 0.5, None if mv is None else float(mv))
    same(host(out), rd.astype(np.float32))
    same(host(corr), rc)


# agree over disparity patterns: flat runs, +-1/+-2 jitter, jumps, matches off either edge
# of the row, invalid pixels, negative disparities, NaN correlations (written for a
# 4-pixels-per-lane agree that was measured slower and dropped: profiles/quad_px_r03.jsonl)
@pytest.mark.parametrize("n", [2, 7, 8, 16, 24, 33, 40])
@pytest.mark.parametrize("minvar", [None, 2.0])
def test_agree_disparity_patterns(gpu, oracle, n, minvar):
    H, W = 8, 1024
    L, R = stereo_stack(n, H, W, np.uint8, dmin=3, drange=40, seed=n + 1000)
    rng = np.random.default_rng(n)
    raw = np.empty((H, W), np.int16)
    raw[0] = 17                                              # flat
    raw[1] = 20 + rng.integers(-1, 2, size=W)                # jitter within a lane
    raw[2] = 30 + rng.integers(-2, 3, size=W)
    raw[3] = np.where(np.arange(W) % 64 < 32, 5, 250)        # jumps wider than the window
    raw[4] = rng.integers(-40, 1100, size=W)                 # anything, incl. off-row matches
    raw[5] = 12
    raw[5, ::7] = -32768                                     # invalid pixels in flat runs
    raw[6] = np.arange(W) % 9 - 4                            # negative disparities (col1 > col0)
    raw[7] = 1023                                            # col1 = col0 - 1023: only col 1023 in row
    R[:, 0, 40:48] = 9                                       # flat right pixels: NaN correlations
    mv = None if minvar is None else np.float32(minvar) * np.float32(n)
    rd, rc = oracle.agree(raw, L, R, 0.5, mv)
    out, corr = gpu.agree(dev(raw), dev(L), dev(R), 0.5, None if mv is None else float(mv))
    same(host(out), rd.astype(np.float32))
    same(host(corr), rc)


# agree over disparity spreads 0..23 columns within 64 pixels at every alignment of the
# first matched column, invalid pixels and far outliers inside otherwise narrow waves, a width
# that is not a multiple of 4 inside a 4-byte aligned pitch (the last wave partly live). Written
# for a per-wave LDS window of the right samples (round 4, parity-green, measured slower:
# profiles/agree_win_r04.jsonl); kept for the LDS-tile agree.
@pytest.mark.parametrize("n", [2, 8, 9, 16, 17, 24, 25, 33])
def test_agree_window_spans(gpu, oracle, n):
    import torch
    H, W, P = 48, 1021, 1024
    L, R = stereo_stack(n, H, W, np.uint8, dmin=20, drange=4, seed=n + 77)
    y = np.arange(H)[:, None]
    x = np.arange(W)[None, :]
    raw = (20 + y % 4 + x % (y // 2 + 1)).astype(np.int16)
    raw[5::6, ::13] = -32768                  # invalid pixels
    raw[7::8, 100::97] = 500                  # outliers: that wave gathers per lane
    raw[3, :] = -32768                        # a row without any match
    raw[9, 960:] = -5                         # col1 > col0, and off the row's end
    R[:, 1, 200:210] = 7                      # constant right samples: NaN correlations
    buf0 = torch.zeros((n, H, P), dtype=torch.uint8, device="cuda")
    buf1 = torch.zeros((n, H, P), dtype=torch.uint8, device="cuda")
    buf0[:, :, :W] = dev(L)
    buf1[:, :, :W] = dev(R)
    for mv in (None, np.float32(2.0) * np.float32(n)):
        rd, rc = oracle.agree(raw, L, R, 0.5, mv)
        out, corr = gpu.agree(dev(raw), buf0[:, :, :W], buf1[:, :, :W], 0.5,
                              None if mv is None else float(mv))
        same(host(out), rd.astype(np.float32))
        same(host(corr), rc)


# n covers exact buckets and padded ones (2, 12, 25, 45, 60: slots n..MAXN-1 are exact
# no-ops) in both loop structures (pipelined MAXN <= 40, top-of-step above); steps cover
# 41/20/8 x values, 3 and a single x (step > 2)
@pytest.mark.parametrize("n,dt", [(2, np.uint8), (6, np.uint8), (8, np.uint8), (10, np.uint8),
                                  (12, np.uint8), (12, np.uint16), (16, np.uint8),
                                  (20, np.uint8), (25, np.uint8),
                                  (33, np.uint8), (33, np.uint16), (40, np.uint8),
                                  (45, np.uint16), (60, np.uint8), (65, np.uint8)])
@pytest.mark.parametrize("step,minvar", [(0.1, None), (0.25, 1.0), (0.05, None), (0.7, None),
                                         (2.5, 1.0)])
def test_subpixel_bit_exact(gpu, oracle, n, dt, step, minvar):
    H, W = 7, 160
    L = random_stack(n, H, W, dt, seed=n + 1)
    R = random_stack(n, H, W, dt, seed=n + 2)
    rng = np.random.default_rng(n)
    raw = rng.integers(-3, 12, size=(H, W)).astype(np.int16)
    raw[:, 3] = 3            # col1 == 0 edge
    raw[:, W - 1] = 0        # col1 == W-1 edge
    raw[rng.random((H, W)) < 0.1] = -32768
    mv = None if minvar is None else np.float32(minvar) * np.float32(n)
    ro, rc = oracle.agree_subpixel(raw, L, R, 0.2, step, mv)
    out, corr = gpu.agree(dev(raw), dev(L), dev(R), 0.2, None if mv is None else float(mv),
                          step=step)
    same(host(out), ro)
    same(host(corr), rc)


# Subpixel over several tiles per row with mixed rows: matches spread over 500 columns,
# rows without a valid match, matches on both edge columns, padded buckets.
@pytest.mark.parametrize("n,dt", [(8, np.uint8), (16, np.uint8), (25, np.uint8), (33, np.uint8),
                                  (12, np.uint16), (24, np.uint16), (33, np.uint16)])
def test_subpixel_mixed_rows(gpu, oracle, n, dt):
    H, W = 24, 512
    L = random_stack(n, H, W, dt, seed=3 * n + 1)
    R = random_stack(n, H, W, dt, seed=3 * n + 2)
    rng = np.random.default_rng(n + 100)
    raw = rng.integers(-3, 40, size=(H, W)).astype(np.int16)
    raw[3] = rng.integers(0, 500, size=W)       # matches spread over the whole row
    raw[5] = -32768                              # no match in the row
    raw[7, :] = np.arange(W) - (np.arange(W) % 2) * (W - 1)  # col1 = 0 / W-1 edges
    raw[rng.random((H, W)) < 0.1] = -32768
    ro, rc = oracle.agree_subpixel(raw, L, R, 0.2, 0.1, None)
    out, corr = gpu.agree(dev(raw), dev(L), dev(R), 0.2, None, step=0.1)
    same(host(out), ro)
    same(host(corr), rc)


# Narrow images and every col1 (0, 1, interior, cols-2, cols-1): the subpixel kernel reads
# the right neighbours with one window load except below 4 columns (byte loads).
@pytest.mark.parametrize("W", [3, 4, 5, 9])
@pytest.mark.parametrize("n,dt", [(8, np.uint8), (17, np.uint16), (33, np.uint8)])
def test_subpixel_narrow_images_every_col1(gpu, oracle, W, n, dt):
    H = 6
    L = random_stack(n, H, W, dt, seed=W + n)
    R = random_stack(n, H, W, dt, seed=W + n + 1)
    raw = np.empty((H, W), np.int16)
    for y in range(H):
        for x in range(W):
            raw[y, x] = x - ((x + y) % W)  # col1 = (x + y) % W: all columns appear
    ro, rc = oracle.agree_subpixel(raw, L, R, 0.1, 0.25, None)
    out, corr = gpu.agree(dev(raw), dev(L), dev(R), 0.1, None, step=0.25)
    same(host(out), ro)
    same(host(corr), rc)


# -------------------------------------------------------------- full match
CFGS = [
    dict(nxcorr_threshold=None),
    dict(nxcorr_threshold=0.9),
    dict(nxcorr_threshold=0.96, min_variance=2.0),
    dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1),
    dict(nxcorr_threshold=0.5, variant=1, max_lr_diff=1),
    dict(nxcorr_threshold=None, variant=1, max_lr_diff=3, no_dupes=True),
]


@pytest.mark.parametrize("n,H,W,dt,mode", [
    (8, 24, 640, np.uint8, 0), (33, 16, 2048, np.uint8, 0), (40, 8, 1024, np.uint8, 0),
    (17, 12, 700, np.uint16, 0), (10, 12, 300, np.uint8, 1), (16, 6, 257, np.uint16, 1),
    (2, 5, 96, np.uint8, 0), (65, 4, 400, np.uint8, 0),
])
def test_match_bit_exact(gpu, oracle, n, H, W, dt, mode):
    L, R = stereo_stack(n, H, W, dt)
    for cfg in CFGS:
        ref = oracle.match(L, R, cfg_of(oracle, mode=mode, **cfg))
        got = gpu_match(gpu, L, R, mode=mode, **cfg)
        same(got[0], ref[0])
        if ref[1] is not None:
            same(got[1], ref[1])


def test_cfg1_through_pybicos(gpu, oracle):
    """BASELINE configs[0]: 8-image 640x480 stack, nxcorr 0.9, via pybicos.match."""
    import pybicos
    L, R = stereo_stack(8, 480, 640)
    cfg = pybicos.Config()
    cfg.nxcorr_threshold = 0.9
    d, c = pybicos.match(list(L), list(R), cfg)
    rd, rc = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=0.9))
    assert d.dtype == np.float32 and c.dtype == np.float32
    same(d, rd)
    same(c, rc)


def test_pybicos_consistency_and_subpixel(gpu, oracle):
    import pybicos
    L, R = stereo_stack(40, 12, 512, np.uint16)
    cfg = pybicos.Config()
    cfg.nxcorr_threshold = 0.6
    cfg.subpixel_step = 0.25
    cfg.min_variance = 1.0
    cfg.set_consistency(max_lr_diff=2, no_dupes=True)
    d, c = pybicos.match(list(L), list(R), cfg)
    rd, rc = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=0.6, subpixel_step=0.25,
                                                    min_variance=1.0, variant=1, max_lr_diff=2,
                                                    no_dupes=True))
    same(d, rd)
    same(c, rc)


# ------------------------------------------------- full size (BASELINE shapes)
# Whole frames against tests/golden/frames.json (tests/golden/make_frames.py): the C oracle's
# sha256 of the full disparity map and corrmap of every BASELINE config and the reference
# README's full-match shape. Every pixel is compared; a mismatch names its 64-row bands and
# the oracle is re-run on the first bad band for the message.
_FRAMES = None
_STACKS = {}


def _frames():
    global _FRAMES
    if _FRAMES is None:
        import json
        import os
        _FRAMES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "frames.json")))
    return _FRAMES


def _frame_stacks(n, H, W, dtype="u8", maxval=None):
    key = (n, H, W, dtype, maxval)
    if key not in _STACKS:
        _STACKS.clear()  # one frame's stacks at a time (cfg5: 0.55 GB of host memory)
        _STACKS[key] = stereo_stack(n, H, W, np.uint16 if dtype == "u16" else np.uint8,
                                    maxval=maxval)
    return _STACKS[key]


def _check_frame(gpu, oracle, name):
    from tests.golden.make_frames import band_hashes, sha
    rec = _frames()[name]
    n, H, W, cfg = rec["n"], rec["H"], rec["W"], rec["config"]
    L, R = _frame_stacks(n, H, W, rec.get("dtype", "u8"), rec.get("maxval"))
    assert [sha(L), sha(R)] == rec["inputs_sha256"], "synthetic generator changed"
    got_d, got_c = gpu_match(gpu, L, R, **cfg)
    assert str(got_d.dtype) == rec["disparity_dtype"]
    maps = [("disparity", got_d)] + ([("corrmap", got_c)] if rec["corrmap_sha256"] else [])
    for what, m in maps:
        if sha(m) == rec[what + "_sha256"]:
            continue
        bad = [i for i, (a, b) in enumerate(zip(band_hashes(m, rec["band_rows"]),
                                                rec[what + "_bands"])) if a != b]
        b0 = bad[0] * rec["band_rows"]
        e0 = min(H, b0 + rec["band_rows"])
        rd, rc = oracle.match(L[:, b0:e0], R[:, b0:e0], oracle.OracleConfig(**cfg))
        try:
            same(m[b0:e0].copy(), rd if what == "disparity" else rc)
        except AssertionError as ex:
            raise AssertionError("%s %s: %d of %d bands differ; rows %d-%d: %s" % (
                name, what, len(bad), len(rec[what + "_bands"]), b0, e0, ex))
        raise AssertionError("%s %s: %d bands differ, yet rows %d-%d match the oracle" % (
            name, what, len(bad), b0, e0))
    return got_d, got_c


def _planted(got_d, H):
    truth = (16 + (48 * np.arange(H)) // H)[:, None]
    d = got_d.astype(np.float64)
    valid = np.isfinite(d) & (d != -32768)
    return valid, np.abs(d - truth)


def test_full_frame_cfg1(gpu, oracle):
    """BASELINE cfg1 (8 images, 640x480, nxcorr 0.9): the whole frame."""
    _check_frame(gpu, oracle, "cfg1")


def test_full_frame_cfg2(gpu, oracle):
    """2048x1536x33 LIMITED (128-bit), thr 0.96: every pixel vs the oracle + planted truth."""
    got_d, _ = _check_frame(gpu, oracle, "cfg2")
    valid, err = _planted(got_d, 1536)
    assert valid.mean() > 0.95
    assert (err[valid] == 0).mean() > 0.99


def test_full_frame_cfg2_search(gpu, oracle):
    """cfg2 without the NXC stage: the int16 NoDuplicates search result, every pixel."""
    _check_frame(gpu, oracle, "cfg2_raw")


def test_full_frame_cfg3(gpu, oracle):
    got_d, _ = _check_frame(gpu, oracle, "cfg3")
    valid, err = _planted(got_d, 1536)
    assert valid.mean() > 0.9
    assert (err[valid] <= 1.0).all()


def test_full_frame_cfg4(gpu, oracle):
    got_d, _ = _check_frame(gpu, oracle, "cfg4")
    valid, _ = _planted(got_d, 1536)
    assert valid.mean() > 0.9


def test_full_frame_readme(gpu, oracle):
    """The reference README's published full match (README.md:80,90): 3208x2200 x33,
    --limited --threshold 0.96 --variance 2.0 --step 0.1."""
    got_d, _ = _check_frame(gpu, oracle, "readme")
    valid, err = _planted(got_d, 2200)
    assert valid.mean() > 0.9
    assert (err[valid] <= 1.0).all()


# FULL mode at the reference integration bench's shape and settings (bench/cuda.cu:297-323:
# FULL, threshold 0.9, n = 6/8/12/16, subpixel none / 0.25 / 0.1), and 16-bit stacks at the
# cfg2 shape (12-bit camera; full 16-bit range with min-variance + subpixel)
@pytest.mark.parametrize("name", ["full_n6", "full_n8", "full_n12", "full_n16", "full_n8_s25",
                                  "full_n16_s10", "cfg2_u16", "cfg3_u16"])
def test_full_frame_modes(gpu, oracle, name):
    # every pixel is the check (the hashes); the planted disparity is recovered wherever the
    # search keeps a pixel (FULL n = 6 keeps few: 27-bit descriptors tie often)
    got_d, _ = _check_frame(gpu, oracle, name)
    valid, err = _planted(got_d, _frames()[name]["H"])
    assert valid.mean() > 0.1
    assert (err[valid] <= 1.0).mean() > 0.9


# The search's hard paths at size: the int16 result of bicos_search_device on 128-bit
# descriptors at 3300x2200 (the reference kernel-bench shape) -- random, periodic-64 (every
# minimum duplicated) and low-texture (ties decide ~30 % of pixels) -- through NODUPES,
# CONSISTENCY and NODUPES|CONSISTENCY (max_lr_diff 3), every pixel against the oracle's hash;
# round 5: random 32- and 64-bit descriptors (the reference bench's other widths, the
# packed-key search at size)
_SEARCH_NAMES = ["search_%s_%s" % (i, f)
                 for i in ("random", "periodic64", "lowtex", "random_u32", "random_u64")
                 for f in ("nodupes", "cons", "both")]
_SEARCH_IN = {}


@pytest.mark.parametrize("name", _SEARCH_NAMES)
def test_full_frame_search_inputs(gpu, oracle, name):
    import torch
    from tests.golden.make_frames import band_hashes, search_inputs, sha
    rec = _frames()[name]
    H, W, words = rec["H"], rec["W"], rec["words"]
    if rec["input"] not in _SEARCH_IN:
        _SEARCH_IN.clear()  # one input at a time (2 x 116 MB of descriptors)
        d0, d1, bits = search_inputs(rec["input"], oracle)
        assert [sha(d0), sha(d1)] == rec["inputs_sha256"], "descriptor generator changed"
        pitch = gpu._L.bicos_desc_pitch(W, words)
        assert pitch == W * words  # 3300 x 1/2/4 words: rows need no padding
        _SEARCH_IN[rec["input"]] = (
            d0, d1, torch.from_numpy(d0.view(np.int32).reshape(H, pitch)).cuda(),
            torch.from_numpy(d1.view(np.int32).reshape(H, pitch)).cuda(), bits)
    d0, d1, t0, t1, bits = _SEARCH_IN[rec["input"]]
    assert bits == rec["bits"]
    got = host(gpu.search(t0, t1, W, words, rec["flags"], rec["max_lr_diff"], bits=bits))
    if sha(got) == rec["disparity_sha256"]:
        return
    bad = [i for i, (a, b) in enumerate(zip(band_hashes(got, rec["band_rows"]),
                                            rec["disparity_bands"])) if a != b]
    b0 = bad[0] * rec["band_rows"]
    e0 = min(H, b0 + rec["band_rows"])
    ref = oracle.search(d0[b0:e0], d1[b0:e0], rec["flags"], rec["max_lr_diff"])
    same(got[b0:e0].copy(), ref)
    raise AssertionError("%s: %d bands differ, yet rows %d-%d match the oracle" % (
        name, len(bad), b0, e0))


def test_row_band_sharding_is_exact(gpu):
    """Sharded bands (as the multi-GPU path computes them) == the whole-frame match."""
    L, R = stereo_stack(33, 96, 1024)
    cfg = dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1)
    full_d, full_c = gpu_match(gpu, L, R, **cfg)
    from libbicos_amd.distributed import band_rows
    for world in (2, 3, 8):
        parts = [gpu_match(gpu, L[:, b:e], R[:, b:e], **cfg)
                 for b, e in (band_rows(96, world, r) for r in range(world))]
        same(np.concatenate([p[0] for p in parts]), full_d)
        same(np.concatenate([p[1] for p in parts]), full_c)


# ---------------------------------------------------------------- edge cases
def test_empty_and_tiny(gpu, oracle):
    from libbicos_amd.device import MatchConfig
    import torch
    z = torch.zeros((4, 0, 10), dtype=torch.uint8, device="cuda")
    d, c = gpu.match(z, z, MatchConfig())
    assert d.shape == (0, 10)
    z = torch.zeros((4, 3, 0), dtype=torch.uint8, device="cuda")
    d, c = gpu.match(z, z, MatchConfig())
    assert d.shape == (3, 0)
    L, R = stereo_stack(8, 1, 1)
    for cfg in CFGS:
        same(gpu_match(gpu, L, R, **cfg)[0], oracle.match(L, R, cfg_of(oracle, **cfg))[0])


# Consistency on the VALU cross-check search (forward + full reverse search16_kernel): rows
# wider than one LDS stage, reverse duplicates (low-entropy stacks), every register
# blocking / col1 split, and several col0 tiles per row.
@pytest.mark.parametrize("n,H,W,maxval", [(40, 3, 2600, None), (17, 5, 3000, None),
                                          (8, 6, 700, 3), (33, 4, 1100, 2)])
@pytest.mark.parametrize("no_dupes", [False, True])
def test_valu_consistency_edges(gpu, oracle, n, H, W, maxval, no_dupes):
    if maxval is None:
        L, R = stereo_stack(n, H, W, dmin=4, drange=40, seed=n + W)
    else:
        L = random_stack(n, H, W, seed=n, maxval=maxval)
        R = random_stack(n, H, W, seed=n + 1, maxval=maxval)
    kw = dict(nxcorr_threshold=None, variant=1, max_lr_diff=2, no_dupes=no_dupes)
    rd, _ = oracle.match(L, R, cfg_of(oracle, **kw))
    for R_, split in [(0, 0), (2, 0), (4, 2), (2, 4), (4, 8)]:
        gpu.tune(16, R_, 8, split)
        try:
            d, _ = gpu_match(gpu, L, R, **kw)
        finally:
            gpu.tune(0, 0, 0, 0)
        same(d, rd)


@contextlib.contextmanager
def xk_keys(eng):
    """The matrix-core search with XK keys for first-minimum searches too (no FK keys)."""
    eng.tune(67)
    try:
        yield
    finally:
        eng.tune(0)


@pytest.mark.parametrize("n,H,W,dt,kw", [
    (40, 6, 2048, np.uint8, dict(variant=1, max_lr_diff=1)),   # widest FK row (|col1 - B| < 2048)
    (40, 3, 2049, np.uint8, dict(variant=1, max_lr_diff=1)),   # one column more: XK keys
    (20, 4, 515, np.uint8, dict(variant=1, max_lr_diff=2, nxcorr_threshold=0.6)),  # 75 bits
    (8, 5, 700, np.uint16, dict(variant=1, max_lr_diff=0)),    # 32-bit descriptors
    (33, 4, 640, np.uint8, dict(variant=1, max_lr_diff=1)),    # 125 bits: no free half, XK
])
def test_fk_keys_equal_xk_keys(gpu, oracle, n, H, W, dt, kw):
    """KEYS 3 (float keys, the column carried in the free K half with an E8M0 scale of
    2^-12, C = 0) against the XK keys (engine tuned to variant 67) and the oracle."""
    L, R = stereo_stack(n, H, W, dt, dmin=2, drange=40, seed=n * 13 + W)
    with xk_keys(gpu):
        d_x, c_x = gpu_match(gpu, L, R, **kw)
    d_f, c_f = gpu_match(gpu, L, R, **kw)
    same(d_f, d_x)
    if c_x is not None:
        same(c_f, c_x)
    do, _ = oracle.match(L, R, cfg_of(oracle, **kw))
    same(d_f, do)


@pytest.mark.parametrize("words,bits,W", [(8, 150, 2048), (8, 160, 1000), (4, 90, 777), (1, 32, 301)])
def test_fk_search_ties(gpu, words, bits, W):
    """First-minimum search (flags 0) on low-entropy descriptors (few set bits: many equal
    costs, so the lowest-col1 tie rule decides most pixels): FK keys == XK keys == numpy."""
    import torch
    rng = np.random.default_rng(words * 1000 + W)
    rows = 3
    nb = bits
    pitch = gpu._L.bicos_desc_pitch(W, words)

    def desc():
        # AND of three random words: each bit set with p = 1/8 (low entropy, many ties)
        w = rng.integers(0, 2**32, size=(3, rows, W, words), dtype=np.uint64)
        v = (w[0] & w[1] & w[2]).astype(np.uint32)
        for q in range(words):
            lo = 32 * q
            v[:, :, q] &= np.uint32(0 if lo >= nb else (0xFFFFFFFF if nb - lo >= 32 else (1 << (nb - lo)) - 1))
        d = np.zeros((rows, pitch), np.uint32)
        d[:, :W * words] = v.reshape(rows, W * words)
        return d
    d0, d1 = desc(), desc()
    t0 = torch.from_numpy(d0.view(np.int32)).cuda()
    t1 = torch.from_numpy(d1.view(np.int32)).cuda()
    with xk_keys(gpu):
        ox = host(gpu.search(t0, t1, W, words, flags=0, bits=bits))
    of = host(gpu.search(t0, t1, W, words, flags=0, bits=bits))
    same(of, ox)
    # numpy: popcount Hamming, lowest col1 among the minima, disparity = col0 - col1
    pc = np.array([bin(i).count("1") for i in range(256)], np.uint8)
    for r in range(rows):
        a = d0[r, :W * words].reshape(W, words).view(np.uint8).reshape(W, 1, words * 4)
        b = d1[r, :W * words].reshape(W, words).view(np.uint8).reshape(1, W, words * 4)
        ham = pc[a ^ b].sum(axis=2, dtype=np.int32)
        exp = np.arange(W) - ham.argmin(axis=1)
        assert np.array_equal(of[r].astype(np.int64), exp), r


def test_errors(gpu):
    import torch
    from libbicos_amd import BicosError
    from libbicos_amd.device import MatchConfig
    s = torch.zeros((1, 4, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(BicosError, match="at least two"):
        gpu.match(s, s)
    s = torch.zeros((66, 4, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(BicosError, match="too large"):
        gpu.match(s, s)
    s = torch.zeros((17, 4, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(BicosError, match="too large"):
        gpu.match(s, s, MatchConfig(mode=1))
    s = torch.zeros((8, 4, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(BicosError, match="subpixel_step"):
        gpu.match(s, s, MatchConfig(subpixel_step=0.0))
    # x + step == x somewhere in [-1, 1]: the reference loops forever; rejected here
    with pytest.raises(BicosError, match="too small"):
        gpu.match(s, s, MatchConfig(nxcorr_threshold=0.5, subpixel_step=1e-9))
    raw = torch.zeros((4, 4), dtype=torch.int16, device="cuda")
    with pytest.raises(BicosError, match="too small"):
        gpu.agree(raw, s, s, 0.5, step=1e-5)


def test_pybicos_errors(gpu):
    import pybicos
    a = [np.zeros((8, 8), np.uint8)] * 8
    b = [np.zeros((8, 9), np.uint8)] * 8
    with pytest.raises(RuntimeError):
        pybicos.match(a, b)
    with pytest.raises(RuntimeError):
        pybicos.match(a[:1], a[:1])
    with pytest.raises(ValueError):
        pybicos.match([np.zeros((8, 8), np.int32)] * 8, a)


def test_double_precision(gpu, oracle):
    """Precision::DOUBLE (CUDA-build feature, agree.cuh:35-65): no CPU oracle; compare
    the float64 correlation with a float64 numpy restatement (no fma there: 1e-12)."""
    L, R = stereo_stack(33, 8, 512)
    d32, c32 = gpu_match(gpu, L, R, nxcorr_threshold=0.5)
    d64, c64 = gpu_match(gpu, L, R, nxcorr_threshold=0.5, precision=1)
    assert c64.dtype == np.float64
    raw, _ = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=None))
    rr, cc = np.nonzero(raw != -32768)
    col1 = cc - raw[rr, cc].astype(np.int64)
    ok = (col1 >= 0) & (col1 < 512)
    rr, cc, col1 = rr[ok], cc[ok], col1[ok]
    a = L[:, rr, cc].astype(np.float64)
    b = R[:, rr, col1].astype(np.float64)
    a -= a.mean(0)
    b -= b.mean(0)
    ref = (a * b).sum(0) / np.sqrt((a * a).sum(0) * (b * b).sum(0))
    got = c64[rr, cc]
    fin = np.isfinite(ref)
    assert np.abs(got[fin] - ref[fin]).max() < 1e-12
    assert np.abs(c32[rr, cc][fin] - ref[fin]).max() < FLOAT_TOL


def _subpixel_f64(L, R, raw, thr, step, minvar):
    """float64 restatement of the DOUBLE subpixel refine (reference agree.cuh:161-259 with
    TPrecision = double): the quadratic interpolation stays float32 exactly as in the float
    path (oracle/ref_numpy.py agree_subpixel), the correlation and its argmax are float64
    (numpy, no fma: compare within 1e-12), min-variance on the float64 variances."""
    from oracle import ref_numpy as N
    n, H, W = L.shape
    f32 = np.float32
    out = np.full((H, W), np.nan, np.float32)
    corr = np.full((H, W), np.nan, np.float64)

    def nxc64(a, b):
        a = a.astype(np.float64)
        b = b.astype(np.float64)
        a = a - a.sum(0) / n
        b = b - b.sum(0) / n
        v0, v1 = (a * a).sum(0), (b * b).sum(0)
        with np.errstate(divide="ignore", invalid="ignore"):
            r = (a * b).sum(0) / np.sqrt(v0 * v1)
        if minvar is not None:
            r = np.where((v0 < minvar) | (v1 < minvar), -1.0, r)
        return r
    d = raw.astype(np.int64)
    rr, cc = np.nonzero(raw != -32768)
    col1 = cc - d[rr, cc]
    keep = (col1 >= 0) & (col1 < W)
    rr, cc, col1 = rr[keep], cc[keep], col1[keep]
    edge = (col1 == 0) | (col1 == W - 1)
    er, ec, e1 = rr[edge], cc[edge], col1[edge]
    if er.size:
        v = nxc64(L[:, er, ec], R[:, er, e1])
        corr[er, ec] = v
        ok = ~(v < thr)
        out[er[ok], ec[ok]] = d[er[ok], ec[ok]].astype(np.float32)
    ir, ic, i1 = rr[~edge], cc[~edge], col1[~edge]
    y0 = R[:, ir, i1 - 1].astype(np.float32)
    y1 = R[:, ir, i1].astype(np.float32)
    y2 = R[:, ir, i1 + 1].astype(np.float32)
    A = (f32(0.5) * ((y0 - f32(2.0) * y1).astype(np.float32) + y2)).astype(np.float32)
    B = (f32(0.5) * (-R[:, ir, i1 - 1].astype(np.int64) + R[:, ir, i1 + 1].astype(np.int64)
                     ).astype(np.float32)).astype(np.float32)
    best_x = np.zeros(ir.size, np.float32)
    best = np.full(ir.size, -1.0)
    for x in N.x_steps(step):
        ax = (A * x).astype(np.float32)
        v = (((ax * x).astype(np.float32) + (B * x).astype(np.float32)).astype(np.float32)
             + y1).astype(np.float32)
        c = nxc64(L[:, ir, ic], N._narrow(v, L.dtype))
        win = best < c
        best_x = np.where(win, x, best_x)
        best = np.where(win, c, best)
    corr[ir, ic] = best
    ok = ~(best < thr)
    out[ir[ok], ic[ok]] = (d[ir[ok], ic[ok]].astype(np.float32) - best_x[ok]).astype(np.float32)
    return out, corr


# Precision::DOUBLE subpixel at the exact-kernel depths n = 6 / 10 / 12 (the reference's
# integration and kernel-bench depths; ADVICE r04: only the float path was pinned there)
@pytest.mark.parametrize("n", [6, 10, 12])
@pytest.mark.parametrize("step,minvar", [(0.25, None), (0.1, 2.0)])
def test_double_subpixel_exact_depths(gpu, oracle, n, step, minvar):
    L, R = stereo_stack(n, 6, 300, dmin=3, drange=30, seed=n + 17)
    raw, _ = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=None, mode=1))
    mv = None if minvar is None else float(np.float32(minvar) * np.float32(n))
    out, corr = gpu.agree(dev(raw), dev(L), dev(R), 0.5, mv, step=step, precision=1)
    ref_d, ref_c = _subpixel_f64(L, R, raw, 0.5, step, mv)
    got_c = host(corr)
    assert got_c.dtype == np.float64
    fin = np.isfinite(ref_c)
    assert (np.isfinite(got_c) == fin).all()
    assert np.abs(got_c[fin] - ref_c[fin]).max() < 1e-12
    same(host(out), ref_d)


def test_deterministic(gpu):
    L, R = stereo_stack(33, 32, 1024)
    a = gpu_match(gpu, L, R, nxcorr_threshold=0.9, subpixel_step=0.1)
    b = gpu_match(gpu, L, R, nxcorr_threshold=0.9, subpixel_step=0.1)
    same(a[0], b[0])
    same(a[1], b[1])


@pytest.mark.parametrize("words", [1, 2, 4, 8])
def test_search_tuning_settings_are_exact(gpu, oracle, words):
    """Every (variant, col0/lane, waves, col1-split) produces the oracle's result."""
    H, W = 6, 1100
    rng = np.random.default_rng(words)
    a = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    b = a[:, np.roll(np.arange(W), 7)] ^ (rng.random((H, W, words)) < 0.03).astype(np.uint32)
    if words == 8:   # descriptors from the transform never use bit 255 (4n-6 <= 254)
        a[..., 7] &= 0x7FFFFFFF
        b[..., 7] &= 0x7FFFFFFF
    lo = _low_entropy_desc(H, W, words, 3)
    settings = [(16, 2, 8, 1), (16, 2, 8, 2),
                (16, 2, 8, 4), (16, 4, 4, 2), (16, 4, 8, 4), (16, 2, 1, 1), (16, 2, 2, 2),
                (64, 2, 8, 0), (64, 4, 8, 0), (64, 8, 8, 0), (64, 2, 1, 0), (64, 8, 4, 0),
                (65, 8, 8, 0), (65, 2, 4, 0), (66, 8, 8, 0), (66, 4, 2, 0)]
    try:
        for flags, lr in ((1, -1), (3, 1), (2, 2)):
            for (x, y) in ((a, b), (lo, lo[:, ::-1].copy())):
                ref = oracle.search(x, y, flags, lr)
                for s in settings:
                    gpu.tune(*s)
                    out = host(gpu.search(dev(_pack(x)), dev(_pack(y)), W, words, flags, lr))
                    same(out, ref)
    finally:
        gpu.tune(0, 0, 0, 0)


# Matrix-core search (search_mx.hip): extreme Hamming keys (x = +-255: all-zero left vs
# all-one right descriptors), rows that are not a multiple of the 32-column block, rows
# wider than one LDS chunk, every tile count -- against the oracle and the VALU search.
@pytest.mark.parametrize("words", [1, 2, 4, 8])
@pytest.mark.parametrize("W", [1, 31, 33, 95, 2049, 4111, 8161, 16385])
def test_mx_search_edges(gpu, oracle, words, W):
    H = 3
    rng = np.random.default_rng(W * 10 + words)
    a = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    b = a[:, np.roll(np.arange(W), 5)] ^ (rng.random((H, W, words)) < 0.05).astype(np.uint32)
    full = np.uint32(0xFFFFFFFF)
    a[0, : W // 2] = 0          # left all zero, right all one: the extreme keys
    b[0, W // 3:] = full
    b[1] = full                 # every col1 ties: the minimum is duplicated everywhere
    if words == 8:
        a[..., 7] &= 0x7FFFFFFF
        b[..., 7] &= 0x7FFFFFFF
    try:
        for flags, lr in ((1, -1), (0, -1), (3, 1), (2, 0)):
            ref = oracle.search(a, b, flags, lr)
            for s in [(64, 2, 8, 0), (65, 8, 8, 0), (66, 8, 8, 0), (66, 4, 2, 0), (16, 0, 0, 0)]:
                gpu.tune(*s)
                out = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, flags, lr))
                same(out, ref)
    finally:
        gpu.tune(0, 0, 0, 0)


# Tail workgroups (search_mx.hip launch_mx_tt / launch_pk, round 4): a row remainder of at most
# half a workgroup and 8 waves x 2 tiles goes to one extra workgroup per row with 1 or 2 tiles
# per wave. Widths on either side of every selection boundary for 4-tile (per workgroup 1024
# col0) and 8-tile (2048) main workgroups -- remainder 1, 255/256 (1 tile), 257, 512 (2 tiles),
# 513 (no tail) -- the README width, through NoDuplicates and NoDuplicates|Consistency (both
# passes take the tail), one-product keys (128/256-bit) and packed keys (32/64-bit, with the
# used-bits hint), against the oracle.
@pytest.mark.parametrize("words", [1, 2, 4, 8])
@pytest.mark.parametrize("W", [1025, 1279, 1280, 1281, 1536, 1537, 2049, 2560, 2561, 3208])
def test_search_tail_workgroups(gpu, oracle, words, W):
    H = 3
    rng = np.random.default_rng(W * 7 + words)
    a = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    b = a[:, np.roll(np.arange(W), 9)] ^ (rng.random((H, W, words)) < 0.03).astype(np.uint32)
    b[1, :, :] = b[1, :1, :]    # every col1 ties
    a[2] &= 0x0F0F0F0F          # low-entropy row: duplicates and ties everywhere
    b[2] &= 0x0F0F0F0F
    if words == 8:
        a[..., 7] &= 0x7FFFFFFF
        b[..., 7] &= 0x7FFFFFFF
    bits = 32 * words if words <= 2 else 0
    try:
        for flags, lr in ((1, -1), (3, 1)):
            ref = oracle.search(a, b, flags, lr)
            for s in [(0, 0, 0, 0), (64, 4, 8, 0), (64, 8, 8, 0)]:
                gpu.tune(*s)
                out = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, flags, lr,
                                      bits=bits))
                same(out, ref)
    finally:
        gpu.tune(0, 0, 0, 0)


# Packed Hamming keys (search_mx.hip search_pk_kernel, the default NoDuplicates search when
# the used-bits hint is <= 127): two distances per accumulator register, no column in the
# key, first column and in-block duplicates resolved where the running minimum drops.
# Extreme distances (0 and `bits`), rows where every col1 ties, tie-heavy sparse rows,
# planted matches, ragged widths, one and several LDS chunks, every wide-tile count --
# against the oracle and the one-product search (variant 65).
@pytest.mark.parametrize("words,bits", [(1, 27), (1, 32), (2, 61), (2, 64), (4, 99), (4, 126),
                                        (4, 127)])
@pytest.mark.parametrize("W", [1, 31, 33, 95, 700, 2049, 4111, 9000])
def test_pk_search(gpu, oracle, words, bits, W):
    H = 5
    rng = np.random.default_rng(W * 100 + bits)
    mask = np.zeros(words, dtype=np.uint64)
    for w in range(words):
        lo = 32 * w
        mask[w] = 0 if lo >= bits else (2 ** min(32, bits - lo)) - 1
    a = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64)
    b = a[:, np.roll(np.arange(W), 11)] ^ (rng.random((H, W, words)) < 0.05)
    a[0, : W // 2] = 0          # distances 0 .. bits: the extreme keys
    b[0] = np.uint64(0xFFFFFFFF)
    b[0, : W // 3] = 0
    b[1] = np.uint64(0xFFFFFFFF)  # every col1 ties
    sp = rng.integers(0, 2 ** 32, size=(2, W, words), dtype=np.uint64)
    for _ in range(3):          # sparse bits: small distances, many ties
        sp &= rng.integers(0, 2 ** 32, size=(2, W, words), dtype=np.uint64)
    a[2], b[2] = sp[0], sp[1]
    b[3] = a[3, np.maximum(np.arange(W) - 40, 0)]  # planted disparities with repeats
    a = (a & mask).astype(np.uint32)
    b = (b & mask).astype(np.uint32)
    try:
        for flags, lr in ((1, -1), (3, 1)):
            ref = oracle.search(a, b, flags, lr)
            for s in [(0, 0, 0, 0), (64, 2, 8, 0), (64, 4, 8, 0), (68, 8, 8, 0), (68, 4, 4, 32),
                      (68, 2, 8, 16), (65, 4, 8, 0)]:
                gpu.tune(*s)
                out = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, flags, lr, bits=bits))
                same(out, ref)
    finally:
        gpu.tune(0, 0, 0, 0)


@pytest.mark.parametrize("k", [2, 4, 6])
@pytest.mark.parametrize("W", [777, 2048, 4100])
def test_mx_tie_only_blocks(gpu, oracle, k, W):
    """NoDuplicates on sparse random descriptors (each bit set with p = 2^-k: small integer
    costs, so most blocks TIE the running minimum cost without lowering it, the case the
    paired search records with the block's own key instead of the last-minimum tree), for
    the 2-tile pipelined kernel (few rows) and the 4-tile one (tuned), one and several LDS
    chunks; against the oracle."""
    H, words = 3, 4
    rng = np.random.default_rng(W * 10 + k)

    def sparse():
        v = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64)
        for _ in range(k - 1):
            v &= rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64)
        return v.astype(np.uint32)
    a, b = sparse(), sparse()
    b[1] = a[1, np.roll(np.arange(W), 9)]  # one row with planted unique matches
    ref = oracle.search(a, b, 1, -1)
    try:
        for s in [(0, 0, 0, 0), (64, 4, 8, 0), (64, 2, 8, 0)]:
            gpu.tune(*s)
            same(host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, 1, -1)), ref)
    finally:
        gpu.tune(0, 0, 0, 0)


@pytest.mark.parametrize("B", [129, 154, 192])
def test_mx_search_used_bits(gpu, oracle, B):
    """256-bit descriptors whose bits >= B are zero (transform output of n = 33..49
    LIMITED): with the used-bits hint the search multiplies 3 K-steps instead of 4 and
    still matches the oracle, for every flag combination and tile count."""
    H, W, words = 3, 700, 8
    rng = np.random.default_rng(B)
    a = rng.integers(0, 2 ** 32, size=(H, W, words), dtype=np.uint64).astype(np.uint32)
    b = a[:, np.roll(np.arange(W), 7)] ^ (rng.random((H, W, words)) < 0.05).astype(np.uint32)
    b[1] = b[1, :1]             # every col1 ties on row 1
    for arr in (a, b):
        for w in range(words):
            lo = 32 * w
            if lo >= B:
                arr[..., w] = 0
            elif lo + 32 > B:
                arr[..., w] &= np.uint32((1 << (B - lo)) - 1)
    try:
        for flags, lr in ((1, -1), (0, -1), (3, 1), (2, 0)):
            ref = oracle.search(a, b, flags, lr)
            for s in [(0, 0, 0, 0), (64, 2, 8, 0), (64, 4, 8, 0), (65, 4, 8, 0), (66, 2, 4, 0)]:
                gpu.tune(*s)
                out = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, words, flags, lr, bits=B))
                same(out, ref)
    finally:
        gpu.tune(0, 0, 0, 0)


def test_mx_is_the_default_search(gpu):
    """The engine runs the matrix-core search unless tuned to a VALU variant."""
    from libbicos_amd import _lib
    assert "mx" in _lib.lib().bicos_build_info().decode()


# ---------------------------------------------- cfg5: 4K frame, 8 row bands of 270
def test_cfg5_full_size_and_bands(gpu, oracle):
    """3840x2160x33 (BASELINE cfg5) on one GPU: the whole frame against the oracle's hashes
    (tests/golden/frames.json), and the 8 row bands of 270 the 8-GPU run computes are
    byte-identical to it -- band r matched on GPU r % device_count (distinct GPUs where the box
    has them), then all 8 gathered onto GPU 0 by bicos_match_bands_device (peer copies)."""
    import torch
    from libbicos_amd.device import Engine, MatchConfig, match_bands
    from libbicos_amd.distributed import band_rows
    n, H, W = 33, 2160, 3840
    cfg = MatchConfig(nxcorr_threshold=0.96)
    got_d, got_c = _check_frame(gpu, oracle, "cfg5")
    L, R = _frame_stacks(n, H, W)
    s0, s1 = dev(L), dev(R)
    nd = torch.cuda.device_count()
    engines = {0: gpu}
    bands0, bands1 = [], []
    for r in range(8):
        b, e = band_rows(H, 8, r)
        assert e - b == 270
        d = r % nd
        b0, b1 = s0[:, b:e], s1[:, b:e]
        if d:
            b0, b1 = b0.to("cuda:%d" % d), b1.to("cuda:%d" % d)
            engines.setdefault(d, Engine(d))
        bands0.append(b0)
        bands1.append(b1)
        bd, bc = engines[d].match(b0, b1, cfg)
        same(host(bd), got_d[b:e])
        same(host(bc), got_c[b:e])
    gd, gc = match_bands(bands0, bands1, cfg)
    same(host(gd), got_d)
    same(host(gc), got_c)
    truth = (16 + (48 * np.arange(H)) // H)[:, None]
    d = got_d.astype(np.float64)
    valid = np.isfinite(d) & (d != -32768)
    assert valid.mean() > 0.95
    assert (np.abs(d - truth)[valid] == 0).mean() > 0.99


# ------------------------------------------------ the shared default engine, two threads
def test_default_engine_two_threads(gpu, oracle):
    """pybicos.match (host path) and device.match (device path) on the process-wide engine
    from two threads at once: the engine lock + workspace event keep both exact."""
    import threading
    import torch
    from libbicos_amd import device, pybicos
    cfg = dict(nxcorr_threshold=0.9)
    L1, R1 = stereo_stack(8, 96, 640, seed=11)
    L2, R2 = stereo_stack(33, 64, 1300, seed=12)   # bigger: forces workspace growth
    ref1 = oracle.match(L1, R1, oracle.OracleConfig(**cfg))
    ref2 = oracle.match(L2, R2, oracle.OracleConfig(**cfg))
    errors = []

    def host_path():
        try:
            pc = pybicos.Config()
            pc.nxcorr_threshold = 0.9
            for _ in range(6):
                d, c = pybicos.match(list(L1), list(R1), pc)
                same(d, ref1[0])
                same(c, ref1[1])
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(ex)

    def device_path():
        try:
            s0, s1 = dev(L2), dev(R2)
            st = torch.cuda.Stream()
            for _ in range(6):
                with torch.cuda.stream(st):
                    d, c = device.match(s0, s1, device.MatchConfig(**cfg))
                st.synchronize()
                same(host(d), ref2[0])
                same(host(c), ref2[1])
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    ts = [threading.Thread(target=host_path), threading.Thread(target=device_path)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errors, errors


def test_one_engine_alternating_streams(gpu, oracle):
    """One engine, frames enqueued back to back with no host sync on streams 0,1,1,0,2,...:
    the workspace wait is skipped when the previous use was on the same stream and kept
    across streams (and across a workspace growth in the middle) -- every map exact."""
    import torch
    from libbicos_amd import device
    cfg = dict(nxcorr_threshold=0.9)
    frames = [stereo_stack(8, 48, 640, seed=21), stereo_stack(33, 40, 1300, seed=22),
              stereo_stack(12, 56, 900, seed=23)]
    refs = [oracle.match(L, R, oracle.OracleConfig(**cfg)) for L, R in frames]
    devs = [(dev(L), dev(R)) for L, R in frames]
    eng = device.Engine()
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    order = [0, 1, 1, 0, 2, 2, 1, 0, 0, 2, 1, 2]
    outs = []
    torch.cuda.synchronize()
    for k, si in enumerate(order):
        f = k % len(frames)
        with torch.cuda.stream(streams[si]):
            outs.append((f, eng.match(devs[f][0], devs[f][1], device.MatchConfig(**cfg))))
    torch.cuda.synchronize()
    for f, (d, c) in outs:
        same(host(d), refs[f][0])
        same(host(c), refs[f][1])


def test_device_outputs_are_validated(gpu):
    import torch
    from libbicos_amd.device import MatchConfig
    L, R = stereo_stack(8, 16, 64)
    s0, s1 = dev(L), dev(R)
    bad_corr = torch.empty((16, 64), dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError):  # DOUBLE writes float64
        gpu.match(s0, s1, MatchConfig(precision=1), corrmap=bad_corr)
    with pytest.raises(ValueError):  # no nxcorr: int16 disparity
        gpu.match(s0, s1, MatchConfig(nxcorr_threshold=None),
                  out=torch.empty((16, 64), dtype=torch.float32, device="cuda"))
    with pytest.raises(ValueError):
        gpu.match(s0, s1, MatchConfig(), out=torch.empty((16, 63), dtype=torch.float32,
                                                         device="cuda"))


# ------------------------------------- padded row pitch with an odd image width
@pytest.mark.parametrize("W,P,dt", [(190, 192, np.uint8), (190, 256, np.uint8), (301, 320, np.uint8),
                                    (515, 576, np.uint8), (190, 192, np.uint16), (77, 80, np.uint16)])
def test_padded_pitch_odd_width(gpu, oracle, W, P, dt):
    """Stacks whose rows are padded to an aligned pitch while cols % 4 != 0 (what a
    pitched allocation or the C++ staging path produces): the last pixels of the frame share
    a dword with bytes past the stack; every stage must still read them (the aligned agree
    kernel once read the last row's last pixels of plane n-1 as 0)."""
    import torch
    from libbicos_amd.device import MatchConfig
    n, H = 10, 21
    L, R = stereo_stack(n, H, W, dt)
    tdt = torch.uint8 if dt == np.uint8 else torch.int16
    buf = torch.zeros((2 * n, H, P), dtype=tdt, device="cuda")
    buf[:n, :, :W] = dev(L)
    buf[n:, :, :W] = dev(R)
    for cfg in (dict(nxcorr_threshold=0.5), dict(nxcorr_threshold=0.5, mode=1),
                dict(nxcorr_threshold=0.5, min_variance=1.0, subpixel_step=0.2),
                dict(nxcorr_threshold=0.5, variant=1, max_lr_diff=2, no_dupes=True),
                dict(nxcorr_threshold=None)):
        rd, rc = oracle.match(L, R, oracle.OracleConfig(**cfg))
        d, c = gpu.match(buf[:n, :, :W], buf[n:, :, :W], MatchConfig(**cfg))
        same(host(d), rd)
        if rc is not None:
            same(host(c), rc)


# ------------------------------- int16 disparity with the NXC stage (bicos_match_device_i16)
# (float) of the int16 map is the float32 map byte for byte, the corrmap is unchanged, for
# every variant without subpixel; a subpixel config is rejected. The second half writes into
# views of one packed uint8 band buffer, exactly as bench.py's gather path does.
@pytest.mark.parametrize("n,H,W,dt,kw", [
    (33, 9, 2048, np.uint8, dict(nxcorr_threshold=0.96)),
    (17, 5, 1300, np.uint16, dict(nxcorr_threshold=0.8, min_variance=1.5)),
    (40, 4, 900, np.uint8, dict(nxcorr_threshold=0.9, variant=1, max_lr_diff=1)),
    (8, 7, 640, np.uint8, dict(nxcorr_threshold=0.9, precision=1)),
])
def test_int16_disparity_entry(gpu, n, H, W, dt, kw):
    import torch
    from libbicos_amd.device import MatchConfig
    L, R = stereo_stack(n, H, W, dt, dmin=3, drange=30, seed=n + H)
    L[:, 1, 100:140] = 7  # flat patch: NaN correlations pass the threshold
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    fo, fc = gpu.match(s0, s1, cfg)
    io = torch.empty((H, W), dtype=torch.int16, device="cuda")
    io, ic = gpu.match(s0, s1, cfg, out=io)
    assert io.dtype == torch.int16
    same(host(io).astype(np.float32), host(fo))
    same(host(ic), host(fc))
    if kw.get("precision"):
        return
    # packed [int16 disparity | pad | float32 corrmap] band buffer of hb >= H rows
    hb = H + 1
    dbytes = hb * W * 2
    off = (dbytes + 3) // 4 * 4
    buf = torch.full((off + hb * W * 4,), 0xAB, dtype=torch.uint8, device="cuda")
    dv = buf[:dbytes].view(torch.int16).view(hb, W)
    cv = buf[off:].view(torch.float32).view(hb, W)
    gpu.match(s0, s1, cfg, out=dv[:H], corrmap=cv[:H])
    same(host(dv[:H]), host(io))
    same(host(cv[:H]), host(ic))
    assert (host(buf[H * W * 2:off]) == 0xAB).all()  # nothing written past the band
    assert (host(buf[off + H * W * 4:]) == 0xAB).all()


@pytest.mark.parametrize("step", [None, 0.25])
def test_agree_stage_double_equals_match(gpu, step):
    """bicos_agree_stage_device with precision 1 (the reference kernel-bench's double NXC /
    subpixel, tools/ref_kernel_bench.py) == the DOUBLE match on the same search result."""
    from libbicos_amd.device import MatchConfig, descriptor_words
    n, H, W = 10, 12, 640
    L, R = stereo_stack(n, H, W, dmin=3, drange=30, seed=77)
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(nxcorr_threshold=0.5, min_variance=1.0, subpixel_step=step, precision=1)
    md, mc = gpu.match(s0, s1, cfg)
    words = descriptor_words(n, 0)
    raw = gpu.search(gpu.transform(s0, 0, words), gpu.transform(s1, 0, words), W, words, 1)
    ad, ac = gpu.agree(raw, s0, s1, 0.5, float(np.float32(1.0) * np.float32(n)), step=step,
                       precision=1)
    assert ac.dtype == mc.dtype
    same(host(ad), host(md))
    same(host(ac), host(mc))


def test_int16_disparity_rejects_subpixel(gpu):
    import torch
    from libbicos_amd.device import MatchConfig
    L, R = stereo_stack(8, 16, 64)
    with pytest.raises(ValueError):
        gpu.match(dev(L), dev(R), MatchConfig(subpixel_step=0.1),
                  out=torch.empty((16, 64), dtype=torch.int16, device="cuda"))


# ------------------- agree fused into the search launch (search_mx.hip fused_agree, round 5)
# The headline shape (128-bit NoDuplicates search with 4 tiles per wave and no tail launch,
# u8 stacks of n = 33, float, no subpixel) runs the agree inside the search's workgroups.
# Frames tall enough for that geometry (300 rows x 1800 / 2048 columns: >= 2 workgroups per
# CU, no tail; the last workgroup of an 1800-column row holds 776 col0) against the separate
# search + agree stages (the stage API launches them apart), with and without min-variance,
# float32 and int16 disparity maps; the whole-frame cfg2 / cfg5 tests pin it to the oracle.
# 60 / 40 rows: small grids take 2 tiles per wave (the N = 8 band shape), also fused.
@pytest.mark.parametrize("H,W", [(300, 1800), (300, 2048), (60, 2048), (40, 1800)])
@pytest.mark.parametrize("kw", [dict(nxcorr_threshold=0.96),
                                dict(nxcorr_threshold=0.5, min_variance=2.0)])
def test_fused_search_agree_equals_stages(gpu, H, W, kw):
    import torch
    from libbicos_amd.device import MatchConfig, descriptor_words
    n = 33
    L, R = stereo_stack(n, H, W, np.uint8, dmin=3, drange=40, seed=W + H + len(kw))
    L[:, 5, 200:260] = 9  # flat patch: NaN / low-variance correlations
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    #  the match of this shape really runs the fused launch
    assert gpu.plan(s0, s1, cfg) & _lib.PLAN_AGREE_IN_SEARCH
    md, mc = gpu.match(s0, s1, cfg)
    words = descriptor_words(n, 0)
    raw = gpu.search(gpu.transform(s0, 0, words), gpu.transform(s1, 0, words), W, words, 1)
    mv = float(np.float32(kw["min_variance"]) * np.float32(n)) if "min_variance" in kw else None
    ad, ac = gpu.agree(raw, s0, s1, kw["nxcorr_threshold"], mv)
    same(host(md), host(ad))
    same(host(mc), host(ac))
    io = torch.empty((H, W), dtype=torch.int16, device="cuda")
    io, ic = gpu.match(s0, s1, cfg, out=io)
    same(host(io).astype(np.float32), host(md))
    same(host(ic), host(mc))


# The packed-key search's fused agree (search_pk_kernel AG: 32-bit words, one wide tile per
# wave, no tail, u8 n = 8 -- cfg1's shape), against the separate stages as above; 700 columns
# leave the row's second workgroup 188 col0.
@pytest.mark.parametrize("H,W", [(480, 640), (100, 700)])
def test_fused_pk_search_agree_equals_stages(gpu, H, W):
    import torch
    from libbicos_amd.device import MatchConfig, descriptor_words
    n = 8
    L, R = stereo_stack(n, H, W, np.uint8, dmin=3, drange=40, seed=H + W)
    L[:, 3, 100:150] = 11  # flat patch
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(nxcorr_threshold=0.9)
    plan = gpu.plan(s0, s1, cfg)
    assert plan & _lib.PLAN_AGREE_IN_SEARCH and plan & _lib.PLAN_PACKED_KEYS
    md, mc = gpu.match(s0, s1, cfg)
    words = descriptor_words(n, 0)
    d0, d1 = gpu.transform(s0, 0, words), gpu.transform(s1, 0, words)
    raw = gpu.search(d0, d1, W, words, 1, bits=4 * n - 5)
    ad, ac = gpu.agree(raw, s0, s1, 0.9)
    same(host(md), host(ad))
    same(host(mc), host(ac))
    io = torch.empty((H, W), dtype=torch.int16, device="cuda")
    io, ic = gpu.match(s0, s1, cfg, out=io)
    same(host(io).astype(np.float32), host(md))
    same(host(ic), host(mc))


# ------------------------ the row bands an N-GPU run matches, against the oracle
# bench.py --gpus N splits cfg2's 1536 rows into N bands of 1536 / N; each rank matches its
# band alone, so the band's grid is what the N-GPU run executes (192 rows at N = 8: the
# 2-tile fused search + agree). Each band, matched as its own frame, must
# equal the oracle's whole-frame fixture on those rows: frames.json holds the C oracle's
# sha256 of every 64-row band of cfg2 (tests/golden/make_frames.py), disparity and corrmap.
# Reference semantics: agree.hpp:53-93, bicos.hpp:78-113 (row-local, so a band is exact).
@pytest.mark.parametrize("N", [8, 4, 2])
def test_cfg2_row_bands_match_oracle_fixture(gpu, N):
    from libbicos_amd.device import MatchConfig
    from libbicos_amd.distributed import band_rows
    from tests.golden.make_frames import band_hashes, sha
    rec = _frames()["cfg2"]
    n, H, W, B = rec["n"], rec["H"], rec["W"], rec["band_rows"]
    L, R = _frame_stacks(n, H, W)
    assert [sha(L), sha(R)] == rec["inputs_sha256"], "synthetic generator changed"
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**rec["config"])
    for r in range(N):
        b, e = band_rows(H, N, r)
        assert (e - b) % B == 0 and b % B == 0
        t0, t1 = s0[:, b:e], s1[:, b:e]
        # the band shape takes the fused search + agree launch (2 tiles per wave at N = 8)
        assert gpu.plan(t0, t1, cfg) & _lib.PLAN_AGREE_IN_SEARCH, (N, r)
        d, c = gpu.match(t0, t1, cfg)
        hd, hc = host(d), host(c)
        assert band_hashes(hd, B) == rec["disparity_bands"][b // B:e // B], ("disparity", N, r)
        assert band_hashes(hc, B) == rec["corrmap_bands"][b // B:e // B], ("corrmap", N, r)


# ---------------------------- the match past its transform (bicos_search_agree_device)
# bench.py times the launches the match issues after its transform through this entry; it
# must produce the match's maps for every plan: fused search + agree (cfg1 / cfg2 shapes),
# search + subpixel (cfg3), Consistency with its check inside the agree (cfg4), no NXC.
@pytest.mark.parametrize("n,H,W,dt,kw", [
    (8, 64, 640, np.uint8, dict(nxcorr_threshold=0.9)),
    (33, 300, 2048, np.uint8, dict(nxcorr_threshold=0.96)),
    (33, 40, 1024, np.uint8, dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1)),
    (40, 24, 1100, np.uint8, dict(nxcorr_threshold=0.96, variant=1, max_lr_diff=1)),
    (17, 9, 700, np.uint16, dict(nxcorr_threshold=0.8, variant=1, max_lr_diff=0, no_dupes=True)),
    (12, 16, 500, np.uint8, dict(nxcorr_threshold=None)),
])
def test_search_agree_entry_equals_match(gpu, n, H, W, dt, kw):
    from libbicos_amd.device import MatchConfig, descriptor_words
    L, R = stereo_stack(n, H, W, dt, dmin=3, drange=40, seed=n + W)
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    md, mc = gpu.match(s0, s1, cfg)
    words = descriptor_words(n, 0)
    d0, d1 = gpu.transform(s0, 0, words), gpu.transform(s1, 0, words)
    sd, sc = gpu.search_agree(d0, d1, s0, s1, cfg)
    same(host(sd), host(md))
    if mc is not None:
        same(host(sc), host(mc))


# -------------------- Consistency's left-right check inside the agree (agree_lds_kernel CONS)
# With NXC and aligned stacks the check of consistency_kernel (bicos.hpp:99-106) runs in the
# agree launch (bicos_match_plan PLAN_CONSISTENCY_IN_AGREE): every max_lr_diff, with and
# without NoDuplicates, u8 / u16, min-variance, against the oracle; a subpixel config
# keeps the separate check kernel.
@pytest.mark.parametrize("n,H,W,dt,kw", [
    (40, 6, 2048, np.uint8, dict(nxcorr_threshold=0.96, variant=1, max_lr_diff=1)),
    (40, 5, 1300, np.uint8, dict(nxcorr_threshold=0.5, variant=1, max_lr_diff=0, no_dupes=True)),
    (9, 7, 332, np.uint8, dict(nxcorr_threshold=0.7, variant=1, max_lr_diff=5, min_variance=1.0)),
    (17, 6, 900, np.uint16, dict(nxcorr_threshold=0.8, variant=1, max_lr_diff=2)),
    (33, 4, 1032, np.uint8, dict(nxcorr_threshold=0.9, variant=1, max_lr_diff=3)),
    (65, 3, 260, np.uint8, dict(nxcorr_threshold=0.2, variant=1, max_lr_diff=1)),
])
def test_consistency_in_agree(gpu, oracle, monkeypatch, n, H, W, dt, kw):
    from libbicos_amd.device import MatchConfig
    monkeypatch.setenv("BICOS_LR_ONE_PASS", "0")  # (n = 40 first minimum: the one-pass form)
    L, R = stereo_stack(n, H, W, dt, dmin=2, drange=50, seed=n * 7 + W)
    L[:, 1, 40:90] = 5  # flat patch: NaN correlations pass
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    assert gpu.plan(s0, s1, cfg) & _lib.PLAN_CONSISTENCY_IN_AGREE
    d, c = gpu.match(s0, s1, cfg)
    rd, rc = oracle.match(L, R, oracle.OracleConfig(**kw))
    same(host(d), rd)
    same(host(c), rc)
    # both precisions against the two-launch form: the check alone (no NXC: the int16 map of
    # consistency_kernel), then the agree stage on it
    raw, _ = gpu.match(s0, s1, MatchConfig(**dict(kw, nxcorr_threshold=None)))
    mv = kw.get("min_variance")
    mv = None if mv is None else float(np.float32(mv) * np.float32(n))
    for prec in (0, 1):
        pd, pc = gpu.match(s0, s1, MatchConfig(**dict(kw, precision=prec)))
        ad, ac = gpu.agree(raw, s0, s1, kw["nxcorr_threshold"], mv, precision=prec)
        same(host(pd), host(ad))
        same(host(pc), host(ac))
    sub = MatchConfig(**dict(kw, subpixel_step=0.25))
    assert not gpu.plan(s0, s1, sub) & _lib.PLAN_CONSISTENCY_IN_AGREE


# ------------------------ Consistency's dense-row fast path (search_mx.hip dense_row)
# Rows whose forward search kept >= 7/8 of their col0 run the reverse search over every col0
# instead of the compacted entries; sparse rows keep the prologue. A frame mixing both (planted
# stereo rows, rows with an unrelated right image, rows between) against the oracle, every
# width class of the search (packed keys, one-product keys 128 / 256-bit, FK keys).
@pytest.mark.parametrize("n,W,kw", [
    (40, 700, dict(variant=1, max_lr_diff=1)),
    (40, 2048, dict(variant=1, max_lr_diff=2, no_dupes=True)),
    (33, 1100, dict(variant=1, max_lr_diff=1)),
    (8, 900, dict(variant=1, max_lr_diff=0, no_dupes=True)),
    (17, 640, dict(variant=1, max_lr_diff=3)),
])
@pytest.mark.parametrize("nxc", [None, 0.8])
def test_consistency_dense_rows(gpu, oracle, monkeypatch, n, W, kw, nxc):
    from libbicos_amd.device import MatchConfig
    monkeypatch.setenv("BICOS_LR_ONE_PASS", "0")  # (n = 40 first minimum: the one-pass form)
    H = 12
    L, R = stereo_stack(n, H, W, dmin=2, drange=40, seed=n + W)
    Rr = random_stack(n, H, W, seed=n * W)
    R[:, 4:8] = Rr[:, 4:8]            # rows 4-7: nothing to match -> sparse rows
    R[:, 8:10, W // 2:] = Rr[:, 8:10, W // 2:]  # rows 8-9: half of each row matches
    cfg = dict(kw, nxcorr_threshold=nxc)
    s0, s1 = dev(L), dev(R)
    plan = gpu.plan(s0, s1, MatchConfig(**cfg))
    assert plan & _lib.PLAN_DENSE_ROWS and plan & _lib.PLAN_REVERSE_COMPACTED
    d, c = gpu.match(s0, s1, MatchConfig(**cfg))
    rd, rc = oracle.match(L, R, oracle.OracleConfig(**cfg))
    same(host(d), rd)
    if rc is not None:
        same(host(c), rc)


# ------------------------------- Consistency in one pass (search_mx.hip search_lr_kernel)
# First-minimum Consistency over 256-bit descriptors with 129..154 used bits and <= 2048
# columns: both searches from one set of matrix products and the left-right check in the same
# workgroup. Descriptor level (bicos_search_device with the used-bits hint) on random,
# shifted-copy and low-entropy descriptors (ties everywhere, both directions' first minimum),
# all-zero / all-one columns (|a| = 0 / bits), every width class of the pass split, against
# the oracle and against the two-launch form (BICOS_LR_ONE_PASS=0).
def _lr_desc(H, W, bits, seed, kind):
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 2 ** 32, size=(H, W, 8), dtype=np.uint64).astype(np.uint32)
    if kind == "low":
        d[...] = 0
        d[..., 0] = rng.integers(0, 16, size=(H, W), dtype=np.uint32)
        d[..., 4] = np.where(rng.random((H, W)) < 0.5, np.uint32(0x3FFFFFF), np.uint32(0))
    d = _lr_mask(d, bits)
    if kind != "low" and W > 4:  # |a| = 0 and |a| = bits
        d[0, 1] = 0
        d[0, 3] = _lr_mask(np.full(8, 0xFFFFFFFF, np.uint32), bits)
    return d


@pytest.mark.parametrize("W", [1, 31, 65, 333, 700, 1030, 2048])
@pytest.mark.parametrize("bits", [129, 154])
def test_search_lr_one_pass(gpu, oracle, monkeypatch, W, bits):
    H = 3
    rng = np.random.default_rng(W + bits)
    for kind in ("random", "shifted", "low"):
        a = _lr_desc(H, W, bits, W * 3 + bits, kind)
        if kind == "shifted":  # a stereo-like match 5 columns away, 3 % of the words off by one bit
            flip = (rng.random((H, W, 8)) < 0.03).astype(np.uint32) << rng.integers(0, 32, (H, W, 8)).astype(np.uint32)
            b = _lr_mask(a[:, np.roll(np.arange(W), 5)] ^ flip, bits)
        else:
            b = _lr_desc(H, W, bits, W * 5 + bits + 1, kind)
        for lr in (0, 1, 4):
            ref = oracle.search(a, b, 2, lr)
            monkeypatch.delenv("BICOS_LR_ONE_PASS", raising=False)
            out = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, 8, 2, lr, bits=bits))
            same(out, ref)
            monkeypatch.setenv("BICOS_LR_ONE_PASS", "0")
            two = host(gpu.search(dev(_pack(a)), dev(_pack(b)), W, 8, 2, lr, bits=bits))
            same(two, ref)


def _lr_mask(d, bits):
    full = np.zeros(8, np.uint32)
    for b in range(bits):
        full[b // 32] |= np.uint32(1 << (b % 32))
    return d & full


# the match: LIMITED n = 34..40 and FULL n = 13 (146 bits), u8 / u16, with and without NXC,
# min-variance, a subpixel step (the one-pass map feeds the subpixel refine), flat patches
@pytest.mark.parametrize("n,H,W,dt,kw", [
    (40, 6, 2048, np.uint8, dict(nxcorr_threshold=0.96, variant=1, max_lr_diff=1)),
    (40, 5, 1300, np.uint8, dict(nxcorr_threshold=None, variant=1, max_lr_diff=0)),
    (40, 7, 1000, np.uint8, dict(nxcorr_threshold=0.5, variant=1, max_lr_diff=2, min_variance=1.0)),
    (40, 3, 77, np.uint8, dict(nxcorr_threshold=0.0, variant=1, max_lr_diff=0)),
    (34, 4, 700, np.uint16, dict(nxcorr_threshold=0.8, variant=1, max_lr_diff=3, min_variance=1.0)),
    (37, 4, 333, np.uint8, dict(nxcorr_threshold=0.9, variant=1, max_lr_diff=2, subpixel_step=0.25)),
    (13, 4, 517, np.uint8, dict(nxcorr_threshold=0.5, variant=1, max_lr_diff=1, mode=1)),
])
def test_consistency_one_pass(gpu, oracle, monkeypatch, n, H, W, dt, kw):
    from libbicos_amd.device import MatchConfig
    L, R = stereo_stack(n, H, W, dt, dmin=2, drange=50, seed=n * 11 + W)
    L[:, 1, 40:90] = 5  # flat patch: every distance ties
    R[:, 1, 30:95] = 5
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    monkeypatch.delenv("BICOS_LR_ONE_PASS", raising=False)
    plan = gpu.plan(s0, s1, cfg)
    assert plan & _lib.PLAN_CONSISTENCY_ONE_PASS and not plan & _lib.PLAN_AGREE_IN_SEARCH
    d, c = gpu.match(s0, s1, cfg)
    rd, rc = oracle.match(L, R, oracle.OracleConfig(**kw))
    same(host(d), rd)
    if rc is not None:
        same(host(c), rc)
    assert not gpu.plan(s0, s1, MatchConfig(**dict(kw, no_dupes=True))) & _lib.PLAN_CONSISTENCY_ONE_PASS
    monkeypatch.setenv("BICOS_LR_ONE_PASS", "0")
    assert not gpu.plan(s0, s1, cfg) & _lib.PLAN_CONSISTENCY_ONE_PASS
    d2, c2 = gpu.match(s0, s1, cfg)
    same(host(d2), host(d))
    if c is not None:
        same(host(c2), host(c))


# ------------------ the 128-bit packed-key search with its fused agree (variant 68 / BICOS_PK128=1)
# Not the default (it ties or loses in the frames), still a supported tuning:
# engines tuned to variant 68 run search_pk_kernel<4, ...> with lazy drops and, for cfg2's
# shapes, the agree inside the same launch. Byte-identical to the default engine's maps; the
# 192-row band (one wide tile per wave) and a 300-row frame (two) against cfg2's oracle hashes.
@pytest.mark.parametrize("rows", [192, 300])
def test_pk128_fused_equals_default(gpu, rows):
    from libbicos_amd.device import Engine, MatchConfig
    from tests.golden.make_frames import band_hashes
    rec = _frames()["cfg2"]
    n, W = rec["n"], rec["W"]
    L, R = _frame_stacks(n, rec["H"], W)
    s0, s1 = dev(L[:, :rows]), dev(R[:, :rows])
    cfg = MatchConfig(**rec["config"])
    e68 = Engine(0)
    e68.tune(68)
    plan = e68.plan(s0, s1, cfg)
    assert plan & _lib.PLAN_PACKED_KEYS and plan & _lib.PLAN_AGREE_IN_SEARCH
    d, c = e68.match(s0, s1, cfg)
    dd, dc = gpu.match(s0, s1, cfg)
    same(host(d), host(dd))
    same(host(c), host(dc))
    if rows == 192:
        assert band_hashes(host(d), 64) == rec["disparity_bands"][:3]
        assert band_hashes(host(c), 64) == rec["corrmap_bands"][:3]


# ------------- the one-launch Consistency search, randomised (tests/lr_stress.py: 300 cases)
def test_lr_stress(gpu):
    from tests.lr_stress import run
    n, bad = run(300, 6, None)
    assert bad is None, bad
    assert n == 300
