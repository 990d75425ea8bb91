"""Generate tests/golden/frames.json -- whole-frame parity fixtures at the BASELINE sizes.

SURVEY.md s8(c) asks for hashes of full outputs at the benchmark shapes. For every
BASELINE config (cfg1-cfg5) and the reference README's published full-match shape
(README.md:80,90: 3208x2200 x33, --limited --threshold 0.96 --variance 2.0 --step 0.1)
this runs the C oracle (oracle/bicos_oracle.c, a restatement of reference
src/impl/cpu.cpp:100-159, bicos.hpp:50-113, agree.hpp:53-191) over the WHOLE synthetic
frame and stores

  * the sha256 of both input stacks (catches a change of the synthetic generator),
  * the sha256 of the full disparity map and corrmap, exactly as the API returns them
    (int16 without NXC, float32 otherwise; C order, raw bytes incl. NaN payloads),
  * the sha256 of every band of BAND rows of both maps, so a mismatch names its rows,
  * the valid fraction of the disparity map (a sanity figure, not a check).

The GPU tests (tests/test_gpu_parity.py::test_full_frame_*) hash the GPU's whole frame
against these: 100 % of the pixels are compared, not a row sample.

  python tests/golden/make_frames.py [name ...]     (about 10 minutes on 8 cores)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from libbicos_amd.synthetic import (SEED, low_texture_stack, random_descriptors,  # noqa: E402
                                    stereo_stack)
from oracle import oracle as O  # noqa: E402
from oracle import ref_numpy as N  # noqa: E402

BAND = 64
PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frames.json")

# name -> (n, H, W, match config[, stack generator options]); the BASELINE shapes and configs
# of bench.py CONFIGS, the README shape, and (round 4) FULL mode and u16 stacks at size
FRAMES = {
    "cfg1": (8, 480, 640, dict(nxcorr_threshold=0.9)),
    "cfg2": (33, 1536, 2048, dict(nxcorr_threshold=0.96)),
    "cfg3": (33, 1536, 2048, dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1)),
    "cfg4": (40, 1536, 2048, dict(nxcorr_threshold=0.96, variant=1, max_lr_diff=1)),
    "cfg5": (33, 2160, 3840, dict(nxcorr_threshold=0.96)),
    "readme": (33, 2200, 3208, dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1)),
    # cfg2 without the NXC stage: the int16 search result itself, every pixel
    "cfg2_raw": (33, 1536, 2048, dict(nxcorr_threshold=None)),
    # the reference's integration bench: FULL mode, threshold 0.9, n = 6/8/12/16, subpixel
    # step none / 0.25 / 0.2 / 0.15 / 0.1 (bench/cuda.cu:297-323,397-401) at the dataset's
    # 3208x2200. FULL n = 16 is 227 bits -> 256-bit descriptors with NoDuplicates, a search
    # shape no BASELINE config has (cfg4 is 256-bit Consistency).
    "full_n6": (6, 2200, 3208, dict(nxcorr_threshold=0.9, mode=1)),
    "full_n8": (8, 2200, 3208, dict(nxcorr_threshold=0.9, mode=1)),
    "full_n12": (12, 2200, 3208, dict(nxcorr_threshold=0.9, mode=1)),
    "full_n16": (16, 2200, 3208, dict(nxcorr_threshold=0.9, mode=1)),
    "full_n8_s25": (8, 2200, 3208, dict(nxcorr_threshold=0.9, mode=1, subpixel_step=0.25)),
    "full_n16_s10": (16, 2200, 3208, dict(nxcorr_threshold=0.9, mode=1, subpixel_step=0.1)),
    # 16-bit stacks (CV_16UC1, reference src/impl/cpu.cpp:113): a 12-bit camera at the cfg2
    # shape, and the full 16-bit range with min-variance + subpixel, where the interpolated
    # samples leave [0, 65535] and the narrowing wraps through int32 (agree.hpp:163-166)
    "cfg2_u16": (33, 1536, 2048, dict(nxcorr_threshold=0.96), dict(dtype="u16", maxval=4095)),
    "cfg3_u16": (33, 1536, 2048, dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1),
                 dict(dtype="u16", maxval=65535)),
}

# Raw-search frames (round 4): the int16 result of the stage entry bicos_search_device on
# host-generated 128-bit descriptors at the reference kernel-bench shape 3300x2200
# (bench/cuda.cu:44,182-256), for its three flag sets: NODUPES, CONSISTENCY and
# NODUPES|CONSISTENCY with max_lr_diff 3 (bicos.hpp:50-113). Inputs:
#   random      independent splitmix64 words left / right (the reference bench's input)
#   periodic64  the same random row repeated every 64 columns on both sides: every minimum
#               is attained W/64 times (NoDuplicates rejects all; first-minimum ties decide
#               the rest)
#   lowtex      LIMITED n = 33 descriptors of a weakly textured scene (synthetic
#               low_texture_stack: 8 grey levels in 4-column runs + independent noise, right
#               view moved 5 columns) -- duplicate and tied minima decide ~30 % of pixels
# Round 5: random_u32 / random_u64, the reference bench's 32- and 64-bit descriptor points
# (bench/cuda.cu:353-366; the packed-key search at size), every descriptor bit random.
SEARCH_SHAPE = (2200, 3300)
SEARCH_FLAGS = {"nodupes": (1, -1), "cons": (2, 3), "both": (3, 3)}
SEARCH_INPUTS = {"random": 4, "periodic64": 4, "lowtex": 4, "random_u32": 1, "random_u64": 2}
SEARCH_FRAMES = {"search_%s_%s" % (i, f): (i, f) for i in SEARCH_INPUTS for f in SEARCH_FLAGS}


def search_inputs(kind, O=None, row_begin=0, row_end=None):
    """(left, right) descriptor words [rows, W, words] uint32 of rows [row_begin, row_end) of
    an input, and its used-bits hint."""
    H, W = SEARCH_SHAPE
    words = SEARCH_INPUTS[kind]
    rows = dict(row_begin=row_begin, row_end=row_end)
    if kind in ("random", "random_u32", "random_u64"):
        return (random_descriptors(H, W, words, SEED, **rows),
                random_descriptors(H, W, words, SEED ^ 0xA5A5A5A5, **rows), 0)
    if kind == "periodic64":
        d = random_descriptors(H, W, words, SEED, period=64, **rows)
        return d, d.copy(), 0
    if kind == "lowtex":
        O = O or _oracle()
        n = 33
        left = O.transform(low_texture_stack(n, H, W, **rows), 0, words)
        right = O.transform(low_texture_stack(n, H, W, shift=5, noise_seed=2, **rows), 0, words)
        return left, right, 4 * n - 5
    raise KeyError(kind)


def _oracle():
    from oracle import oracle as O
    return O


def frame_stacks(spec, row_begin=0, row_end=None):
    """The synthetic stacks of a FRAMES entry (u8, or u16 with the entry's maxval)."""
    n, H, W = spec[:3]
    gen = spec[4] if len(spec) > 4 else {}
    dt = np.uint16 if gen.get("dtype") == "u16" else np.uint8
    return stereo_stack(n, H, W, dt, maxval=gen.get("maxval"), row_begin=row_begin,
                        row_end=row_end)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def band_hashes(a, band=BAND):
    return [sha(a[b:b + band]) for b in range(0, a.shape[0], band)]


def frame_record(n, H, W, cfg, L, R, d, c, maxval=None):
    dd = d.astype(np.float64)
    valid = np.isfinite(dd) & (dd != -32768)
    rec = {
        "n": n, "H": H, "W": W, "dtype": "u16" if L.dtype == np.uint16 else "u8",
        "config": cfg, "band_rows": BAND,
        "inputs_sha256": [sha(L), sha(R)],
        "disparity_dtype": str(d.dtype),
        "disparity_sha256": sha(d),
        "disparity_bands": band_hashes(d),
        "corrmap_sha256": None if c is None else sha(c),
        "corrmap_bands": None if c is None else band_hashes(c),
        "valid_fraction": round(float(valid.mean()), 6),
    }
    if maxval is not None:
        rec["maxval"] = maxval
    return rec


def search_record(name, O):
    kind, fl = SEARCH_FRAMES[name]
    flags, lr = SEARCH_FLAGS[fl]
    H, W = SEARCH_SHAPE
    words = SEARCH_INPUTS[kind]
    d0, d1, bits = search_inputs(kind, O)
    d = O.search(d0, d1, flags, lr, variant="v3")
    # the numpy restatement agrees on two rows (tests/test_oracle.py cross-checks the rest)
    for y in (0, H // 2 + 1):
        nd = N.search(d0[y:y + 1], d1[y:y + 1], flags, lr)
        assert np.array_equal(nd, d[y:y + 1]), (name, y)
    return {
        "kind": "search", "input": kind, "H": H, "W": W, "words": words, "bits": bits,
        "flags": flags, "max_lr_diff": lr, "band_rows": BAND,
        "inputs_sha256": [sha(d0), sha(d1)],
        "disparity_dtype": "int16", "disparity_sha256": sha(d), "disparity_bands": band_hashes(d),
        "valid_fraction": round(float((d != -32768).mean()), 6),
    }


def main(names):
    O.build()
    db = json.load(open(PATH)) if os.path.exists(PATH) else {}
    for name in names:
        t = time.time()
        if name in SEARCH_FRAMES:
            db[name] = search_record(name, O)
            print("%-24s valid %.4f  %.1f s" % (name, db[name]["valid_fraction"], time.time() - t),
                  flush=True)
            json.dump(db, open(PATH, "w"), indent=1, sort_keys=True)
            continue
        spec = FRAMES[name]
        n, H, W, cfg = spec[:4]
        L, R = frame_stacks(spec)
        d, c = O.match(L, R, O.OracleConfig(**cfg), variant="v3")
        # the independent numpy restatement agrees on two rows of the frame (it is too slow
        # for the whole of it; rows are independent, SURVEY.md s8 e)
        for y in (0, H // 2 + 1):
            nd, nc = N.match(L[:, y:y + 1], R[:, y:y + 1], **cfg)
            assert np.array_equal(nd.view(np.uint8), d[y:y + 1].view(np.uint8)), (name, y)
            if c is not None:
                assert np.array_equal(nc.view(np.uint8), c[y:y + 1].view(np.uint8)), (name, y)
        db[name] = frame_record(n, H, W, cfg, L, R, d, c,
                                (spec[4] if len(spec) > 4 else {}).get("maxval"))
        print("%-8s %dx%dx%d  valid %.4f  %.1f s" % (name, W, H, n, db[name]["valid_fraction"],
                                                     time.time() - t), flush=True)
        json.dump(db, open(PATH, "w"), indent=1, sort_keys=True)
    print("wrote", PATH)


if __name__ == "__main__":
    main(sys.argv[1:] or list(FRAMES) + list(SEARCH_FRAMES))
