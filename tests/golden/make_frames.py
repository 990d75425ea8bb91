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

  python tests/golden/make_frames.py [name ...]     (about 3 minutes on 8 cores)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from libbicos_amd.synthetic import stereo_stack  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import ref_numpy as N  # noqa: E402

BAND = 64
PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frames.json")

# name -> (n, H, W, match config); the same shapes and configs as bench.py CONFIGS
FRAMES = {
    "cfg1": (8, 480, 640, dict(nxcorr_threshold=0.9)),
    "cfg2": (33, 1536, 2048, dict(nxcorr_threshold=0.96)),
    "cfg3": (33, 1536, 2048, dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1)),
    "cfg4": (40, 1536, 2048, dict(nxcorr_threshold=0.96, variant=1, max_lr_diff=1)),
    "cfg5": (33, 2160, 3840, dict(nxcorr_threshold=0.96)),
    "readme": (33, 2200, 3208, dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1)),
    # cfg2 without the NXC stage: the int16 search result itself, every pixel
    "cfg2_raw": (33, 1536, 2048, dict(nxcorr_threshold=None)),
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def band_hashes(a, band=BAND):
    return [sha(a[b:b + band]) for b in range(0, a.shape[0], band)]


def frame_record(n, H, W, cfg, L, R, d, c):
    dd = d.astype(np.float64)
    valid = np.isfinite(dd) & (dd != -32768)
    return {
        "n": n, "H": H, "W": W, "dtype": "u8", "config": cfg, "band_rows": BAND,
        "inputs_sha256": [sha(L), sha(R)],
        "disparity_dtype": str(d.dtype),
        "disparity_sha256": sha(d),
        "disparity_bands": band_hashes(d),
        "corrmap_sha256": None if c is None else sha(c),
        "corrmap_bands": None if c is None else band_hashes(c),
        "valid_fraction": round(float(valid.mean()), 6),
    }


def main(names):
    O.build()
    db = json.load(open(PATH)) if os.path.exists(PATH) else {}
    for name in names:
        n, H, W, cfg = FRAMES[name]
        t = time.time()
        L, R = stereo_stack(n, H, W, np.uint8)
        d, c = O.match(L, R, O.OracleConfig(**cfg), variant="v3")
        # the independent numpy restatement agrees on two rows of the frame (it is too slow
        # for the whole of it; rows are independent, SURVEY.md s8 e)
        for y in (0, H // 2 + 1):
            nd, nc = N.match(L[:, y:y + 1], R[:, y:y + 1], **cfg)
            assert np.array_equal(nd.view(np.uint8), d[y:y + 1].view(np.uint8)), (name, y)
            if c is not None:
                assert np.array_equal(nc.view(np.uint8), c[y:y + 1].view(np.uint8)), (name, y)
        db[name] = frame_record(n, H, W, cfg, L, R, d, c)
        print("%-8s %dx%dx%d  valid %.4f  %.1f s" % (name, W, H, n, db[name]["valid_fraction"],
                                                     time.time() - t), flush=True)
        json.dump(db, open(PATH, "w"), indent=1, sort_keys=True)
    print("wrote", PATH)


if __name__ == "__main__":
    main(sys.argv[1:] or list(FRAMES))
