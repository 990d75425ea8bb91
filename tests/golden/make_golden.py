"""Generate tests/golden/golden.npz -- regression vectors for the BICOS hot path.

The reference ships no golden vectors and cannot be built here, so these
are produced by the C oracle (oracle/bicos_oracle.c, cross-checked against the numpy
restatement at generation time). Inputs are regenerated from the seeded synthetic
generator; their sha256 is stored so a generator change is caught.

  python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from libbicos_amd.synthetic import random_stack, stereo_stack  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import ref_numpy as N  # noqa: E402

CASES = [
    # name, n, H, W, dtype, mode, generator
    ("n8_u8_limited", 8, 24, 96, np.uint8, 0, "stereo"),
    ("n33_u8_limited", 33, 12, 257, np.uint8, 0, "stereo"),
    ("n40_u8_limited", 40, 8, 130, np.uint8, 0, "stereo"),
    ("n17_u16_limited", 17, 10, 120, np.uint16, 0, "stereo"),
    ("n10_u8_full", 10, 10, 100, np.uint8, 1, "stereo"),
    ("n12_u8_random", 12, 6, 64, np.uint8, 0, "random"),
]
CONFIGS = [
    ("plain", dict(nxcorr_threshold=None)),
    ("nxc", dict(nxcorr_threshold=0.9)),
    ("minvar", dict(nxcorr_threshold=0.8, min_variance=2.0)),
    ("subpix", dict(nxcorr_threshold=0.5, subpixel_step=0.1)),
    ("cons", dict(nxcorr_threshold=0.5, variant=1, max_lr_diff=1)),
    ("cons_nd", dict(nxcorr_threshold=None, variant=1, max_lr_diff=3, no_dupes=True)),
]


def inputs(n, H, W, dt, gen):
    if gen == "stereo":
        return stereo_stack(n, H, W, dt, dmin=2, drange=12)
    return (random_stack(n, H, W, dt, seed=21, maxval=40),
            random_stack(n, H, W, dt, seed=22, maxval=40))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    O.build()
    out = {}
    for name, n, H, W, dt, mode, gen in CASES:
        L, R = inputs(n, H, W, dt, gen)
        out[name + "/inputs_sha256"] = np.array(sha(L) + sha(R))
        for cname, cfg in CONFIGS:
            c = dict(cfg, mode=mode)
            d, corr = O.match(L, R, O.OracleConfig(**c))
            d2, corr2 = N.match(L, R, **c)
            assert np.array_equal(d.view(np.uint8), d2.view(np.uint8)), (name, cname)
            out["%s/%s/disparity" % (name, cname)] = d
            if corr is not None:
                out["%s/%s/corrmap" % (name, cname)] = corr
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    main()
