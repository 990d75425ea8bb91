"""Per-rank compute of the row-band split on one GPU: one match of a cfg2 band of
H/N rows (N = 1, 2, 4, 8), steady state (after a clock spin-up), no collective.
This is the compute floor of `bench.py --gpus N` (strong scaling) before the gather.

  python tools/band_bench.py [--config cfg2] [--ns 1,2,4,8] [--reps 50]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from libbicos_amd import device  # noqa: E402
from libbicos_amd.distributed import band_rows  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    mcfg = device.MatchConfig(**C["cfg"])
    eng = device.Engine(0)
    for N in [int(v) for v in args.ns.split(",")]:
        b, e = band_rows(H, N, 0)
        rows = e - b
        L, R = stereo_stack(n, H, W, np.uint8, row_begin=b, row_end=e)
        s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
        has_corr = mcfg.nxcorr_threshold is not None
        out = torch.empty((rows, W), dtype=torch.float32 if has_corr else torch.int16, device="cuda")
        corr = torch.empty((rows, W), dtype=torch.float32, device="cuda") if has_corr else None
        t_end = time.perf_counter() + 0.15
        while time.perf_counter() < t_end:
            for _ in range(4):
                eng.match(s0, s1, mcfg, out=out, corrmap=corr)
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.match(s0, s1, mcfg, out=out, corrmap=corr)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.reps * 1e3
        print(json.dumps({"config": args.config, "N": N, "band_rows": rows, "ms_per_match": round(ms, 4),
                          "frame_Mpix_s_if_perfect": round(H * W / (ms * 1e-3) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
