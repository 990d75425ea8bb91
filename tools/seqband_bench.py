"""A whole frame matched as k sequential row bands on one GPU (k = 1, 2, 3, 4), one stream and
two frames in flight, interleaved rounds: does keeping a band's stacks + descriptors inside the
256 MB last-level cache (cfg2: 207 MB of stacks + 101 MB of descriptors per frame) make the
agree read its stacks from there instead of HBM? Every band writes its rows of the frame's maps
(views), so the result is the whole-frame match (checked against k = 1 byte for byte).

  python tools/seqband_bench.py [--config cfg2] [--ks 1,2,3,4] [--reps 20] [--rounds 3]
"""
import argparse
import json
import os
import statistics
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
    ap.add_argument("--ks", default="1,2,3,4")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    mcfg = device.MatchConfig(**C["cfg"])
    L, R = stereo_stack(n, H, W, np.uint8)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    del L, R
    F = 2
    engines = [device.Engine(0) for _ in range(F)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
    outs = [torch.empty((H, W), dtype=torch.float32, device="cuda") for _ in range(F)]
    corrs = [torch.empty((H, W), dtype=torch.float32, device="cuda") for _ in range(F)]
    ks = [int(v) for v in args.ks.split(",")]

    def frame(k, f):
        with torch.cuda.stream(streams[f]):
            for b in range(k):
                r0, r1 = band_rows(H, k, b)
                engines[f].match(s0[:, r0:r1], s1[:, r0:r1], mcfg, out=outs[f][r0:r1],
                                 corrmap=corrs[f][r0:r1])

    ref = None
    for k in ks:
        frame(k, 0)
        torch.cuda.synchronize()
        got = (outs[0].cpu().numpy().tobytes(), corrs[0].cpu().numpy().tobytes())
        if ref is None:
            ref = got
        elif got != ref:
            raise SystemExit("k=%d: maps differ from the whole-frame match" % k)
    t_end = time.perf_counter() + 0.2
    while time.perf_counter() < t_end:
        frame(1, 0)
        torch.cuda.synchronize()
    res = {(k, F_): [] for k in ks for F_ in (1, 2)}
    for _ in range(args.rounds):
        for k in ks:
            for nf in (1, 2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.reps):
                    frame(k, i % nf)
                torch.cuda.synchronize()
                res[(k, nf)].append((time.perf_counter() - t0) / args.reps * 1e3)
    for (k, nf), v in res.items():
        print(json.dumps({"config": args.config, "bands": k, "frames_in_flight": nf,
                          "ms_per_frame_median": round(statistics.median(v), 4),
                          "ms_min": round(min(v), 4)}), flush=True)


if __name__ == "__main__":
    main()
