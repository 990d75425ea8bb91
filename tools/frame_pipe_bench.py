"""Consecutive frames on S streams (one engine per stream): frame k runs on stream k % S, so
the HBM-bound transform / agree of one frame can use the compute-unit slots the search of
the previous frame leaves idle (its last round of workgroups on narrow row bands). Prints
ms per frame for S = 1 and S = 2 at each band height, interleaved in one process.

  python tools/frame_pipe_bench.py [--config cfg2] [--ns 1,8] [--reps 50] [--rounds 3]
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
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--streams", default="1,2", help="stream counts S to compare")
    ap.add_argument("--tunes", default="0:0:0:0",
                    help="search geometries to compare, each variant:T:waves:LDS-KiB "
                         "(bicos_engine_tune; 0:0:0:0 = the default)")
    args = ap.parse_args()
    Ss = [int(v) for v in args.streams.split(",")]
    SM = max(Ss + [2])
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    mcfg = device.MatchConfig(**C["cfg"])
    engines = [device.Engine(0) for _ in range(SM)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(SM - 1)]
    tunes = [tuple(int(x) for x in t.split(":")) for t in args.tunes.split(",")]
    for N, tune in [(N, t) for N in [int(v) for v in args.ns.split(",")] for t in tunes]:
        for e_ in engines:
            e_.tune(*tune)
        b, e = band_rows(H, N, 0)
        rows = e - b
        L, R = stereo_stack(n, H, W, np.uint8, row_begin=b, row_end=e)
        s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
        outs = [(torch.empty((rows, W), dtype=torch.float32, device="cuda"),
                 torch.empty((rows, W), dtype=torch.float32, device="cuda")) for _ in range(SM)]

        def run(S, reps):
            for k in range(reps):
                i = k % S
                engines[i].match(s0, s1, mcfg, out=outs[i][0], corrmap=outs[i][1], stream=streams[i])
            torch.cuda.synchronize()

        run(2, 8)
        ref = [t.clone() for t in outs[0]]
        run(1, 1)
        assert all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(ref, outs[0]))
        t_end = time.perf_counter() + 0.15
        while time.perf_counter() < t_end:
            run(1, 4)
        res = {S: [] for S in Ss}
        for _ in range(args.rounds):
            for S in Ss:
                t0 = time.perf_counter()
                run(S, args.reps)
                res[S].append((time.perf_counter() - t0) / args.reps * 1e3)
        for S in Ss:
            print(json.dumps({"config": args.config, "N": N, "band_rows": rows, "streams": S,
                              "tune": ":".join(map(str, tune)),
                              "ms_per_frame": round(statistics.median(res[S]), 4),
                              "ms_min": round(min(res[S]), 4)}), flush=True)


if __name__ == "__main__":
    main()
