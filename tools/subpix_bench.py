"""Time the agree stages (NXC, NXC + subpixel) alone across stack depths n.

  python tools/subpix_bench.py [--ns 8,16,24,25,33,40,48,65] [--rows 768]

Prints one JSON line per (n, stage): ms per launch and ps per (pixel x image x x-step),
the unit the subpixel kernel's VALU work scales with, so occupancy effects between the
MAXN buckets show directly.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from libbicos_amd import device  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="8,16,24,25,33,40,48,65")
    ap.add_argument("--rows", type=int, default=768)
    ap.add_argument("--cols", type=int, default=2048)
    ap.add_argument("--step", type=float, default=0.1)
    ap.add_argument("--steps", default=None, help="comma list of subpixel steps (overrides --step)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--depth", type=int, default=1)
    args = ap.parse_args()
    eng = device.Engine(0)
    dt = np.uint8 if args.depth == 1 else np.uint16
    for n in [int(v) for v in args.ns.split(",")]:
        L, R = stereo_stack(n, args.rows, args.cols, dt)
        conv = (lambda a: torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a).cuda())
        s0, s1 = conv(L), conv(R)
        cfg = device.MatchConfig(nxcorr_threshold=None)
        raw, _ = eng.match(s0, s1, cfg)
        raw = raw.to(torch.int16) if raw.dtype != torch.int16 else raw
        valid = float((raw != -32768).float().mean().item())
        st = torch.cuda.current_stream()
        stages = [("nxcorr", None)] + [("subpixel", float(v)) for v in
                                       (args.steps.split(",") if args.steps else [args.step])]
        for stage, step in stages:
            steps = 0
            if step:
                x = np.float32(-1.0)
                while x <= 1.0:
                    steps += 1
                    x = np.float32(x + np.float32(step))
            eng.agree(raw, s0, s1, 0.9, minvar_scaled=2.0 * n, step=step)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(args.reps):
                eng.agree(raw, s0, s1, 0.9, minvar_scaled=2.0 * n, step=step)
            b.record(st)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.reps
            units = args.rows * args.cols * valid * n * (steps if step else 1)
            print(json.dumps({"n": n, "stage": stage, "xsteps": steps, "ms": round(ms, 4),
                              "valid": round(valid, 3),
                              "ps_per_unit": round(ms * 1e9 / units, 3)}), flush=True)


if __name__ == "__main__":
    main()
