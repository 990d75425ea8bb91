"""Fused transform -> search (BICOS_FUSE_TRANSFORM=1) vs the transform kernel + search,
timed in ONE process with the two forms interleaved.

  python tools/fused_tf_bench.py [--configs cfg2,cfg5] [--rounds 5] [--reps 10]

Prints one JSON line per (config, form): median / min ms per full match (device-resident
stacks, the bench's synthetic frame) and the transform + search part alone (the match
without NXC, which is exactly the two kernels, or the one fused kernel), after checking
both forms give identical maps.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from libbicos_amd import device  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg2,cfg5")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    eng = device.Engine(0)
    for name in args.configs.split(","):
        C = bench.CONFIGS[name]
        n, H, W = C["n"], C["H"], C["W"]
        L, R = stereo_stack(n, H, W, np.uint8)
        s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
        full = device.MatchConfig(**C["cfg"])
        kw = dict(C["cfg"])
        kw.pop("min_variance", None)
        kw.pop("subpixel_step", None)
        kw["nxcorr_threshold"] = None  # no NXC (the reference's default is 0.5)
        bare = device.MatchConfig(**kw)  # transform + search only
        out = {}
        for form in ("0", "1"):
            os.environ["BICOS_FUSE_TRANSFORM"] = form
            out[form] = [t.clone() for t in eng.match(s0, s1, full) if t is not None]
        for a, b in zip(out["0"], out["1"]):
            if not torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a,
                               b.view(torch.int32) if b.dtype == torch.float32 else b):
                raise SystemExit("%s: fused and separate maps differ" % name)
        times = {(f, what): [] for f in ("0", "1") for what in ("match", "transform+search")}
        st = torch.cuda.current_stream()
        for _ in range(args.rounds):
            for form in ("0", "1"):
                os.environ["BICOS_FUSE_TRANSFORM"] = form
                for what, cfg in (("match", full), ("transform+search", bare)):
                    eng.match(s0, s1, cfg)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    for _ in range(args.reps):
                        eng.match(s0, s1, cfg)
                    b.record(st)
                    torch.cuda.synchronize()
                    times[(form, what)].append(a.elapsed_time(b) / args.reps)
        for (form, what), v in times.items():
            print(json.dumps({"config": name, "form": "fused" if form == "1" else "separate",
                              "what": what, "ms_median": round(statistics.median(v), 4),
                              "ms_min": round(min(v), 4)}), flush=True)
    os.environ.pop("BICOS_FUSE_TRANSFORM", None)


if __name__ == "__main__":
    main()
