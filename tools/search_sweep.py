"""A/B the search-kernel variants in ONE process, interleaved rounds (guide s5.4 rule 24).

  python tools/search_sweep.py [--config cfg2] [--rounds 5] [--reps 5] [--rows R]

Prints one JSON line per (variant, col0_per_lane, waves) with median/min ms per launch
and Tops/s (algorithmic int32 lane-ops), after checking every variant's output is
identical to the first one's.
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
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rows", type=int, default=0, help="row band size (0 = full frame)")
    ap.add_argument("--variants", default="0:0:0,16:2:8,16:4:8,16:2:4,16:4:4")
    ap.add_argument("--all-bits", action="store_true", help="no used-bits hint (all K-steps)")
    ap.add_argument("--random", action="store_true", help="random descriptors (u128 kernel-bench input)")
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    rows = args.rows or H
    cfg = device.MatchConfig(**C["cfg"])
    words = device.descriptor_words(n, cfg.mode)
    L, R = stereo_stack(n, H, W, np.uint8, row_begin=0, row_end=rows)
    eng = device.Engine(0)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    d0, d1 = eng.transform(s0, cfg.mode, words), eng.transform(s1, cfg.mode, words)
    flags = (2 | (1 if cfg.no_dupes else 0)) if cfg.variant == 1 else 1
    ops = bench.search_ops(rows, W, words, C["cfg"])
    bits = 0 if args.all_bits else device.used_bits(n, cfg.mode)
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    variants = [v + (0,) * (4 - len(v)) for v in variants]
    if args.random:
        g = torch.Generator(device="cuda").manual_seed(1)
        for d in (d0, d1):
            d.copy_(torch.randint(-2**31, 2**31 - 1, d.shape, dtype=torch.int32, device="cuda", generator=g))
            if bits:  # only the bits the transform would set (the FK keys need the rest 0)
                v = d[:, :W * words].view(rows, W, words)
                for q in range(words):
                    keep = 0 if 32 * q >= bits else min(32, bits - 32 * q)
                    m = (1 << keep) - 1
                    v[:, :, q] &= (m - (1 << 32) if m >= 1 << 31 else m)
    times = {v: [] for v in variants}
    ref = None
    st = torch.cuda.current_stream()
    for rnd in range(args.rounds):
        for v in variants:
            eng.tune(*v)
            out = eng.search(d0, d1, W, words, flags, cfg.max_lr_diff, bits=bits)
            if rnd == 0:
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                elif not torch.equal(ref, out):
                    raise SystemExit("variant %s output differs" % (v,))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(args.reps):
                eng.search(d0, d1, W, words, flags, cfg.max_lr_diff, out=out, bits=bits)
            b.record(st)
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b) / args.reps)
    for v in variants:
        med, mn = statistics.median(times[v]), min(times[v])
        print(json.dumps({"config": args.config, "rows": rows, "variant": v[0], "col0_per_lane": v[1],
                          "waves": v[2], "split": v[3], "random": args.random, "ms_median": round(med, 4), "ms_min": round(mn, 4),
                          "Tops": round(ops / (med * 1e-3) / 1e12, 2)}))


if __name__ == "__main__":
    main()
