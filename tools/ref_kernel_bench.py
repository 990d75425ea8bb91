"""Our stages on the reference's own kernel-bench shapes (reference bench/cuda.cu), next to
the RTX 4090 numbers it publishes (bench/baselines/cuda-rtx4090.txt). All at 3300x2200
(bench/cuda.cu:44), random inputs as there (cv::randu over the full u8 / u16 range):

  transform  LIMITED with the largest stack per descriptor width (u32: n = 9, u64: 17,
             u128: 33) and FULL (u32: 6, u64: 8, u128: 12) -- bench/cuda.cu:258-295
  agree      n = 10, random disparities in [-1, 3300), threshold 0.9, min-variance 10,
             double precision -- bench/cuda.cu:99-137
  subpixel   the same, step 0.25 -- bench/cuda.cu:139-180
  search     u128 NoDuplicates on random descriptors (bicos_kernel_smem) -- :218-256

Each is timed with HIP events on the stream it runs on, median of 3 rounds of --reps.

  python tools/ref_kernel_bench.py [--reps 20] [--out profiles/ref_kernel_bench_r03.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libbicos_amd import device  # noqa: E402

H, W = 2200, 3300
REF = {  # ns, bench/baselines/cuda-rtx4090.txt
    ("transform", "u8", 0, 1): 212004, ("transform", "u16", 0, 1): 201617,
    ("transform", "u8", 0, 2): 348477, ("transform", "u16", 0, 2): 378625,
    ("transform", "u8", 0, 4): 1027874, ("transform", "u16", 0, 4): 1075632,
    ("transform", "u8", 1, 1): 202812, ("transform", "u16", 1, 1): 213822,
    ("transform", "u8", 1, 2): 369482, ("transform", "u16", 1, 2): 374232,
    ("transform", "u8", 1, 4): 929152, ("transform", "u16", 1, 4): 936285,
    ("agree", "u8"): 1947801, ("agree", "u16"): 1949397,
    ("subpixel", "u8"): 2022930, ("subpixel", "u16"): 1980028,
    ("search", "u128"): 18821371,
}
LIMITED_N = {1: 9, 2: 17, 4: 33}
FULL_N = {1: 6, 2: 8, 4: 12}  # max_stacksize_v FULL (impl/common.hpp:69-73)


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return statistics.median(ts)


def rand_stack(n, dt, g):
    if dt == "u8":
        return torch.randint(0, 256, (n, H, W), dtype=torch.uint8, device="cuda", generator=g)
    # u16 over the full range, held as int16 bit patterns (the engine reads them as u16)
    return torch.randint(-32768, 32768, (n, H, W), dtype=torch.int16, device="cuda", generator=g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--stages", default="transform,agree,search",
                    help="comma list of transform / agree (agree + subpixel) / search")
    args = ap.parse_args()
    stages = set(args.stages.split(","))
    eng = device.Engine(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x600DF00D)
    lines = []

    def emit(d):
        ref = REF.get(d.pop("key"))
        if ref:
            d["reference_rtx4090_ms"] = round(ref / 1e6, 4)
            d["speedup_vs_rtx4090"] = round(ref / 1e6 / d["ms"], 2)
        lines.append(d)
        print(json.dumps(d), flush=True)

    for dt in ("u8", "u16"):
        for mode, table in ((0, LIMITED_N), (1, FULL_N)) if "transform" in stages else ():
            for words, n in table.items():
                s = rand_stack(n, dt, g)
                out = eng.transform(s, mode, words)
                ms = timed(lambda: eng.transform(s, mode, words, out=out), args.reps)
                px = H * W
                emit({"stage": "transform", "input": dt, "mode": ["LIMITED", "FULL"][mode],
                      "n": n, "descriptor_bits": 32 * words, "ms": round(ms, 4),
                      "GBps": round(px * (n * (1 if dt == "u8" else 2) + 4 * words) / ms / 1e6, 1),
                      "key": ("transform", dt, mode, words)})
                del s, out
        if "agree" not in stages:
            continue
        n = 10
        s0, s1 = rand_stack(n, dt, g), rand_stack(n, dt, g)
        raw = torch.randint(-1, W, (H, W), dtype=torch.int16, device="cuda", generator=g)
        for prec in (1, 0):
            for stage, step in (("agree", None), ("subpixel", 0.25)):
                ms = timed(lambda: eng.agree(raw, s0, s1, 0.9, 10.0, step=step, precision=prec),
                           args.reps)
                emit({"stage": stage, "input": dt, "n": n, "precision": ["SINGLE", "DOUBLE"][prec],
                      "step": step, "threshold": 0.9, "minvar_scaled": 10.0, "ms": round(ms, 4),
                      "key": (stage, dt) if prec else None})
        del s0, s1, raw
    if "search" in stages:
        words = 4
        pitch = eng._L.bicos_desc_pitch(W, words)
        d0 = torch.randint(-2 ** 31, 2 ** 31 - 1, (H, pitch), dtype=torch.int32, device="cuda", generator=g)
        d1 = torch.randint(-2 ** 31, 2 ** 31 - 1, (H, pitch), dtype=torch.int32, device="cuda", generator=g)
        out = eng.search(d0, d1, W, words, 1)
        ms = timed(lambda: eng.search(d0, d1, W, words, 1, out=out), max(3, args.reps // 4))
        emit({"stage": "search", "input": "random u128 descriptors", "flags": "NODUPES",
              "ms": round(ms, 4), "key": ("search", "u128")})
    if args.out:
        with open(args.out, "a") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
