"""The search kernel on the reference's own kernel-bench input:
random 128-bit descriptors at 3300x2200 (reference bench/cuda.cu:44,218-256; RTX 4090:
bicos_kernel_smem<u128,NODUPES> 18.82 ms, <u128,CONSISTENCY> 36.76 ms, <u128,NODUPES|
CONSISTENCY> 18.95 ms -- bench/baselines/cuda-rtx4090.txt:50-54), next to inputs of other
textures at the same size: the planted-disparity synthetic stack (transform output), a
low-texture stack (8 grey levels + noise) and a repeating pattern (period 64 columns:
every minimum duplicated). The matrix-core search skips last-minimum work where a block
cannot hold the minimum, so its speed depends on the data; this measures how much.

Round 5: the 32- and 64-bit random points of the same bench (bench/cuda.cu:353-366,
cuda-rtx4090.txt:38-48; `--words 1,2,4`), and the reverse search over only the col1 the
forward search kept (BICOS_REV_FULL=1 in the environment times the full reverse pass).

  python tools/random_search_bench.py [--reps 10] [--words 1,2,4] [--inputs random]
                                      [--out profiles/random_search_r05.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from libbicos_amd import device  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402

H, W = 2200, 3300
WORDS = 4
# RTX 4090, the faster of bicos_kernel / bicos_kernel_smem (bench/baselines/cuda-rtx4090.txt:38-54)
REF_MS = {1: {1: 9.43, 2: 11.15, 3: 9.49}, 2: {1: 11.31, 2: 18.38, 3: 11.43},
          4: {1: 18.82, 2: 36.76, 3: 18.95}}


def time_search(eng, d0, d1, flags, lr, reps, bits):
    out = eng.search(d0, d1, W, WORDS, flags, lr, bits=bits)
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(3):
        for _ in range(3):
            eng.search(d0, d1, W, WORDS, flags, lr, out=out, bits=bits)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            eng.search(d0, d1, W, WORDS, flags, lr, out=out, bits=bits)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    o = out.cpu().numpy()
    return statistics.median(ts), min(ts), float((o != -32768).mean() if flags != 2 else (o != -32768).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--words", default="4", help="random-descriptor widths: 1, 2, 4 words")
    ap.add_argument("--inputs", default="", help="comma list of input names (default: all)")
    args = ap.parse_args()
    eng = device.Engine(0)
    pitch = eng._L.bicos_desc_pitch(W, WORDS)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x600DF00D)

    def rand_desc(words=WORDS):
        return torch.randint(-2 ** 31, 2 ** 31 - 1, (H, eng._L.bicos_desc_pitch(W, words)),
                             dtype=torch.int32, device="cuda", generator=g)

    wanted = set(filter(None, args.inputs.split(",")))
    inputs = {}
    for w in (int(x) for x in args.words.split(",")):
        inputs["random_u%d" % (32 * w)] = (rand_desc(w), rand_desc(w), 0, w)
    if wanted and not (wanted - set(inputs)):
        return run(eng, inputs, args)
    n = 33
    L, R = stereo_stack(n, H, W, np.uint8)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    inputs["planted_stereo_n33"] = (eng.transform(s0, 0, WORDS), eng.transform(s1, 0, WORDS),
                                    device.used_bits(n, 0), WORDS)
    rng = np.random.default_rng(7)
    flat = (rng.integers(0, 8, size=(n, H, W)) * 32 + rng.integers(0, 3, size=(n, H, W))).astype(np.uint8)
    t = torch.from_numpy(flat).cuda()
    inputs["low_texture_n33"] = (eng.transform(t, 0, WORDS), eng.transform(t, 0, WORDS).roll(WORDS * 5, 1),
                                 device.used_bits(n, 0), WORDS)
    base = rand_desc()[:, :64 * WORDS]
    rep = base.repeat(1, (pitch + 64 * WORDS - 1) // (64 * WORDS))[:, :pitch].contiguous()
    inputs["periodic64_u128"] = (rep, rep.clone(), 0, WORDS)
    del L, R, s0, s1, t, flat
    if wanted:
        inputs = {k: v for k, v in inputs.items() if k in wanted}
    run(eng, inputs, args)


def run(eng, inputs, args):
    global WORDS
    lines = []
    rev = "full" if os.environ.get("BICOS_REV_FULL", "0") not in ("", "0") else "kept col1 only"
    for name, (d0, d1, bits, words) in inputs.items():
        WORDS = words
        for flags, lr, label in ((1, -1, "NODUPES"), (2, 3, "CONSISTENCY"),
                                 (3, 3, "NODUPES|CONSISTENCY")):
            med, mn, valid = time_search(eng, d0, d1, flags, lr, args.reps, bits)
            ref_ms = REF_MS[words][flags] if name.startswith("random_") else None
            line = {"input": name, "rows": H, "cols": W, "descriptor_bits": 32 * words,
                    "flags": label, "ms_median": round(med, 4), "ms_min": round(mn, 4),
                    "Gpairs_per_s": round(H * W * W / (med * 1e-3) / 1e9, 1),
                    "valid_fraction": round(valid, 4),
                    "reverse_search": rev if flags & 2 else None,
                    "rtx4090_reference_ms": ref_ms,
                    "x_rtx4090": round(ref_ms / med, 2) if ref_ms else None}
            print(json.dumps(line), flush=True)
            lines.append(line)
    if args.out:
        with open(args.out, "a") as f:
            for l in lines:
                f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main()
