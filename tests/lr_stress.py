"""Randomised parity stress of the one-launch Consistency search (search_mx.hip
search_lr_kernel) against the oracle at the descriptor level: random widths (1..2048), used
bits (129..154), max_lr_diff (0..6), row counts and descriptor families (random, shifted
copies with bit flips, low-entropy with heavy ties both ways, few distinct popcounts). Test
infrastructure (it runs the oracle): the GPU suite runs 300 cases (test_lr_stress); run
directly for more, one JSON line per case to --out, exiting non-zero at the first mismatch
(its case is the last line):

    python tests/lr_stress.py --cases 4000 --out gpurun_out/lr_stress.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mask_bits(d, bits):
    full = np.zeros(8, np.uint32)
    for b in range(bits):
        full[b // 32] |= np.uint32(1 << (b % 32))
    return d & full


def family(rng, H, W, bits, kind):
    if kind == "random":
        d = rng.integers(0, 2 ** 32, size=(H, W, 8), dtype=np.uint64).astype(np.uint32)
    elif kind == "low":
        d = np.zeros((H, W, 8), np.uint32)
        d[..., 0] = rng.integers(0, 1 << int(rng.integers(1, 6)), size=(H, W), dtype=np.uint32)
        d[..., 4] = np.where(rng.random((H, W)) < 0.5, np.uint32(0xFFFFFFFF), np.uint32(0))
    else:  # "popcount": a few descriptors repeated, ties on distance everywhere
        base = rng.integers(0, 2 ** 32, size=(int(rng.integers(1, 5)), 8), dtype=np.uint64).astype(np.uint32)
        d = base[rng.integers(0, len(base), size=(H, W))]
    return mask_bits(d, bits)


def run(cases, seed, out):
    """Returns (number of bit-exact cases, the first mismatching case's record or None)."""
    import torch
    from libbicos_amd.device import Engine
    from oracle import oracle
    from tests.test_gpu_parity import _pack
    eng = Engine(0)
    rng = np.random.default_rng(seed)
    if out:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    t0 = time.time()
    with open(out or os.devnull, "w") as f:
        for i in range(cases):
            W = int(rng.choice([1, 2, 31, 32, 33, 63, 64, 65, 127, 128, 129, 383, 384, 385, 511,
                                512, 513, 1023, 1024, 1025, 1536, 2047, 2048,
                                int(rng.integers(1, 2049))]))
            H = int(rng.integers(1, 6))
            bits = int(rng.integers(129, 155))
            lr = int(rng.integers(0, 7))
            kind = str(rng.choice(["random", "low", "popcount", "shifted"]))
            a = family(rng, H, W, bits, "random" if kind == "shifted" else kind)
            if kind == "shifted":
                flip = (rng.random((H, W, 8)) < 0.03).astype(np.uint32) << \
                    rng.integers(0, 32, (H, W, 8)).astype(np.uint32)
                b = mask_bits(a[:, np.roll(np.arange(W), int(rng.integers(0, 9)))] ^ flip, bits)
            else:
                b = family(rng, H, W, bits, kind)
            ref = oracle.search(a, b, 2, lr)
            d0 = torch.from_numpy(_pack(a)).cuda()
            d1 = torch.from_numpy(_pack(b)).cuda()
            res = eng.search(d0, d1, W, 8, 2, lr, bits=bits).cpu().numpy()
            ok = bool(np.array_equal(res, ref))
            rec = {"case": i, "W": W, "H": H, "bits": bits, "lr": lr, "kind": kind, "ok": ok,
                   "valid": float((ref != -32768).mean())}
            f.write(json.dumps(rec) + "\n")
            f.flush()
            if not ok:
                bad = np.argwhere(res != ref)[0]
                rec["first"] = [bad.tolist(), int(res[tuple(bad)]), int(ref[tuple(bad)])]
                return i, rec
            if i % 250 == 0:
                print("case %d ok (%.0f s)" % (i, time.time() - t0), flush=True)
    return cases, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--seed", type=int, default=6)
    ap.add_argument("--out", default="gpurun_out/lr_stress.jsonl")
    args = ap.parse_args()
    n, bad = run(args.cases, args.seed, args.out)
    if bad:
        print("MISMATCH", bad)
        return 1
    print("all %d cases bit-exact" % n)
    return 0


if __name__ == "__main__":
    sys.exit(main())
