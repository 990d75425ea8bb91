"""How often the matrix-core NoDuplicates search (search_mx.hip, KEYS 2) takes its
last-minimum branch, for a given block visiting order -- a CPU simulation on real
descriptors of the synthetic stereo frame (or random ones).

A (tile, block) unit "reaches" when some col0 of the 32-column tile has its block minimum
cost <= its running minimum cost over the blocks visited before; the kernel then runs the
last-minimum tree of that tile for that block. The transform here is a plain numpy LIMITED
transform (bit order is irrelevant to Hamming costs); nothing here is used by the library.

  python tools/reach_sim.py [--config cfg2] [--rows 4] [--random]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from libbicos_amd.synthetic import random_stack, stereo_stack  # noqa: E402

POP = np.array([bin(i).count("1") for i in range(256)], np.uint8)


def limited_bits(stack):
    """[n, rows, W] -> [rows, W, nbits] bool (LIMITED comparisons, any fixed order)."""
    s = stack.astype(np.int64)
    n = s.shape[0]
    mean = s.sum(axis=0) / n
    bits = []
    for t in range(n - 2):
        a, b, c = s[t], s[t + 1], s[t + 2]
        bits += [a < b, a < c, a < mean]
        if t >= 2:
            bits.append(s[t - 2] + s[t - 1] < a + b)
    a, b = s[n - 2], s[n - 1]
    bits += [a < b, a < mean, b < mean, s[n - 4] + s[n - 3] < a + b]
    return np.stack(bits, axis=-1)


def pack(bits):
    nb = bits.shape[-1]
    pad = (-nb) % 8
    if pad:
        bits = np.concatenate([bits, np.zeros(bits.shape[:-1] + (pad,), bool)], axis=-1)
    return np.packbits(bits, axis=-1)


def costs(d0, d1):
    """[W, B] x [W, B] bytes -> [W0, W1] Hamming costs."""
    x = d0[:, None, :] ^ d1[None, :, :]
    return POP[x].sum(axis=-1, dtype=np.int32)


def order_current(c0_wave, wg_c0_hi, cols, chunk):
    """The kernel's order: chunks downwards from the one holding the workgroup's highest col0,
    in each chunk full blocks downwards from the one holding the wave's highest col0."""
    nchunks = (cols + chunk - 1) // chunk
    cstart = min(cols - 1, wg_c0_hi) // chunk
    out = []
    for k in range(nchunks):
        ci = (cstart - k) % nchunks
        base = ci * chunk
        ncols = min(chunk, cols - base)
        nfull = ncols // 32
        if ncols % 32:
            out.append(base + 32 * nfull)
        sb = max(0, min(nfull - 1, (c0_wave + 127 - base) // 32))
        for i in range(nfull):
            out.append(base + 32 * ((sb - i) % nfull))
    return out


def order_from(c0_ref):
    def f(c0_wave, wg_c0_hi, cols, chunk):
        nchunks = (cols + chunk - 1) // chunk
        cstart = min(cols - 1, wg_c0_hi) // chunk
        out = []
        for k in range(nchunks):
            ci = (cstart - k) % nchunks
            base = ci * chunk
            ncols = min(chunk, cols - base)
            nfull = ncols // 32
            if ncols % 32:
                out.append(base + 32 * nfull)
            sb = max(0, min(nfull - 1, (c0_wave + c0_ref - base) // 32))
            for i in range(nfull):
                out.append(base + 32 * ((sb - i) % nfull))
        return out
    return f


def simulate(C, order_fn, cols, waves=8, T=4, chunk=1024):
    units = reach = 0
    per_wg = waves * T * 32
    for wg in range((cols + per_wg - 1) // per_wg):
        for w in range(waves):
            c0_wave = wg * per_wg + w * T * 32
            if c0_wave >= cols:
                continue
            blocks = order_fn(c0_wave, (wg + 1) * per_wg - 1, cols, chunk)
            for t in range(T):
                lo, hi = c0_wave + 32 * t, min(cols, c0_wave + 32 * t + 32)
                if lo >= cols:
                    continue
                run = np.full(hi - lo, 1 << 30)
                for B in blocks:
                    bm = C[lo:hi, B:min(cols, B + 32)].min(axis=1)
                    units += 1
                    if (bm <= run).any():
                        reach += 1
                    run = np.minimum(run, bm)
    return reach, units


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4)
    ap.add_argument("--W", type=int, default=2048)
    ap.add_argument("--n", type=int, default=33)
    ap.add_argument("--random", action="store_true")
    args = ap.parse_args()
    H = 1536
    rows = np.linspace(0, H - 1, args.rows).astype(int)
    orders = {"current (wave top)": order_current, "wave col0 + 96": order_from(96),
              "wave col0 + 64": order_from(64), "wave col0 + 32": order_from(32),
              "wave col0": order_from(0)}
    tot = {k: [0, 0] for k in orders}
    for r in rows:
        if args.random:
            L = random_stack(args.n, 1, args.W, seed=int(r) + 1)
            R = random_stack(args.n, 1, args.W, seed=int(r) + 7)
        else:
            L, R = stereo_stack(args.n, H, args.W, row_begin=int(r), row_end=int(r) + 1)
        d0, d1 = pack(limited_bits(L))[0], pack(limited_bits(R))[0]
        C = costs(d0, d1)
        for k, f in orders.items():
            a, b = simulate(C, f, args.W)
            tot[k][0] += a
            tot[k][1] += b
    for k, (a, b) in tot.items():
        print("%-22s reaching %.4f of (tile, block) units" % (k, a / b))


if __name__ == "__main__":
    main()
