"""TEST INFRASTRUCTURE ONLY -- a second, independent restatement of the
reference CPU path in vectorised numpy, used to cross-check bicos_oracle.c on
small inputs (the reference binary itself cannot be built here; see
bicos_oracle.h for the parity status). Python loops only over image planes,
descriptor bits, rows and subpixel steps -- keep inputs small.

Follows: include/impl/cpu/descriptor_transform.hpp:31-123,
include/impl/cpu/bicos.hpp:29-113, include/impl/cpu/agree.hpp:28-191,
src/impl/cpu.cpp:35-159 (all paths relative to the reference checkout).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

f32 = np.float32
INVALID16 = np.int16(-32768)


# ------------------------------------------------------------------ float32 fma
def fma32(a, b, c):
    """Correctly rounded float32 fma(a, b, c) (std::fmaf) without hardware fma:
    the float64 product of two float32 is exact; the float64 sum is made
    round-to-odd from its TwoSum error term, after which a single rounding to
    float32 is correct (53 >= 24 + 2 bits)."""
    a = np.asarray(a, np.float32).astype(np.float64)
    b = np.asarray(b, np.float32).astype(np.float64)
    c = np.asarray(c, np.float32).astype(np.float64)
    p = a * b
    s = p + c
    bb = s - p
    err = (p - (s - bb)) + (c - bb)
    bits = s.view(np.int64)
    even = (bits & 1) == 0
    fix = (err != 0) & even & np.isfinite(s)
    s = np.where(fix, np.nextafter(s, np.where(err > 0, np.inf, -np.inf)), s)
    return s.astype(np.float32)


# -------------------------------------------------------------------- transform
def _mean(planes: List[np.ndarray]) -> np.ndarray:
    av = np.zeros(planes[0].shape, np.float32)
    for p in planes:
        av = (av + p.astype(np.float32)).astype(np.float32)
    return (av / f32(len(planes))).astype(np.float32)


def _pack(bits: List[np.ndarray], words: int) -> np.ndarray:
    out = np.zeros(bits[0].shape + (words,), np.uint32)
    for i, b in enumerate(bits):
        if i // 32 < words:
            out[..., i // 32] |= b.astype(np.uint32) << np.uint32(i % 32)
    return out


def transform(stack: np.ndarray, mode: int, words: int) -> np.ndarray:
    n = stack.shape[0]
    p = [stack[t].astype(np.int64) for t in range(n)]
    av = _mean([stack[t] for t in range(n)])
    bits: List[np.ndarray] = []
    if mode == 0:  # LIMITED (descriptor_transform.hpp:31-73)
        ring = [None, None]
        for t in range(n - 2):
            a, b, c = p[t], p[t + 1], p[t + 2]
            bits += [a < b, a < c, a.astype(np.float32) < av]
            cur = a + b
            if ring[t % 2] is not None:
                bits.append(ring[t % 2] < cur)
            ring[t % 2] = cur
        a, b = p[n - 2], p[n - 1]
        bits += [a < b, a.astype(np.float32) < av, b.astype(np.float32) < av]
        prev = ring[(n - 2) % 2]
        bits.append(np.ones_like(a, bool) if prev is None else prev < a + b)
    else:  # FULL (descriptor_transform.hpp:75-123)
        for t in range(n - 2):
            a, b, c = p[t], p[t + 1], p[t + 2]
            bits += [a < b, a < c, a.astype(np.float32) < av]
        ps = [p[t] + p[t + 1] for t in range(n - 1)]
        a, b = p[n - 2], p[n - 1]
        bits += [a < b, a.astype(np.float32) < av, b.astype(np.float32) < av]
        for t in range(n - 1):
            for i in range(n - 1):
                if i in (t - 1, t, t + 1):
                    continue
                bits.append(ps[t] < ps[i])
    return _pack(bits, words)


# ----------------------------------------------------------------------- search
def _row_costs(d0row: np.ndarray, d1row: np.ndarray) -> np.ndarray:
    x = d0row[:, None, :] ^ d1row[None, :, :]
    return np.bitwise_count(x).sum(axis=2).astype(np.int64)  # [col0, col1]


def _argmin_rows(cost: np.ndarray, nodupes: bool) -> np.ndarray:
    best = np.argmin(cost, axis=1)  # first minimum = lowest index (strict '<' scan)
    if nodupes:
        mins = cost[np.arange(cost.shape[0]), best]
        dup = (cost == mins[:, None]).sum(axis=1) > 1
        best = np.where(dup, -1, best)
    return best


def search(d0: np.ndarray, d1: np.ndarray, flags: int, max_lr_diff: int = -1) -> np.ndarray:
    H, W, _ = d0.shape
    out = np.full((H, W), INVALID16, np.int16)
    nodupes = bool(flags & 1)
    for r in range(H):
        cost = _row_costs(d0[r], d1[r])
        fwd = _argmin_rows(cost, nodupes)
        col0 = np.arange(W)
        if flags & 2:
            rev = _argmin_rows(cost.T, nodupes)  # ham is symmetric
            ok = fwd >= 0
            r0 = np.where(ok, rev[np.maximum(fwd, 0)], -1)
            ok &= (r0 >= 0) & (np.abs(col0 - r0) <= max_lr_diff)
            val = (col0 + r0) // 2 - fwd
        else:
            ok = fwd >= 0
            val = col0 - fwd
        out[r] = np.where(ok, val, INVALID16).astype(np.int16)
    return out


# ------------------------------------------------------------------------ agree
def nxcorr(pix0: np.ndarray, pix1: np.ndarray, minvar: Optional[float]) -> np.ndarray:
    """pix0, pix1: [n, K] integer samples -> [K] float32 (agree.hpp:28-51)."""
    n = pix0.shape[0]
    m0 = np.zeros(pix0.shape[1:], np.float32)
    m1 = np.zeros(pix0.shape[1:], np.float32)
    for i in range(n):
        m0 = (m0 + pix0[i].astype(np.float32)).astype(np.float32)
        m1 = (m1 + pix1[i].astype(np.float32)).astype(np.float32)
    m0 = (m0 / f32(n)).astype(np.float32)
    m1 = (m1 / f32(n)).astype(np.float32)
    cov = np.zeros_like(m0)
    v0 = np.zeros_like(m0)
    v1 = np.zeros_like(m0)
    for i in range(n):
        a = (pix0[i].astype(np.float32) - m0).astype(np.float32)
        b = (pix1[i].astype(np.float32) - m1).astype(np.float32)
        cov = fma32(a, b, cov)
        v0 = fma32(a, a, v0)
        v1 = fma32(b, b, v1)
    with np.errstate(divide="ignore", invalid="ignore"):
        res = (cov / np.sqrt((v0 * v1).astype(np.float32))).astype(np.float32)
    if minvar is not None:
        mv = f32(minvar)
        res = np.where((v0 < mv) | (v1 < mv), f32(-1.0), res).astype(np.float32)
    return res


def agree(disp: np.ndarray, s0: np.ndarray, s1: np.ndarray, thr: float, minvar):
    n, H, W = s0.shape
    d = disp.astype(np.int16).copy()
    corr = np.full((H, W), np.nan, np.float32)
    rr, cc = np.nonzero(d != INVALID16)
    idx1 = cc - d[rr, cc].astype(np.int64)
    oob = (idx1 < 0) | (idx1 >= W)
    d[rr[oob], cc[oob]] = INVALID16
    rr, cc, idx1 = rr[~oob], cc[~oob], idx1[~oob]
    nxc = nxcorr(s0[:, rr, cc], s1[:, rr, idx1], minvar)
    corr[rr, cc] = nxc
    bad = nxc < f32(thr)
    d[rr[bad], cc[bad]] = INVALID16
    return d, corr


def x_steps(step: float) -> List[np.float32]:
    xs = []
    x = f32(-1.0)
    while x <= f32(1.0):
        xs.append(x)
        x = f32(x + f32(step))
    return xs


def _narrow(v: np.ndarray, dtype) -> np.ndarray:
    i = np.rint(v).astype(np.int64).astype(np.int32)  # values are small: exact
    return (i & (0xFF if dtype == np.uint8 else 0xFFFF)).astype(np.int64)


def agree_subpixel(disp, s0, s1, thr: float, step: float, minvar):
    n, H, W = s0.shape
    out = np.full((H, W), np.nan, np.float32)
    corr = np.full((H, W), np.nan, np.float32)
    d = disp.astype(np.int64)
    rr, cc = np.nonzero(disp != INVALID16)
    col1 = cc - d[rr, cc]
    keep = (col1 >= 0) & (col1 < W)
    rr, cc, col1 = rr[keep], cc[keep], col1[keep]
    edge = (col1 == 0) | (col1 == W - 1)

    # edges: plain correlation, integer disparity
    er, ec, e1 = rr[edge], cc[edge], col1[edge]
    if er.size:
        nxc = nxcorr(s0[:, er, ec], s1[:, er, e1], minvar)
        corr[er, ec] = nxc
        ok = ~(nxc < f32(thr))
        out[er[ok], ec[ok]] = d[er[ok], ec[ok]].astype(np.float32)

    ir, ic, i1 = rr[~edge], cc[~edge], col1[~edge]
    if ir.size:
        left = s0[:, ir, ic]
        y0 = s1[:, ir, i1 - 1].astype(np.float32)
        y1 = s1[:, ir, i1].astype(np.float32)
        y2 = s1[:, ir, i1 + 1].astype(np.float32)
        A = (f32(0.5) * ((y0 - f32(2.0) * y1).astype(np.float32) + y2)).astype(np.float32)
        B = (f32(0.5) * (-s1[:, ir, i1 - 1].astype(np.int64)
                         + s1[:, ir, i1 + 1].astype(np.int64)).astype(np.float32)).astype(np.float32)
        C = y1
        best_x = np.zeros(ir.size, np.float32)
        best = np.full(ir.size, -1.0, np.float32)
        for x in x_steps(step):
            ax = (A * x).astype(np.float32)
            v = (((ax * x).astype(np.float32) + (B * x).astype(np.float32)).astype(np.float32)
                 + C).astype(np.float32)
            interp = _narrow(v, s0.dtype)
            nxc = nxcorr(left, interp, minvar)
            win = best < nxc
            best_x = np.where(win, x, best_x)
            best = np.where(win, nxc, best)
        corr[ir, ic] = best
        ok = ~(best < f32(thr))
        out[ir[ok], ic[ok]] = (d[ir[ok], ic[ok]].astype(np.float32) - best_x[ok]).astype(np.float32)
    return out, corr


# ------------------------------------------------------------------------ match
def desc_words(n: int, mode: int) -> int:
    bits = n * n - 2 * n + 3 if mode == 1 else 4 * n - 7
    for w in (1, 2, 4, 8):
        if bits <= 32 * w:
            return w
    raise ValueError("input stacks too large, would require %d bits" % bits)


def match(s0, s1, nxcorr_threshold=0.5, subpixel_step=None, min_variance=None, mode=0,
          variant=0, max_lr_diff=1, no_dupes=False):
    n = s0.shape[0]
    words = desc_words(n, mode)
    d0 = transform(s0, mode, words)
    d1 = transform(s1, mode, words)
    if variant == 1:
        raw = search(d0, d1, 2 | (1 if no_dupes else 0), max_lr_diff)
    else:
        raw = search(d0, d1, 1)
    if nxcorr_threshold is None:
        return raw, None
    mv = None if min_variance is None else f32(f32(min_variance) * f32(n))
    if subpixel_step is not None:
        return agree_subpixel(raw, s0, s1, nxcorr_threshold, subpixel_step, mv)
    d, corr = agree(raw, s0, s1, nxcorr_threshold, mv)
    return d.astype(np.float32), corr
