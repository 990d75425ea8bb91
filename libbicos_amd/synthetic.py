"""Synthetic multi-shot stereo stacks.

There is no network and the reference's example dataset (data/prepare.sh) is
download-only, so every test and benchmark runs on synthetic planar stacks:

  Left(t, y, x)  ~ U[0, maxval]                       (portable splitmix64 stream)
  Right(t, y, x) = clamp(Left(t, y, x + d(y)) + U{-1,0,1}, 0, maxval)
  d(y)           = dmin + floor(drange * y / H)      (16 + floor(48 y / H) by default)
  columns with x + d(y) >= W are fresh U[0, maxval] draws (out of view)

The planted disparity is therefore d(y) (left col - right col), the sign
convention of the reference (bicos.hpp:109 `col0 - best_col1`). The PRNG is a
counter-based splitmix64 so the same stack can be regenerated bit-identically
from numpy on any host, for any band of rows (multi-GPU shards generate only
their own rows).
"""
from __future__ import annotations

import numpy as np

SEED = 0x600DF00D  # bench/cuda.cu:39 of the reference

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(counter: np.ndarray, seed: int) -> np.ndarray:
    """splitmix64 output for 0-based counters (vectorised, wraps mod 2**64)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (counter.astype(np.uint64) + np.uint64(1)) * _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _uniform(counter: np.ndarray, seed: int, maxval: int) -> np.ndarray:
    # top 32 bits scaled to [0, maxval] (multiply-shift, no modulo bias worth noting)
    hi = splitmix64(counter, seed) >> np.uint64(32)
    return ((hi * np.uint64(maxval + 1)) >> np.uint64(32)).astype(np.int64)


def planted_disparity(rows: int, H: int, dmin: int = 16, drange: int = 48) -> np.ndarray:
    y = np.arange(rows[0], rows[1]) if isinstance(rows, tuple) else np.arange(rows)
    return dmin + (drange * y) // H


def stereo_stack(n: int, H: int, W: int, dtype=np.uint8, seed: int = SEED, row_begin: int = 0,
                 row_end: int | None = None, dmin: int = 16, drange: int = 48,
                 maxval: int | None = None):
    """Returns (left, right) planar stacks of shape [n, rows, W] for rows
    [row_begin, row_end) of an H x W scene."""
    row_end = H if row_end is None else row_end
    maxval = (255 if np.dtype(dtype) == np.uint8 else 4095) if maxval is None else maxval
    rows = row_end - row_begin
    ys = np.arange(row_begin, row_end, dtype=np.int64)[:, None]
    xs = np.arange(W, dtype=np.int64)[None, :]
    d = dmin + (drange * ys) // H
    left = np.empty((n, rows, W), dtype)
    right = np.empty((n, rows, W), dtype)
    P = np.int64(H) * W
    for t in range(n):
        base = np.int64(t) * P
        # left plane t, and the left value Right(y, x) looks at: Left(y, x + d)
        lidx = base + ys * W + xs
        left[t] = _uniform(lidx, seed, maxval)
        src = xs + d
        inview = src < W
        lsrc = base + ys * W + np.minimum(src, W - 1)
        lv = _uniform(lsrc, seed, maxval)
        noise = _uniform(lidx, seed ^ 0x5EED5EED, 2) - 1
        fresh = _uniform(lidx, seed ^ 0x0FF5CE7E, maxval)
        r = np.where(inview, np.clip(lv + noise, 0, maxval), fresh)
        right[t] = r.astype(dtype)
    return left, right


def random_stack(n: int, H: int, W: int, dtype=np.uint8, seed: int = 1, maxval: int | None = None):
    """Unstructured U[0, maxval] planar stack (edge-case tests)."""
    maxval = (255 if np.dtype(dtype) == np.uint8 else 65535) if maxval is None else maxval
    idx = np.arange(n * H * W, dtype=np.int64)
    return _uniform(idx, seed, maxval).astype(dtype).reshape(n, H, W)
