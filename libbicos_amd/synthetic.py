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


def random_descriptors(H: int, W: int, words: int, seed: int = SEED, period: int | None = None,
                       row_begin: int = 0, row_end: int | None = None) -> np.ndarray:
    """[rows, W, words] uint32 descriptor words for rows [row_begin, row_end) of an H x W
    frame: word k of pixel (y, x) is the low half of splitmix64((y W + x') words + k), with
    x' = x % period when a period is given (every minimum of a search then repeats W / period
    times). The reference's search kernel-bench feeds random descriptors the same way
    (bench/cuda.cu:182-256, cv::randu over the descriptor bytes)."""
    row_end = H if row_end is None else row_end
    ys = np.arange(row_begin, row_end, dtype=np.int64)[:, None, None]
    xs = np.arange(W, dtype=np.int64)[None, :, None]
    if period:
        xs = xs % period
    ks = np.arange(words, dtype=np.int64)[None, None, :]
    return (splitmix64((ys * W + xs) * words + ks, seed) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def low_texture_stack(n: int, H: int, W: int, shift: int = 0, noise_seed: int = 1,
                      seed: int = SEED ^ 0x10, run: int = 4, row_begin: int = 0,
                      row_end: int | None = None) -> np.ndarray:
    """u8 planar stack of a weakly textured scene: 8 grey levels (32 apart) constant over runs
    of `run` columns, plus independent U{0,1,2} sensor noise per pixel (`noise_seed`). The
    right view is the same scene moved by `shift` columns with its own noise. Neighbouring
    columns then have near-identical descriptors, so duplicate and tied minima decide many
    pixels (NoDuplicates keeps ~71 % at run 4, NoDuplicates|Consistency ~52 %)."""
    row_end = H if row_end is None else row_end
    rows = row_end - row_begin
    out = np.empty((n, rows, W), np.uint8)
    runs = (W - 1 + shift) // run + 1
    cols = (np.arange(W, dtype=np.int64) + shift) // run
    for t in range(n):
        # level of run c of row y: top 3 bits of splitmix64((t H + y) W + c)
        ys = np.arange(row_begin, row_end, dtype=np.int64)[:, None]
        lv = splitmix64((t * H + ys) * W + np.arange(runs, dtype=np.int64)[None, :], seed)
        level = (lv >> np.uint64(61)).astype(np.uint8)[:, cols]
        # noise of pixel i = (t H + y) W + x: byte i % 8 of splitmix64(i // 8), mod 3
        start = (t * H + row_begin) * W
        c0, c1 = start >> 3, (start + rows * W - 1) >> 3
        raw = splitmix64(np.arange(c0, c1 + 1, dtype=np.int64), noise_seed).view(np.uint8)
        noise = raw[start - (c0 << 3): start - (c0 << 3) + rows * W] % np.uint8(3)
        out[t] = level * np.uint8(32) + noise.reshape(rows, W)
    return out
