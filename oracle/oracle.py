"""TEST INFRASTRUCTURE ONLY -- ctypes front-end for the C restatement in
bicos_oracle.c (the parity checker and the "port" CPU baseline).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module. The product path (libbicos_amd) never does.

Parity status: UNPINNED against the reference binary (see bicos_oracle.h).
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {}

NODUPES = 1
CONSISTENCY = 2


def build(quiet: bool = True) -> None:
    """Compile the oracle shared libraries (gcc; seconds)."""
    out = subprocess.run(["make", "-C", _HERE, "all"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


class _Cfg(ctypes.Structure):
    _fields_ = [
        ("has_nxcorr", ctypes.c_int), ("nxcorr_threshold", ctypes.c_float),
        ("has_step", ctypes.c_int), ("subpixel_step", ctypes.c_float),
        ("has_minvar", ctypes.c_int), ("min_variance", ctypes.c_float),
        ("mode", ctypes.c_int), ("variant", ctypes.c_int),
        ("max_lr_diff", ctypes.c_int), ("no_dupes", ctypes.c_int),
    ]


@dataclasses.dataclass
class OracleConfig:
    """Mirror of BICOS::Config (reference include/common.hpp:73-82)."""
    nxcorr_threshold: Optional[float] = 0.5
    subpixel_step: Optional[float] = None
    min_variance: Optional[float] = None
    mode: int = 0            # 0 LIMITED, 1 FULL
    variant: int = 0         # 0 NoDuplicates, 1 Consistency
    max_lr_diff: int = 1
    no_dupes: bool = False

    def to_c(self) -> _Cfg:
        return _Cfg(
            int(self.nxcorr_threshold is not None), float(self.nxcorr_threshold or 0.0),
            int(self.subpixel_step is not None), float(self.subpixel_step or 0.0),
            int(self.min_variance is not None), float(self.min_variance or 0.0),
            int(self.mode), int(self.variant), int(self.max_lr_diff), int(bool(self.no_dupes)))


def lib(variant: str = "") -> ctypes.CDLL:
    """variant "" = as-shipped flags, "v3" = -march=x86-64-v3 (identical results)."""
    name = "libbicos_oracle%s.so" % ("_" + variant if variant else "")
    if name in _LIBS:
        return _LIBS[name]
    path = os.path.join(_HERE, name)
    if not os.path.exists(path):
        build()
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    I = ctypes.c_int
    F = ctypes.c_float
    L.bicos_oracle_required_bits.argtypes = [I, I]
    L.bicos_oracle_desc_words.argtypes = [I, I]
    L.bicos_oracle_transform.argtypes = [P, I, I, I, I, I, I, P, I]
    L.bicos_oracle_transform.restype = None
    L.bicos_oracle_search.argtypes = [P, P, I, I, I, I, I, P, I]
    L.bicos_oracle_search.restype = None
    L.bicos_oracle_agree.argtypes = [P, P, P, I, I, I, I, F, I, F, P, I]
    L.bicos_oracle_agree.restype = None
    L.bicos_oracle_agree_subpixel.argtypes = [P, P, P, I, I, I, I, F, F, I, F, P, P, I]
    L.bicos_oracle_agree_subpixel.restype = None
    L.bicos_oracle_nxcorr.argtypes = [P, P, I, I, I, F]
    L.bicos_oracle_nxcorr.restype = F
    L.bicos_oracle_match.argtypes = [P, P, I, I, I, I, ctypes.POINTER(_Cfg), P, P, I]
    L.bicos_oracle_match.restype = I
    _LIBS[name] = L
    return L


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def _threads(nthreads: Optional[int]) -> int:
    return nthreads if nthreads else (os.cpu_count() or 1)


def _stack(stack) -> np.ndarray:
    s = np.ascontiguousarray(np.asarray(stack))
    assert s.ndim == 3 and s.dtype in (np.uint8, np.uint16), (s.shape, s.dtype)
    return s


def required_bits(n: int, mode: int) -> int:
    return lib().bicos_oracle_required_bits(n, mode)


def desc_words(n: int, mode: int) -> int:
    return lib().bicos_oracle_desc_words(n, mode)


def transform(stack, mode: int = 0, words: Optional[int] = None, nthreads=None) -> np.ndarray:
    """Planar [n,H,W] stack -> descriptors [H,W,words] uint32."""
    s = _stack(stack)
    n, h, w = s.shape
    words = words or desc_words(n, mode)
    out = np.zeros((h, w, words), np.uint32)
    lib().bicos_oracle_transform(_ptr(s), n, h, w, s.itemsize, mode, words, _ptr(out),
                                 _threads(nthreads))
    return out


def search(d0: np.ndarray, d1: np.ndarray, flags: int = NODUPES, max_lr_diff: int = -1,
           nthreads=None, variant: str = "") -> np.ndarray:
    d0 = np.ascontiguousarray(d0, np.uint32)
    d1 = np.ascontiguousarray(d1, np.uint32)
    h, w, words = d0.shape
    out = np.empty((h, w), np.int16)
    lib(variant).bicos_oracle_search(_ptr(d0), _ptr(d1), h, w, words, flags, max_lr_diff,
                                     _ptr(out), _threads(nthreads))
    return out


def agree(disp: np.ndarray, stack0, stack1, threshold: float, minvar_scaled: Optional[float],
          nthreads=None) -> Tuple[np.ndarray, np.ndarray]:
    s0, s1 = _stack(stack0), _stack(stack1)
    n, h, w = s0.shape
    d = np.array(disp, np.int16, copy=True, order="C")
    corr = np.full((h, w), np.nan, np.float32)
    lib().bicos_oracle_agree(_ptr(d), _ptr(s0), _ptr(s1), n, h, w, s0.itemsize, threshold,
                             int(minvar_scaled is not None), float(minvar_scaled or 0.0),
                             _ptr(corr), _threads(nthreads))
    return d, corr


def agree_subpixel(disp: np.ndarray, stack0, stack1, threshold: float, step: float,
                   minvar_scaled: Optional[float], nthreads=None) -> Tuple[np.ndarray, np.ndarray]:
    s0, s1 = _stack(stack0), _stack(stack1)
    n, h, w = s0.shape
    d = np.ascontiguousarray(disp, np.int16)
    out = np.empty((h, w), np.float32)
    corr = np.full((h, w), np.nan, np.float32)
    lib().bicos_oracle_agree_subpixel(_ptr(d), _ptr(s0), _ptr(s1), n, h, w, s0.itemsize,
                                      threshold, step, int(minvar_scaled is not None),
                                      float(minvar_scaled or 0.0), _ptr(out), _ptr(corr),
                                      _threads(nthreads))
    return out, corr


def nxcorr(pix0, pix1, minvar_scaled: Optional[float] = None) -> float:
    a = np.ascontiguousarray(pix0)
    b = np.ascontiguousarray(pix1, a.dtype)
    return lib().bicos_oracle_nxcorr(_ptr(a), _ptr(b), a.size, a.itemsize,
                                     int(minvar_scaled is not None), float(minvar_scaled or 0.0))


class OracleError(RuntimeError):
    pass


def match(stack0, stack1, cfg: Optional[OracleConfig] = None, nthreads=None,
          variant: str = "") -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """Full BICOS::match restated (reference src/impl/cpu.cpp:100-159).

    Returns (disparity, corrmap); disparity is int16 when no nxcorr threshold is
    set, float32 otherwise; corrmap is None when no nxcorr threshold is set."""
    cfg = cfg or OracleConfig()
    s0, s1 = _stack(stack0), _stack(stack1)
    n, h, w = s0.shape
    buf = np.empty((h, w), np.float32)
    corr = np.empty((h, w), np.float32)
    c = cfg.to_c()
    kind = lib(variant).bicos_oracle_match(_ptr(s0), _ptr(s1), n, h, w, s0.itemsize,
                                           ctypes.byref(c), _ptr(buf), _ptr(corr),
                                           _threads(nthreads))
    if kind < 0:
        raise OracleError({-1: "need at least two images", -2: "bad input depths",
                           -3: "input stacks too large"}[kind])
    if kind == 0:
        return buf.view(np.int16).reshape(-1)[: h * w].reshape(h, w).copy(), None
    return buf, corr
