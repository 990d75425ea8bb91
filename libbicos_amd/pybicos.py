"""pybicos -- drop-in for the reference's Python API (pybicos/__init__.py:1-252).

Same names, argument meaning, return dtypes and error behaviour:
  Config() with nxcorr_threshold / subpixel_step / min_variance / mode /
  precision properties, variant (read-only), set_no_duplicates(),
  set_consistency(max_lr_diff=1, no_dupes=False);
  match(stack0, stack1, cfg=None) -> (disparity, corrmap) numpy copies;
  invalid_disparity(dtype).
Backed by libbicos_amd.so's BICOS_Match (host buffers in, host copies out),
which runs on the gfx950 HIP engine.
"""
from __future__ import annotations

import ctypes
from enum import Enum

import numpy as np

from . import _lib
from ._lib import BicosConfig, BicosResult  # noqa: F401  (re-exported like the reference)

CV_8U, CV_16U, CV_16S, CV_32F, CV_64F = 0, 2, 3, 5, 6


class TransformMode(Enum):
    LIMITED = 0
    FULL = 1


class Precision(Enum):
    SINGLE = 0
    DOUBLE = 1


class VariantType(Enum):
    NO_DUPLICATES = 0
    CONSISTENCY = 1


def _get_cv_type(dtype):
    # reference pybicos/__init__.py:85-97
    if dtype == np.uint8:
        return CV_8U
    elif dtype == np.uint16:
        return CV_16U
    elif dtype == np.int16:
        return CV_16S
    elif dtype == np.float32:
        return CV_32F
    elif dtype == np.float64:
        return CV_64F
    raise ValueError(f"Unsupported numpy dtype: {dtype}")


def _get_np_dtype(cv_type):
    # reference pybicos/__init__.py:99-107
    if cv_type == CV_16S or cv_type == (CV_16S | (1 << 3)):
        return np.int16
    elif cv_type == CV_32F or cv_type == (CV_32F | (1 << 3)):
        return np.float32
    elif cv_type == CV_64F or cv_type == (CV_64F | (1 << 3)):
        return np.float64
    raise ValueError(f"Unsupported OpenCV type: {cv_type}")


class Config:
    """reference pybicos/__init__.py:110-196."""

    def __init__(self):
        self._L = _lib.lib()
        self._c_config = self._L.BICOS_CreateDefaultConfig()

    def __del__(self):
        if getattr(self, "_c_config", None):
            self._L.BICOS_FreeConfig(self._c_config)
            self._c_config = None

    @property
    def nxcorr_threshold(self):
        return self._c_config.contents.nxcorr_threshold

    @nxcorr_threshold.setter
    def nxcorr_threshold(self, value):
        self._c_config.contents.nxcorr_threshold = value

    @property
    def subpixel_step(self):
        val = self._c_config.contents.subpixel_step
        return None if val < 0 else val

    @subpixel_step.setter
    def subpixel_step(self, value):
        self._c_config.contents.subpixel_step = -1.0 if value is None else value

    @property
    def min_variance(self):
        val = self._c_config.contents.min_variance
        return None if val < 0 else val

    @min_variance.setter
    def min_variance(self, value):
        self._c_config.contents.min_variance = -1.0 if value is None else value

    @property
    def mode(self):
        return TransformMode(self._c_config.contents.mode)

    @mode.setter
    def mode(self, value):
        self._c_config.contents.mode = value.value if isinstance(value, TransformMode) else value

    @property
    def precision(self):
        return Precision(self._c_config.contents.precision)

    @precision.setter
    def precision(self, value):
        self._c_config.contents.precision = value.value if isinstance(value, Precision) else value

    @property
    def variant(self):
        if self._c_config.contents.variant_type == VariantType.NO_DUPLICATES.value:
            return "NoDuplicates"
        return {
            "type": "Consistency",
            "max_lr_diff": self._c_config.contents.max_lr_diff,
            "no_dupes": bool(self._c_config.contents.no_dupes),
        }

    def set_no_duplicates(self):
        self._c_config.contents.variant_type = VariantType.NO_DUPLICATES.value

    def set_consistency(self, max_lr_diff=1, no_dupes=False):
        self._c_config.contents.variant_type = VariantType.CONSISTENCY.value
        self._c_config.contents.max_lr_diff = max_lr_diff
        self._c_config.contents.no_dupes = 1 if no_dupes else 0

    def __repr__(self):
        parts = [
            "Config(",
            f"  nxcorr_threshold={self.nxcorr_threshold}",
            f"  subpixel_step={self.subpixel_step}",
            f"  min_variance={self.min_variance}",
            f"  mode={self.mode.name}",
            f"  precision={self.precision.name}",
            f"  variant={self.variant}",
            ")",
        ]
        return "\n".join(parts)


def _marshal(stack):
    k = len(stack)
    data = (ctypes.c_void_p * k)()
    rows = (ctypes.c_int * k)()
    cols = (ctypes.c_int * k)()
    types = (ctypes.c_int * k)()
    keep = []
    for i, img in enumerate(stack):
        img = np.asarray(img)
        if not img.flags["C_CONTIGUOUS"]:
            img = np.ascontiguousarray(img)
        if img.ndim != 2:
            raise ValueError("images must be 2-D (single channel)")
        keep.append(img)
        data[i] = img.ctypes.data_as(ctypes.c_void_p)
        rows[i] = img.shape[0]
        cols[i] = img.shape[1]
        types[i] = _get_cv_type(img.dtype)
    return data, rows, cols, types, keep


def match(stack0, stack1, cfg=None, devices=None):
    """reference pybicos/__init__.py:199-244 -> (disparity, corrmap).

    devices (an extension; the reference is single-GPU): a sequence of GPU indices to split
    the frame's rows over from this process (bicos_match_host_multi: one band per device,
    each uploaded over its own GPU's link); the maps are byte-identical to the one-GPU call.

    Same inputs, outputs, dtypes and errors as the reference wrapper (which goes through
    BICOS_Match: NXC always on, so float32 disparity; corrmap float32, or float64 with
    Precision.DOUBLE). Runs bicos_match_host, which writes the maps straight into the
    returned arrays (no result struct, no extra copies) and overlaps the upload of the
    stacks with the match (include/bicos_c.h)."""
    if stack0 is None or stack1 is None or len(stack0) == 0 or len(stack1) == 0:
        raise ValueError("Empty image stacks")
    if cfg is None:
        cfg = Config()
    L = _lib.lib()
    d0, r0, c0, t0, k0 = _marshal(stack0)
    d1, r1, c1, t1, k1 = _marshal(stack1)
    f = k0[0]
    if len(k0) != len(k1) or any(a.shape != f.shape or a.dtype != f.dtype for a in k0 + k1):
        raise RuntimeError("BICOS matching failed: all images must share size and type "
                           "(and both stacks the same length)")
    rows, cols = f.shape
    ddtype = _get_np_dtype(L.bicos_output_type(cfg._c_config, 1))
    cdtype = np.float64 if cfg._c_config.contents.precision else np.float32
    disparity = np.empty((rows, cols), ddtype)
    corrmap = np.empty((rows, cols), cdtype)
    if devices is None:
        rc = L.bicos_match_host(None, d0, d1, len(k0), rows, cols, 0, f.dtype.itemsize,
                                cfg._c_config, 1, disparity.ctypes.data, corrmap.ctypes.data)
    else:
        devs = [int(d) for d in devices]
        if not devs:
            raise ValueError("devices must name at least one GPU")
        rc = L.bicos_match_host_multi((ctypes.c_int * len(devs))(*devs), len(devs), d0, d1,
                                      len(k0), rows, cols, 0, f.dtype.itemsize, cfg._c_config, 1,
                                      disparity.ctypes.data, corrmap.ctypes.data)
    del k0, k1
    if rc != 0:
        raise RuntimeError("BICOS matching failed: " + L.bicos_last_error().decode(errors="replace"))
    return disparity, corrmap


def invalid_disparity(dtype):
    """reference pybicos/__init__.py:246-252."""
    L = _lib.lib()
    if dtype == np.float32:
        return L.BICOS_InvalidDisparityFloat()
    elif dtype == np.int16:
        return L.BICOS_InvalidDisparityInt16()
    raise ValueError(f"Unsupported dtype for invalid_disparity: {dtype}")
