"""ctypes binding of libbicos_amd.so (include/bicos_c.h).

The product path has exactly one implementation: the gfx950 HIP engine in this
shared library. There is no CPU fallback -- if the library is missing or fails
to load, importing the package's compute entry points raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbicos_amd.so")
CSRC = os.path.join(_HERE, "csrc")

BICOS_OK = 0
BICOS_E_ARG = -1
BICOS_E_BITS = -2
BICOS_E_HIP = -3
BICOS_E_INTERNAL = -4

CV_8U, CV_16U, CV_16S, CV_32F, CV_64F = 0, 2, 3, 5, 6


class BicosConfig(ctypes.Structure):
    """reference src/pybicos_c.cpp:30-41, with `precision` always present."""
    _fields_ = [
        ("nxcorr_threshold", ctypes.c_float),
        ("subpixel_step", ctypes.c_float),
        ("min_variance", ctypes.c_float),
        ("mode", ctypes.c_int),
        ("precision", ctypes.c_int),
        ("variant_type", ctypes.c_int),
        ("max_lr_diff", ctypes.c_int),
        ("no_dupes", ctypes.c_int),
    ]


class BicosResult(ctypes.Structure):
    """reference src/pybicos_c.cpp:44-53."""
    _fields_ = [
        ("disparity_data", ctypes.c_void_p),
        ("disparity_rows", ctypes.c_int),
        ("disparity_cols", ctypes.c_int),
        ("disparity_type", ctypes.c_int),
        ("corrmap_data", ctypes.c_void_p),
        ("corrmap_rows", ctypes.c_int),
        ("corrmap_cols", ctypes.c_int),
        ("corrmap_type", ctypes.c_int),
    ]


# every symbol include/bicos_c.h declares (tests check the .so exports them all)
EXPORTS = (
    "BICOS_CreateDefaultConfig", "BICOS_FreeConfig", "BICOS_FreeResult", "BICOS_Match",
    "BICOS_InvalidDisparityFloat", "BICOS_InvalidDisparityInt16", "bicos_last_error",
    "bicos_engine_create", "bicos_engine_default", "bicos_engine_destroy", "bicos_engine_tune", "bicos_descriptor_words", "bicos_output_type",
    "bicos_match_device", "bicos_match_device_i16", "bicos_match_host", "bicos_match_host_multi", "bicos_match_bands_device",
    "bicos_desc_pitch", "bicos_transform_device", "bicos_search_device",
    "bicos_agree_device", "bicos_subpixel_device", "bicos_agree_stage_device", "bicos_build_info",
    "bicos_match_plan", "bicos_search_agree_device",
)

# bicos_match_plan bits (include/bicos_c.h)
PLAN_MATRIX_CORES = 1
PLAN_PACKED_KEYS = 2
PLAN_AGREE_IN_SEARCH = 4
PLAN_REVERSE_COMPACTED = 8
PLAN_CONSISTENCY_IN_AGREE = 16
PLAN_DENSE_ROWS = 32
PLAN_CONSISTENCY_ONE_PASS = 64


def build(verbose: bool = False, jobs: int = 4) -> str:
    """Compile libbicos_amd.so for gfx950 with hipcc (in-tree)."""
    out = subprocess.run(["make", "-C", CSRC, "-j%d" % jobs, "all"], capture_output=True,
                         text=True)
    if verbose:
        print(out.stdout, out.stderr)
    if out.returncode != 0:
        raise RuntimeError("libbicos_amd build failed:\n" + out.stdout[-4000:] + out.stderr[-4000:])
    return LIB_PATH


_lib = None


class BicosError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libbicos_amd.so not built at %s -- run libbicos_amd._lib.build() "
                          "(hipcc, gfx950)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, I, F, Z = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    PI = ctypes.POINTER(ctypes.c_int)
    PP = ctypes.POINTER(ctypes.c_void_p)
    L.BICOS_CreateDefaultConfig.restype = ctypes.POINTER(BicosConfig)
    L.BICOS_CreateDefaultConfig.argtypes = []
    L.BICOS_FreeConfig.argtypes = [ctypes.POINTER(BicosConfig)]
    L.BICOS_FreeConfig.restype = None
    L.BICOS_FreeResult.argtypes = [ctypes.POINTER(BicosResult)]
    L.BICOS_FreeResult.restype = None
    L.BICOS_Match.argtypes = [PP, PI, PI, PI, I, PP, PI, PI, PI, I, ctypes.POINTER(BicosConfig)]
    L.BICOS_Match.restype = ctypes.POINTER(BicosResult)
    L.BICOS_InvalidDisparityFloat.restype = F
    L.BICOS_InvalidDisparityFloat.argtypes = []
    L.BICOS_InvalidDisparityInt16.restype = ctypes.c_int16
    L.BICOS_InvalidDisparityInt16.argtypes = []
    L.bicos_last_error.restype = ctypes.c_char_p
    L.bicos_last_error.argtypes = []
    L.bicos_engine_create.argtypes = [I, ctypes.POINTER(P)]
    L.bicos_engine_create.restype = I
    L.bicos_engine_default.argtypes = [I]
    L.bicos_engine_default.restype = P
    L.bicos_engine_destroy.argtypes = [P]
    L.bicos_engine_destroy.restype = None
    L.bicos_engine_tune.argtypes = [P, I, I, I, I]
    L.bicos_engine_tune.restype = I
    L.bicos_descriptor_words.argtypes = [I, I]
    L.bicos_descriptor_words.restype = I
    L.bicos_output_type.argtypes = [ctypes.POINTER(BicosConfig), I]
    L.bicos_output_type.restype = I
    L.bicos_match_device.argtypes = [P, P, P, I, I, I, Z, Z, I, ctypes.POINTER(BicosConfig), I,
                                     P, P, P]
    L.bicos_match_device.restype = I
    L.bicos_match_device_i16.argtypes = L.bicos_match_device.argtypes
    L.bicos_match_device_i16.restype = I
    L.bicos_match_host.argtypes = [P, PP, PP, I, I, I, Z, I, ctypes.POINTER(BicosConfig), I, P, P]
    L.bicos_match_host.restype = I
    PZ = ctypes.POINTER(ctypes.c_size_t)
    L.bicos_match_host_multi.argtypes = [PI, I, PP, PP, I, I, I, Z, I,
                                         ctypes.POINTER(BicosConfig), I, P, P]
    L.bicos_match_host_multi.restype = I
    L.bicos_match_bands_device.argtypes = [PI, I, PP, PP, PI, PZ, PZ, I, I, I,
                                           ctypes.POINTER(BicosConfig), I, P, P]
    L.bicos_match_bands_device.restype = I
    L.bicos_desc_pitch.argtypes = [I, I]
    L.bicos_desc_pitch.restype = Z
    L.bicos_transform_device.argtypes = [P, I, I, I, Z, Z, I, I, I, P, P]
    L.bicos_transform_device.restype = I
    L.bicos_search_device.argtypes = [P, P, P, I, I, I, I, I, P, P]
    L.bicos_search_device.restype = I
    L.bicos_agree_device.argtypes = [P, P, P, I, I, I, Z, Z, I, F, I, F, P, P, P]
    L.bicos_agree_device.restype = I
    L.bicos_subpixel_device.argtypes = [P, P, P, I, I, I, Z, Z, I, F, F, I, F, P, P, P]
    L.bicos_subpixel_device.restype = I
    L.bicos_agree_stage_device.argtypes = [P, P, P, I, I, I, Z, Z, I, F, F, I, F, I, P, P, P]
    L.bicos_agree_stage_device.restype = I
    L.bicos_match_plan.argtypes = [P, P, P, I, I, I, Z, Z, I, ctypes.POINTER(BicosConfig), I]
    L.bicos_match_plan.restype = I
    L.bicos_search_agree_device.argtypes = [P, P, P, P, P, I, I, I, Z, Z, I,
                                            ctypes.POINTER(BicosConfig), I, P, P, P]
    L.bicos_search_agree_device.restype = I
    L.bicos_build_info.restype = ctypes.c_char_p
    L.bicos_build_info.argtypes = []
    _lib = L
    return L


def check(rc: int, what: str = "bicos") -> None:
    if rc != BICOS_OK:
        msg = lib().bicos_last_error().decode(errors="replace")
        raise BicosError("%s failed (%d): %s" % (what, rc, msg))
