"""Device-resident BICOS on MI355X: torch tensors in HBM -> libbicos_amd C-ABI.

This is the reference CUDA build's entry point (BICOS::match on cv::cuda::GpuMat
with a cv::cuda::Stream, reference include/match.hpp:31-41) for Python callers
that keep their stacks on the GPU. torch supplies device memory and the stream;
every kernel is hand-written HIP in libbicos_amd.so. There is no CPU fallback.

Stacks are planar tensors [n, rows, cols] (uint8, or uint16 held in an int16 /
uint16 tensor with depth=2), possibly a row band of a larger frame.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence, Tuple

import torch

from . import _lib

INVALID_I16 = -32768


@dataclasses.dataclass
class MatchConfig:
    """Python mirror of BICOS::Config (reference include/common.hpp:73-82)."""
    nxcorr_threshold: Optional[float] = 0.5
    subpixel_step: Optional[float] = None
    min_variance: Optional[float] = None
    mode: int = 0              # 0 LIMITED, 1 FULL
    precision: int = 0         # 0 SINGLE, 1 DOUBLE
    variant: int = 0           # 0 NoDuplicates, 1 Consistency
    max_lr_diff: int = 1
    no_dupes: bool = False

    def to_c(self) -> Tuple[_lib.BicosConfig, int]:
        thr = self.nxcorr_threshold
        if thr is not None and not thr >= 0:
            raise ValueError("device API: nxcorr_threshold must be >= 0 or None "
                             "(BicosConfig maps negatives to the 0.5 default)")
        c = _lib.BicosConfig(
            float(thr if thr is not None else 0.5),
            float(self.subpixel_step if self.subpixel_step is not None else -1.0),
            float(self.min_variance if self.min_variance is not None else -1.0),
            int(self.mode), int(self.precision), int(self.variant), int(self.max_lr_diff),
            int(bool(self.no_dupes)))
        return c, int(thr is not None)


def _depth(t: torch.Tensor) -> int:
    if t.dtype == torch.uint8:
        return 1
    if t.dtype in (torch.int16, getattr(torch, "uint16", torch.int16)):
        return 2
    raise TypeError("stack dtype must be uint8 or (u)int16, got %s" % t.dtype)


def _check_stack(t: torch.Tensor):
    if not t.is_cuda:
        raise ValueError("device API needs CUDA/HIP tensors")
    if t.dim() != 3:
        raise ValueError("stack must be [n, rows, cols]")
    if t.stride(2) != 1:
        raise ValueError("stack rows must be contiguous")
    return t.shape[0], t.shape[1], t.shape[2], t.stride(1), t.stride(0)


def _check_out(t: torch.Tensor, name: str, shape, dtypes, device: torch.device) -> None:
    """The kernels write rows*cols elements of the dtype the config implies straight through
    the tensor's pointer: anything else would be an out-of-bounds HBM write."""
    if t.device != device:
        raise ValueError("%s must be on %s, got %s" % (name, device, t.device))
    if tuple(t.shape) != tuple(shape):
        raise ValueError("%s must have shape %s, got %s" % (name, tuple(shape), tuple(t.shape)))
    if t.dtype not in dtypes:
        raise ValueError("%s must be %s for this config, got %s"
                         % (name, " or ".join(str(d) for d in dtypes), t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous (dense rows)" % name)


def _stream(device: torch.device, stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return s.cuda_stream


class Engine:
    """One bicos_engine (workspace + stream-agnostic launcher) per device."""

    def __init__(self, device=None, shared: bool = False):
        """shared=True wraps the library's process-wide engine for the device (the one
        BICOS_Match / pybicos.match use) instead of creating a private one."""
        if not torch.cuda.is_available():
            raise RuntimeError("libbicos_amd device engine needs a ROCm GPU")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        self._L = _lib.lib()
        self._owned = not shared
        if shared:
            h = ctypes.c_void_p(self._L.bicos_engine_default(self.device.index))
            if not h.value:
                _lib.check(-5, "bicos_engine_default")
        else:
            h = ctypes.c_void_p()
            _lib.check(self._L.bicos_engine_create(self.device.index, ctypes.byref(h)),
                       "bicos_engine_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) and self._owned:
            torch.cuda.synchronize(self.device)
            self._L.bicos_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tune(self, variant: int = 0, col0_per_lane: int = 0, waves: int = 0,
             split: int = 0) -> None:
        """Search-kernel variant / register blocking / waves / col1 split (0 = automatic)."""
        _lib.check(self._L.bicos_engine_tune(self._h, variant, col0_per_lane, waves, split),
                   "bicos_engine_tune")

    # ------------------------------------------------------------------ match
    def match(self, stack0: torch.Tensor, stack1: torch.Tensor,
              cfg: Optional[MatchConfig] = None, want_corrmap: bool = True,
              out: Optional[torch.Tensor] = None, corrmap: Optional[torch.Tensor] = None,
              stream=None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Full BICOS::match on device stacks. Returns (disparity, corrmap) on the
        device; asynchronous on `stream` (default: torch's current stream).

        With the NXC stage and no subpixel step, `out` may also be an int16 tensor: the
        integer disparity map (bicos_match_device_i16), whose float32 conversion is exactly
        the float map -- half the bytes, e.g. for a row band that is gathered elsewhere."""
        cfg = cfg or MatchConfig()
        n, rows, cols, rp, pp = _check_stack(stack0)
        if tuple(stack1.shape) != (n, rows, cols) or stack1.stride() != stack0.stride() or \
                stack1.dtype != stack0.dtype:
            raise ValueError("stack1 must match stack0 in shape, strides and dtype")
        c, has_nxcorr = cfg.to_c()
        dev = stack0.device
        disp_dtype = torch.float32 if has_nxcorr else torch.int16
        corr_dtype = torch.float64 if cfg.precision else torch.float32
        i16 = (out is not None and has_nxcorr and out.dtype == torch.int16 and
               cfg.subpixel_step is None)
        if i16:
            disp_dtype = torch.int16
        if out is None:
            out = torch.empty((rows, cols), dtype=disp_dtype, device=dev)
        _check_out(out, "out", (rows, cols), (disp_dtype,), dev)
        if has_nxcorr and want_corrmap and corrmap is None:
            corrmap = torch.empty((rows, cols), device=dev, dtype=corr_dtype)
        if not (has_nxcorr and want_corrmap):
            corrmap = None
        if corrmap is not None:
            _check_out(corrmap, "corrmap", (rows, cols), (corr_dtype,), dev)
        entry = self._L.bicos_match_device_i16 if i16 else self._L.bicos_match_device
        rc = entry(
            self._h, stack0.data_ptr(), stack1.data_ptr(), n, rows, cols, rp, pp, _depth(stack0),
            ctypes.byref(c), has_nxcorr, out.data_ptr(),
            corrmap.data_ptr() if corrmap is not None else None, _stream(dev, stream))
        _lib.check(rc, "bicos_match_device")
        return out, corrmap

    def plan(self, stack0: torch.Tensor, stack1: torch.Tensor,
             cfg: Optional[MatchConfig] = None) -> int:
        """bicos_match_plan: the _lib.PLAN_* bits of what match() runs past the transform for
        these stacks and this config (fused launches, packed keys, compacted reverse search)."""
        cfg = cfg or MatchConfig()
        n, rows, cols, rp, pp = _check_stack(stack0)
        c, has_nxcorr = cfg.to_c()
        rc = self._L.bicos_match_plan(self._h, stack0.data_ptr(), stack1.data_ptr(), n, rows, cols,
                                      rp, pp, _depth(stack0), ctypes.byref(c), has_nxcorr)
        if rc < 0:
            _lib.check(rc, "bicos_match_plan")
        return rc

    def search_agree(self, desc0: torch.Tensor, desc1: torch.Tensor, stack0: torch.Tensor,
                     stack1: torch.Tensor, cfg: Optional[MatchConfig] = None,
                     out: Optional[torch.Tensor] = None, corrmap: Optional[torch.Tensor] = None,
                     stream=None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """bicos_search_agree_device: match() from its search on, over descriptors from
        transform() of the two stacks -- the very launches match() issues after its
        transform (bench.py times them in the frame)."""
        cfg = cfg or MatchConfig()
        n, rows, cols, rp, pp = _check_stack(stack0)
        if tuple(stack1.shape) != (n, rows, cols) or stack1.stride() != stack0.stride() or \
                stack1.dtype != stack0.dtype:
            raise ValueError("stack1 must match stack0 in shape, strides and dtype")
        words = descriptor_words(n, cfg.mode)
        pitch = self._L.bicos_desc_pitch(cols, words)
        for name, d in (("desc0", desc0), ("desc1", desc1)):
            if d.device != stack0.device or d.dtype != torch.int32 or not d.is_contiguous() or \
                    tuple(d.shape) != (rows, pitch):
                raise ValueError("%s must be a contiguous int32 [%d, %d] tensor on %s"
                                 % (name, rows, pitch, stack0.device))
        c, has_nxcorr = cfg.to_c()
        dev = stack0.device
        disp_dtype = torch.float32 if has_nxcorr else torch.int16
        corr_dtype = torch.float64 if cfg.precision else torch.float32
        if out is None:
            out = torch.empty((rows, cols), dtype=disp_dtype, device=dev)
        _check_out(out, "out", (rows, cols), (disp_dtype,), dev)
        if has_nxcorr and corrmap is None:
            corrmap = torch.empty((rows, cols), device=dev, dtype=corr_dtype)
        if not has_nxcorr:
            corrmap = None
        if corrmap is not None:
            _check_out(corrmap, "corrmap", (rows, cols), (corr_dtype,), dev)
        rc = self._L.bicos_search_agree_device(
            self._h, desc0.data_ptr(), desc1.data_ptr(), stack0.data_ptr(), stack1.data_ptr(),
            n, rows, cols, rp, pp, _depth(stack0), ctypes.byref(c), has_nxcorr, out.data_ptr(),
            corrmap.data_ptr() if corrmap is not None else None, _stream(dev, stream))
        _lib.check(rc, "bicos_search_agree_device")
        return out, corrmap

    # ----------------------------------------------------------------- stages
    def transform(self, stack: torch.Tensor, mode: int = 0, words: Optional[int] = None,
                  out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Descriptors as int32 [rows, desc_pitch] (uint32 bit patterns)."""
        n, rows, cols, rp, pp = _check_stack(stack)
        words = words or descriptor_words(n, mode)
        pitch = self._L.bicos_desc_pitch(cols, words)
        if out is None:
            out = torch.empty((rows, pitch), dtype=torch.int32, device=stack.device)
        _check_out(out, "out", (rows, pitch), (torch.int32,), stack.device)
        rc = self._L.bicos_transform_device(stack.data_ptr(), n, rows, cols, rp, pp,
                                            _depth(stack), mode, words, out.data_ptr(),
                                            _stream(stack.device, stream))
        _lib.check(rc, "bicos_transform_device")
        return out

    def search(self, desc0: torch.Tensor, desc1: torch.Tensor, cols: int, words: int,
               flags: int = 1, max_lr_diff: int = -1, out: Optional[torch.Tensor] = None,
               stream=None, bits: int = 0) -> torch.Tensor:
        """bits: how many low descriptor bits may be set (0 = all; see used_bits) -- the
        matrix-core search skips the K-steps above them (bicos_c.h flags bits 16-24)."""
        if not 0 <= bits <= 256:
            raise ValueError("bits must be in [0, 256]")
        flags = (flags & 0xFFFF) | (bits << 16)
        rows = desc0.shape[0]
        pitch = self._L.bicos_desc_pitch(cols, words)
        for name, d in (("desc0", desc0), ("desc1", desc1)):
            if d.device != desc0.device or d.dtype != torch.int32 or not d.is_contiguous() or \
                    d.dim() != 2 or tuple(d.shape) != (rows, pitch):
                raise ValueError("%s must be a contiguous int32 [%d, %d] tensor on %s "
                                 "(bicos_desc_pitch)" % (name, rows, pitch, desc0.device))
        if out is None:
            out = torch.empty((rows, cols), dtype=torch.int16, device=desc0.device)
        _check_out(out, "out", (rows, cols), (torch.int16,), desc0.device)
        rc = self._L.bicos_search_device(self._h, desc0.data_ptr(), desc1.data_ptr(), rows, cols,
                                         words, flags, max_lr_diff, out.data_ptr(),
                                         _stream(desc0.device, stream))
        _lib.check(rc, "bicos_search_device")
        return out

    def agree(self, raw: torch.Tensor, stack0: torch.Tensor, stack1: torch.Tensor,
              threshold: float, minvar_scaled: Optional[float] = None,
              step: Optional[float] = None, stream=None, precision: int = 0
              ) -> Tuple[torch.Tensor, torch.Tensor]:
        """NXC agree (step None) or subpixel refine of an int16 search result -> (float32
        disparity, corrmap float32 / float64 with precision=1)."""
        if step is not None and not step > 0:
            raise ValueError("subpixel step must be positive")
        n, rows, cols, rp, pp = _check_stack(stack0)
        out = torch.empty((rows, cols), dtype=torch.float32, device=stack0.device)
        corr = torch.empty((rows, cols), dtype=torch.float64 if precision else torch.float32,
                           device=stack0.device)
        hm = int(minvar_scaled is not None)
        mv = float(minvar_scaled or 0.0)
        st = _stream(stack0.device, stream)
        rc = self._L.bicos_agree_stage_device(raw.data_ptr(), stack0.data_ptr(),
                                              stack1.data_ptr(), n, rows, cols, rp, pp,
                                              _depth(stack0), threshold,
                                              -1.0 if step is None else step, hm, mv,
                                              int(bool(precision)), out.data_ptr(),
                                              corr.data_ptr(), st)
        _lib.check(rc, "bicos_agree_stage_device")
        return out, corr


def used_bits(n: int, mode: int = 0) -> int:
    """Upper bound of the descriptor bits the transform sets (LIMITED 4n-6 for n >= 4, 7 for
    n = 3, 4 for n = 2 (descriptor_transform.hpp:62-68 alone); FULL n^2-2n+3; reference
    descriptor_transform.hpp:31-123)."""
    return n * n - 2 * n + 3 if mode else max(4 * n - 5, 4)


def descriptor_words(n: int, mode: int = 0) -> int:
    w = _lib.lib().bicos_descriptor_words(n, mode)
    if w < 0:
        _lib.check(w, "bicos_descriptor_words")
    return w


_ENGINES = {}


def default_engine(device=None) -> Engine:
    idx = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    if idx not in _ENGINES:
        _ENGINES[idx] = Engine(idx, shared=True)
    return _ENGINES[idx]


def match_bands(bands0: Sequence[torch.Tensor], bands1: Sequence[torch.Tensor],
                cfg: Optional[MatchConfig] = None, want_corrmap: bool = True
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Single-process multi-GPU match (bicos_match_bands_device):
    bands0[b] / bands1[b] are the planar stacks [n, rows_b, cols] of row band b (bands in
    frame order), each on the GPU that matches it. Returns the whole frame's (disparity,
    corrmap) on bands0[0]'s device, gathered there by peer copies. Synchronous: the work
    queued on every band device's current stream is finished first."""
    cfg = cfg or MatchConfig()
    if len(bands0) == 0 or len(bands0) != len(bands1):
        raise ValueError("need the same number (>= 1) of left and right bands")
    k = len(bands0)
    shapes = [_check_stack(t) for t in bands0]
    n, _, cols, _, _ = shapes[0]
    for b in range(k):
        t0, t1 = bands0[b], bands1[b]
        if t0.shape[0] != n or t0.shape[2] != cols or t0.dtype != bands0[0].dtype:
            raise ValueError("every band needs the same n, cols and dtype")
        if tuple(t1.shape) != tuple(t0.shape) or t1.stride() != t0.stride() or \
                t1.dtype != t0.dtype or t1.device != t0.device:
            raise ValueError("bands1[%d] must match bands0[%d] in shape, strides, dtype, device"
                             % (b, b))
    c, has_nxcorr = cfg.to_c()
    root = bands0[0].device
    rows = sum(int(t.shape[1]) for t in bands0)
    disp_dtype = torch.float32 if has_nxcorr else torch.int16
    corr_dtype = torch.float64 if cfg.precision else torch.float32
    out = torch.empty((rows, cols), dtype=disp_dtype, device=root)
    corrmap = torch.empty((rows, cols), dtype=corr_dtype, device=root) \
        if has_nxcorr and want_corrmap else None
    for dev in {t.device for t in bands0} | {root}:
        torch.cuda.synchronize(dev)
    devs = (ctypes.c_int * k)(*[t.device.index or 0 for t in bands0])
    p0 = (ctypes.c_void_p * k)(*[t.data_ptr() for t in bands0])
    p1 = (ctypes.c_void_p * k)(*[t.data_ptr() for t in bands1])
    br = (ctypes.c_int * k)(*[int(t.shape[1]) for t in bands0])
    rp = (ctypes.c_size_t * k)(*[s[3] for s in shapes])
    pp = (ctypes.c_size_t * k)(*[s[4] for s in shapes])
    rc = _lib.lib().bicos_match_bands_device(
        devs, k, p0, p1, br, rp, pp, n, cols, _depth(bands0[0]), ctypes.byref(c), has_nxcorr,
        out.data_ptr(), corrmap.data_ptr() if corrmap is not None else None)
    _lib.check(rc, "bicos_match_bands_device")
    return out, corrmap


def match(stack0: torch.Tensor, stack1: torch.Tensor, cfg: Optional[MatchConfig] = None,
          **kw) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Module-level convenience: BICOS::match on device tensors."""
    return default_engine(stack0.device).match(stack0, stack1, cfg, **kw)
