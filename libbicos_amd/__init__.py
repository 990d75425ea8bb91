"""libbicos_amd -- MI355X (gfx950) BICOS correspondence engine.

Drop-in for nexus1203/libBICOS's hot path (BICOS::match / pybicos.match) with
hand-written HIP kernels behind a C-ABI shared library (libbicos_amd.so,
include/bicos_c.h). Submodules:
  pybicos      reference-compatible Python API (host numpy in, numpy out)
  device       device-resident API on torch tensors (the measured path)
  distributed  row-band sharding across GPUs + RCCL gather
  synthetic    deterministic synthetic stereo stacks
"""
from ._lib import BicosError, build  # noqa: F401

__all__ = ["BicosError", "build", "pybicos", "device", "distributed", "synthetic"]
