"""Drop-in alias: `import pybicos` resolves to the MI355X engine's mirror of the
reference's Python API (reference pybicos/__init__.py)."""
from libbicos_amd.pybicos import (  # noqa: F401
    CV_8U, CV_16S, CV_16U, CV_32F, CV_64F, BicosConfig, BicosResult, Config, Precision,
    TransformMode, VariantType, invalid_disparity, match)
