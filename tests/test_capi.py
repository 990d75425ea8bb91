"""CPU tests of the C-ABI boundary (no compute without a GPU)."""
import ctypes
import os
import re
import shutil
import sys
import importlib.util

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "bicos_c.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src)
    skip = {"if", "sizeof", "defined", "extern"}
    return sorted({n for n in names if n not in skip and (n.startswith("BICOS_") or n.startswith("bicos_"))})


def test_library_exports_every_declared_symbol(blib):
    declared = _declared_functions()
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(blib, name), name
    from libbicos_amd import _lib
    assert set(_lib.EXPORTS) == set(declared)


def test_struct_layouts():
    from libbicos_amd._lib import BicosConfig, BicosResult
    # reference src/pybicos_c.cpp:30-53 with `precision` (the Python wrapper's layout)
    assert ctypes.sizeof(BicosConfig) == 32
    assert [f[0] for f in BicosConfig._fields_] == [
        "nxcorr_threshold", "subpixel_step", "min_variance", "mode", "precision",
        "variant_type", "max_lr_diff", "no_dupes"]
    assert ctypes.sizeof(BicosResult) == 48  # void*, 3 ints, pad, void*, 3 ints, pad
    assert BicosResult.corrmap_data.offset == 24


def test_default_config(blib):
    c = blib.BICOS_CreateDefaultConfig()
    v = c.contents
    assert (v.nxcorr_threshold, v.subpixel_step, v.min_variance) == (0.5, -1.0, -1.0)
    assert (v.mode, v.precision, v.variant_type, v.max_lr_diff, v.no_dupes) == (0, 0, 0, 1, 0)
    blib.BICOS_FreeConfig(c)
    blib.BICOS_FreeResult(None)  # must be a no-op


def test_invalid_disparity_values(blib):
    assert np.isnan(blib.BICOS_InvalidDisparityFloat())
    assert blib.BICOS_InvalidDisparityInt16() == -32768


def test_descriptor_words(blib):
    assert blib.bicos_descriptor_words(8, 0) == 1
    assert blib.bicos_descriptor_words(17, 0) == 2
    assert blib.bicos_descriptor_words(33, 0) == 4
    assert blib.bicos_descriptor_words(40, 0) == 8
    assert blib.bicos_descriptor_words(66, 0) == -2
    assert blib.bicos_descriptor_words(16, 1) == 8
    assert blib.bicos_descriptor_words(17, 1) == -2
    assert blib.bicos_desc_pitch(5, 1) == 8 and blib.bicos_desc_pitch(2048, 4) == 8192


def test_pybicos_config_roundtrip():
    import pybicos
    c = pybicos.Config()
    assert c.variant == "NoDuplicates" and c.subpixel_step is None and c.min_variance is None
    c.subpixel_step = 0.1
    c.min_variance = 2.0
    c.mode = pybicos.TransformMode.FULL
    c.precision = pybicos.Precision.DOUBLE
    c.set_consistency(max_lr_diff=3, no_dupes=True)
    assert abs(c.subpixel_step - 0.1) < 1e-7 and c.min_variance == 2.0
    assert c.mode == pybicos.TransformMode.FULL and c.precision == pybicos.Precision.DOUBLE
    assert c.variant == {"type": "Consistency", "max_lr_diff": 3, "no_dupes": True}
    c.set_no_duplicates()
    assert c.variant == "NoDuplicates"
    assert "Config(" in repr(c)


def test_pybicos_errors_without_gpu():
    import torch
    import pybicos
    with pytest.raises(ValueError):
        pybicos.match([], [])
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    z = [np.zeros((4, 4), np.uint8)] * 4
    with pytest.raises(RuntimeError):
        pybicos.match(z, z)


@pytest.mark.skipif(not os.path.isdir("/root/reference/pybicos"), reason="reference not mounted")
def test_reference_python_wrapper_drives_our_abi(tmp_path, blib):
    """The reference's own pybicos/__init__.py, unmodified, loads libbicos_amd.so as its
    pybicos_c.so and drives the config ABI (the struct layout it assumes is ours)."""
    pkg = tmp_path / "refpybicos"
    pkg.mkdir()
    os.symlink("/root/reference/pybicos/__init__.py", pkg / "__init__.py")
    from libbicos_amd import _lib
    os.symlink(_lib.LIB_PATH, pkg / "pybicos_c.so")
    spec = importlib.util.spec_from_file_location("refpybicos", str(pkg / "__init__.py"),
                                                  submodule_search_locations=[str(pkg)])
    mod = importlib.util.module_from_spec(spec)
    # the reference locates its library next to abspath(__file__) -- the symlink dir
    mod.__file__ = str(pkg / "__init__.py")
    spec.loader.exec_module(mod)
    c = mod.Config()
    c.set_consistency(max_lr_diff=4, no_dupes=True)
    assert c.variant == {"type": "Consistency", "max_lr_diff": 4, "no_dupes": True}
    assert c.precision == mod.Precision.SINGLE and c.nxcorr_threshold == 0.5
    assert np.isnan(mod.invalid_disparity(np.float32))
    assert mod.invalid_disparity(np.int16) == -32768


def test_device_out_validation_rejects_bad_tensors():
    """Engine.match / search / transform write through raw pointers: a wrong dtype, shape,
    device or layout must raise before any launch (checked on CPU tensors, no GPU)."""
    import torch
    from libbicos_amd.device import _check_out
    cpu = torch.device("cpu")
    good = torch.empty((4, 6), dtype=torch.float32)
    _check_out(good, "out", (4, 6), (torch.float32,), cpu)
    with pytest.raises(ValueError, match="shape"):
        _check_out(torch.empty((4, 5), dtype=torch.float32), "out", (4, 6), (torch.float32,), cpu)
    with pytest.raises(ValueError, match="float64"):  # DOUBLE corrmap given a float32 tensor
        _check_out(good, "corrmap", (4, 6), (torch.float64,), cpu)
    with pytest.raises(ValueError, match="int16"):  # no-nxcorr disparity given float32
        _check_out(good, "out", (4, 6), (torch.int16,), cpu)
    with pytest.raises(ValueError, match="contiguous"):
        _check_out(torch.empty((6, 4), dtype=torch.float32).t(), "out", (4, 6),
                   (torch.float32,), cpu)
    with pytest.raises(ValueError, match="must be on"):
        _check_out(good, "out", (4, 6), (torch.float32,), torch.device("meta"))


def test_multi_gpu_entries_validate_before_any_gpu_call(blib):
    """bicos_match_host_multi / bicos_match_bands_device reject bad arguments (no device
    list, n < 2, bad depth, negative band heights) before touching a GPU."""
    from libbicos_amd._lib import BicosConfig
    cfg = blib.BICOS_CreateDefaultConfig()
    PP = ctypes.c_void_p * 4
    imgs = PP()
    one = (ctypes.c_int * 1)(0)
    rc = blib.bicos_match_host_multi(None, 0, imgs, imgs, 4, 8, 8, 0, 1, cfg, 1, None, None)
    assert rc == -1 and b"device" in blib.bicos_last_error()
    rc = blib.bicos_match_host_multi(one, 1, imgs, imgs, 1, 8, 8, 0, 1, cfg, 1, None, None)
    assert rc == -1 and b"two images" in blib.bicos_last_error()
    rc = blib.bicos_match_host_multi(one, 1, imgs, imgs, 4, 8, 8, 0, 3, cfg, 1, None, None)
    assert rc == -1 and b"depth" in blib.bicos_last_error()
    br = (ctypes.c_int * 1)(8)
    pz = (ctypes.c_size_t * 1)(8)
    rc = blib.bicos_match_bands_device(None, 0, imgs, imgs, br, pz, pz, 4, 8, 1, cfg, 1, None, None)
    assert rc == -1 and b"device" in blib.bicos_last_error()
    rc = blib.bicos_match_bands_device(one, 1, imgs, imgs, None, pz, pz, 4, 8, 1, cfg, 1, None, None)
    assert rc == -1 and b"band" in blib.bicos_last_error()
    blib.BICOS_FreeConfig(cfg)
