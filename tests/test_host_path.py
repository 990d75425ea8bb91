"""Host-buffer path (bicos_match_host / pybicos.match / BICOS_Match): banded, pipelined
upload -> match -> download. Every band count and layout must give exactly the bytes of
the device-resident match (and of the oracle)."""
import ctypes

import numpy as np
import pytest

from libbicos_amd.synthetic import stereo_stack
from tests.test_gpu_parity import cfg_of, gpu_match, same

pytestmark = pytest.mark.gpu


def _pyconfig(**kw):
    import pybicos
    cfg = pybicos.Config()
    cfg.nxcorr_threshold = kw.get("nxcorr_threshold", 0.5)
    if kw.get("subpixel_step"):
        cfg.subpixel_step = kw["subpixel_step"]
    if kw.get("min_variance") is not None:
        cfg.min_variance = kw["min_variance"]
    if kw.get("variant") == 1:
        cfg.set_consistency(max_lr_diff=kw.get("max_lr_diff", 1), no_dupes=kw.get("no_dupes", False))
    return cfg


# rows -> 1, 1, 2, 4 and 8 bands (ragged last bands included)
@pytest.mark.parametrize("H", [1, 63, 64, 301, 1100])
def test_host_bands_equal_device(gpu, H):
    import pybicos
    L, R = stereo_stack(12, H, 256, dmin=3, drange=20)
    kw = dict(nxcorr_threshold=0.8)
    d, c = pybicos.match(list(L), list(R), _pyconfig(**kw))
    rd, rc = gpu_match(gpu, L, R, **kw)
    same(d, rd)
    same(c, rc)


@pytest.mark.parametrize("kw", [
    dict(nxcorr_threshold=0.6, subpixel_step=0.25, min_variance=1.0),
    dict(nxcorr_threshold=0.6, variant=1, max_lr_diff=2, no_dupes=True),
])
@pytest.mark.parametrize("dt", [np.uint8, np.uint16])
def test_host_configs_equal_oracle(gpu, oracle, kw, dt):
    import pybicos
    L, R = stereo_stack(33, 300, 384, dt, dmin=3, drange=30)
    d, c = pybicos.match(list(L), list(R), _pyconfig(**kw))
    rd, rc = oracle.match(L[:, ::37], R[:, ::37], cfg_of(oracle, **kw))  # every 37th row
    same(d[::37].copy(), rd)
    same(c[::37].copy(), rc)
    gd, gc = gpu_match(gpu, L, R, **kw)
    same(d, gd)
    same(c, gc)


def test_host_strided_and_separate_images(gpu):
    """Row padding (step > cols) and per-image allocations through the C-ABI entry."""
    from libbicos_amd import _lib
    from libbicos_amd.device import MatchConfig
    L, R = stereo_stack(17, 200, 300, np.uint16, dmin=2, drange=25)
    n, H, W = L.shape
    pad = 13
    planes0 = []
    planes1 = []
    for t in range(n):  # separate allocations, padded rows
        a = np.zeros((H, W + pad), np.uint16)
        a[:, :W] = L[t]
        b = np.zeros((H, W + pad), np.uint16)
        b[:, :W] = R[t]
        planes0.append(a)
        planes1.append(b)
    p0 = (ctypes.c_void_p * n)(*[a.ctypes.data for a in planes0])
    p1 = (ctypes.c_void_p * n)(*[b.ctypes.data for b in planes1])
    cfgc, has = MatchConfig(nxcorr_threshold=0.7, subpixel_step=0.1).to_c()
    disp = np.empty((H, W), np.float32)
    corr = np.empty((H, W), np.float32)
    rc = _lib.lib().bicos_match_host(None, p0, p1, n, H, W, (W + pad) * 2, 2, ctypes.byref(cfgc),
                                     has, disp.ctypes.data, corr.ctypes.data)
    _lib.check(rc, "bicos_match_host")
    gd, gc = gpu_match(gpu, L, R, nxcorr_threshold=0.7, subpixel_step=0.1)
    same(disp, gd)
    same(corr, gc)


def test_host_without_nxcorr_is_int16(gpu):
    from libbicos_amd import _lib
    from libbicos_amd.device import MatchConfig
    L, R = stereo_stack(9, 130, 200)
    n, H, W = L.shape
    p0 = (ctypes.c_void_p * n)(*[L[t].ctypes.data for t in range(n)])
    p1 = (ctypes.c_void_p * n)(*[R[t].ctypes.data for t in range(n)])
    cfgc, has = MatchConfig(nxcorr_threshold=None).to_c()
    disp = np.empty((H, W), np.int16)
    rc = _lib.lib().bicos_match_host(None, p0, p1, n, H, W, 0, 1, ctypes.byref(cfgc), has,
                                     disp.ctypes.data, None)
    _lib.check(rc, "bicos_match_host")
    gd, _ = gpu_match(gpu, L, R, nxcorr_threshold=None)
    same(disp, gd)


def test_bicos_match_c_abi_in_place(gpu):
    """BICOS_Match (the reference's ctypes ABI) returns the same maps as pybicos.match."""
    import pybicos
    from libbicos_amd import _lib
    L, R = stereo_stack(20, 150, 240)
    n, H, W = L.shape
    cfg = _pyconfig(nxcorr_threshold=0.9)
    d, c = pybicos.match(list(L), list(R), cfg)
    lib = _lib.lib()
    P = ctypes.c_void_p
    I = ctypes.c_int
    d0 = (P * n)(*[L[t].ctypes.data for t in range(n)])
    d1 = (P * n)(*[R[t].ctypes.data for t in range(n)])
    rows = (I * n)(*([H] * n))
    cols = (I * n)(*([W] * n))
    types = (I * n)(*([0] * n))
    res = lib.BICOS_Match(d0, rows, cols, types, n, d1, rows, cols, types, n, cfg._c_config)
    assert res
    try:
        r = res.contents
        assert (r.disparity_rows, r.disparity_cols, r.disparity_type) == (H, W, 5)
        assert (r.corrmap_rows, r.corrmap_cols, r.corrmap_type) == (H, W, 5)
        gd = np.ctypeslib.as_array((ctypes.c_float * (H * W)).from_address(r.disparity_data))
        gc = np.ctypeslib.as_array((ctypes.c_float * (H * W)).from_address(r.corrmap_data))
        same(gd.reshape(H, W).copy(), d)
        same(gc.reshape(H, W).copy(), c)
    finally:
        lib.BICOS_FreeResult(res)


def test_host_after_device_call_on_side_stream(gpu):
    """The engine orders its shared buffers across streams: a device-path match queued on
    another stream and a host-path match right after both come out right."""
    import torch
    import pybicos
    from libbicos_amd.device import MatchConfig, default_engine
    L, R = stereo_stack(33, 512, 1024)
    ref_d, ref_c = gpu_match(gpu, L, R, nxcorr_threshold=0.9)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    side = torch.cuda.Stream()
    eng = default_engine(0)  # the engine pybicos' host path uses too
    with torch.cuda.stream(side):
        dd, dc = eng.match(s0, s1, MatchConfig(nxcorr_threshold=0.9), stream=side)
    hd, hc = pybicos.match(list(L), list(R), _pyconfig(nxcorr_threshold=0.9))
    side.synchronize()
    same(hd, ref_d)
    same(hc, ref_c)
    same(dd.cpu().numpy(), ref_d)
    same(dc.cpu().numpy(), ref_c)


def test_host_errors(gpu):
    import pybicos
    a = [np.zeros((8, 8), np.uint8)] * 4
    with pytest.raises(RuntimeError):
        pybicos.match(a, [np.zeros((8, 8), np.uint16)] * 4)
    with pytest.raises(RuntimeError):
        pybicos.match(a, a[:3])
    with pytest.raises(RuntimeError, match="subpixel"):
        cfg = pybicos.Config()
        cfg.subpixel_step = 1e-9
        pybicos.match(a, a, cfg)
    d, c = pybicos.match([np.zeros((0, 8), np.uint8)] * 4, [np.zeros((0, 8), np.uint8)] * 4)
    assert d.shape == (0, 8) and c.shape == (0, 8)
