"""Single-process multi-GPU entries (bicos_match_host_multi, bicos_match_bands_device;
SURVEY.md s8(e)) on the GPU box.

Band b runs on device b % torch.cuda.device_count() (`_devices`): on a multi-GPU box the
bands land on distinct GPUs and the cross-device branches run (peer access, peer copies of
the staged maps out of the stream-ordered pool, engines of different devices); on a one-GPU
box every band is on device 0, and the row split, the per-band pipelines (threads and
engines for the host form; the staged maps and the peer-copy gather for the device form,
which every band after the first takes even on the root) and the reassembly are still
exercised as on 8 GPUs, only with the copies on one device.
The bar is byte identity with the one-GPU call, which itself is checked against the oracle
elsewhere -- plus one direct oracle check per form.
"""
import numpy as np
import pytest

from libbicos_amd.synthetic import stereo_stack

pytestmark = pytest.mark.gpu


def dev(a):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    return torch.from_numpy(a).cuda()


def host(t):
    return t.cpu().numpy()


def same(a, b):
    assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
    # bytes, so NaN == NaN and -0 != +0
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), \
        "%d of %d elements differ" % (int((a != b).sum()), a.size)


def _devices(k):
    """Device of band b: round-robin over the visible GPUs (selected by count, not fixed)."""
    import torch
    nd = torch.cuda.device_count()
    return [b % nd for b in range(k)]


def _place(bands):
    """Band b's tensor moved to device _devices(k)[b] (a slice stays a view on its own GPU)."""
    out = []
    for t, d in zip(bands, _devices(len(bands))):
        out.append(t if t.device.index == d else t.to("cuda:%d" % d))
    return out


def test_band_devices_follow_the_device_count(gpu):
    import torch
    nd = torch.cuda.device_count()
    assert _devices(9) == [b % nd for b in range(9)]
    assert len(set(_devices(9))) == min(nd, 9)


def _pyb_cfg(pybicos, thr=0.5, step=None, minvar=None, consistency=False, double=False):
    c = pybicos.Config()
    c.nxcorr_threshold = thr
    if step is not None:
        c.subpixel_step = step
    if minvar is not None:
        c.min_variance = minvar
    if consistency:
        c.set_consistency(max_lr_diff=2, no_dupes=True)
    if double:
        c.precision = pybicos.Precision.DOUBLE
    return c


@pytest.mark.parametrize("n,H,W,dt,kw,ndev", [
    (33, 64, 512, np.uint8, {}, 3),                              # ragged bands (22/21/21)
    (8, 37, 200, np.uint16, {"thr": 0.8}, 4),                   # u16, odd width
    (40, 24, 384, np.uint8, {"step": 0.25, "minvar": 1.0}, 2),  # subpixel + min variance
    (20, 30, 256, np.uint8, {"consistency": True}, 3),          # Consistency
    (16, 16, 300, np.uint8, {"double": True}, 2),               # DOUBLE corrmap
    (8, 2, 64, np.uint8, {}, 5),                                 # fewer rows than devices
])
def test_host_multi_equals_one_gpu(gpu, n, H, W, dt, kw, ndev):
    import pybicos
    L, R = stereo_stack(n, H, W, dt)
    cfg = _pyb_cfg(pybicos, **kw)
    d1, c1 = pybicos.match(list(L), list(R), cfg)
    dm, cm = pybicos.match(list(L), list(R), cfg, devices=_devices(ndev))
    same(dm, d1)
    same(cm, c1)


def test_host_multi_matches_oracle(gpu, oracle):
    import pybicos
    L, R = stereo_stack(33, 40, 640)
    d, c = pybicos.match(list(L), list(R), _pyb_cfg(pybicos, thr=0.9), devices=_devices(4))
    rd, rc = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=0.9))
    same(d, rd)
    same(c, rc)


def test_host_multi_errors(gpu):
    import pybicos
    a = [np.zeros((8, 8), np.uint8)] * 8
    with pytest.raises(RuntimeError, match="device index"):
        pybicos.match(a, a, devices=[0, 4096])
    with pytest.raises(ValueError):
        pybicos.match(a, a, devices=[])


def _bands(H, k):
    from libbicos_amd.distributed import band_rows
    return [band_rows(H, k, b) for b in range(k)]


@pytest.mark.parametrize("n,H,W,dt,kw,k", [
    (33, 96, 1024, np.uint8, {}, 4),
    (17, 50, 333, np.uint16, {"nxcorr_threshold": 0.7}, 3),
    (12, 40, 256, np.uint8, {"nxcorr_threshold": None}, 2),             # int16 maps
    (40, 32, 512, np.uint8, {"subpixel_step": 0.1, "min_variance": 2.0}, 3),
    (20, 33, 256, np.uint8, {"variant": 1, "max_lr_diff": 1}, 2),      # Consistency
    (16, 20, 128, np.uint8, {"precision": 1}, 2),                       # DOUBLE
])
def test_bands_device_equals_whole_frame(gpu, n, H, W, dt, kw, k):
    """Band views of one frame (non-dense plane pitch: each band is a slice of the full
    stack) matched per band and gathered equal the one-call whole-frame match."""
    from libbicos_amd.device import MatchConfig, match_bands
    L, R = stereo_stack(n, H, W, dt)
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    d1, c1 = gpu.match(s0, s1, cfg)
    b = _bands(H, k)
    dm, cm = match_bands(_place([s0[:, r0:r1] for r0, r1 in b]),
                         _place([s1[:, r0:r1] for r0, r1 in b]), cfg)
    same(host(dm), host(d1))
    if c1 is None:
        assert cm is None
    else:
        same(host(cm), host(c1))


def test_bands_device_dense_bands_and_empty_band(gpu, oracle):
    """Separately allocated (dense) bands, one of them empty, against the oracle."""
    from libbicos_amd.device import MatchConfig, match_bands
    L, R = stereo_stack(33, 30, 512)
    cuts = [(0, 11), (11, 11), (11, 30)]
    dm, cm = match_bands(_place([dev(L[:, a:b]) for a, b in cuts]),
                         _place([dev(R[:, a:b]) for a, b in cuts]),
                         MatchConfig(nxcorr_threshold=0.5))
    rd, rc = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=0.5))
    same(host(dm), rd)
    same(host(cm), rc)


def test_bands_device_repeated_calls_reuse_the_stage(gpu):
    """Growing then shrinking band sets on the same engines stay exact (stage reuse)."""
    from libbicos_amd.device import MatchConfig, match_bands
    cfg = MatchConfig()
    for H, k in ((16, 2), (64, 4), (24, 3)):
        L, R = stereo_stack(33, H, 256)
        s0, s1 = dev(L), dev(R)
        d1, c1 = gpu.match(s0, s1, cfg)
        b = _bands(H, k)
        dm, cm = match_bands(_place([s0[:, r0:r1] for r0, r1 in b]),
                         _place([s1[:, r0:r1] for r0, r1 in b]), cfg)
        same(host(dm), host(d1))
        same(host(cm), host(c1))


@pytest.mark.parametrize("W,kw", [(1, {}), (3, {"precision": 1}), (5, {"nxcorr_threshold": None})])
def test_bands_device_one_row_bands_of_narrow_frames(gpu, W, kw):
    """Nine one-row bands of a 1-5 column frame, all but the first through the stage: the
    per-band slack (256-byte slots) dominates the stage size here, the case where a stage
    reserved by a different formula than the enqueue loop's offsets was overrun."""
    from libbicos_amd.device import MatchConfig, match_bands
    L, R = stereo_stack(8, 9, W, dmin=0, drange=2)
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    d1, c1 = gpu.match(s0, s1, cfg)
    b = _bands(9, 9)
    dm, cm = match_bands(_place([s0[:, r0:r1] for r0, r1 in b]),
                         _place([s1[:, r0:r1] for r0, r1 in b]), cfg)
    same(host(dm), host(d1))
    if c1 is not None:
        same(host(cm), host(c1))


@pytest.mark.parametrize("kw,k", [({}, 4), ({"nxcorr_threshold": None}, 3),
                                  ({"subpixel_step": 0.25, "precision": 1}, 3)])
def test_bands_device_host_staged_gather(gpu, monkeypatch, kw, k):
    """The gather's fallback when direct peer DMA is refused (multi.cpp enable_peer_path:
    all or nothing): every band's maps go down to the engine's pinned buffer on
    the band's stream and up into the root's maps on the root's stream behind an event.
    BICOS_GATHER_HOST=1 forces that path, so the one-GPU box runs it too."""
    from libbicos_amd.device import MatchConfig, match_bands
    L, R = stereo_stack(33, 45, 384)
    s0, s1 = dev(L), dev(R)
    cfg = MatchConfig(**kw)
    d1, c1 = gpu.match(s0, s1, cfg)
    b = _bands(45, k)
    monkeypatch.setenv("BICOS_GATHER_HOST", "1")
    for _ in range(2):  # the second call reuses the pinned buffer and its events
        dm, cm = match_bands(_place([s0[:, r0:r1] for r0, r1 in b]),
                             _place([s1[:, r0:r1] for r0, r1 in b]), cfg)
        same(host(dm), host(d1))
        if c1 is not None:
            same(host(cm), host(c1))
