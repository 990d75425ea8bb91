"""CPU tests of the parity oracle (oracle/bicos_oracle.c).

The reference ships no tests or golden vectors and its CPU path cannot be built
here without OpenCV stand-ins (parity UNPINNED). The oracle is
pinned instead by (1) an independent numpy restatement (oracle/ref_numpy.py),
(2) known-answer descriptors derived by hand from the reference source, and
(3) the reference behaviours SURVEY.md Appendix A recorded from the reference
binary in the survey session.
"""
import numpy as np
import pytest

from libbicos_amd.synthetic import random_stack, stereo_stack
from oracle import ref_numpy as N


def _eq(a, b):
    if a is None or b is None:
        return a is None and b is None
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(
        a.view(np.uint8), b.view(np.uint8))


# ------------------------------------------------------------ known answers
# Hand-derived from include/impl/cpu/descriptor_transform.hpp:31-123.
@pytest.mark.parametrize("pix,mode,expect", [
    ([10, 20, 5, 30], 0, 725),   # LIMITED n=4: bits 1,0,1 | 0,1,0 | 1,1,0,1
    ([7, 3], 0, 12),             # LIMITED n=2: tail only, ring sentinel -1 -> last bit 1
    ([1, 2, 3], 0, 79),          # LIMITED n=3: sentinel again (prev_pair_sums[1] == -1)
    ([10, 20, 5, 30], 1, 725),   # FULL n=4: ..., ps0<ps2 = 1, ps2<ps0 = 0 (11 bits)
])
def test_transform_known_answers(oracle, pix, mode, expect):
    s = np.array(pix, np.uint8).reshape(len(pix), 1, 1)
    d = oracle.transform(s, mode, 1)
    assert int(d[0, 0, 0]) == expect
    assert int(N.transform(s, mode, 1)[0, 0, 0]) == expect


@pytest.mark.parametrize("n", [4, 5, 8, 9, 10, 17, 33])
def test_limited_uses_4n_minus_6_bits(oracle, n):
    # SURVEY.md Appendix A item 3 / s8 a6 (verified on the reference for n=4,8,9,10,17,33):
    # the top set bit over random pixels reaches bit 4n-7 and never beyond.
    s = random_stack(n, 64, 64, seed=n)
    d = oracle.transform(s, 0, 8)
    top = 0
    for w in range(8):
        nz = d[..., w] != 0
        if nz.any():
            top = 32 * w + int(np.max(np.floor(np.log2(d[..., w][nz].astype(np.float64)))))
    assert top == 4 * n - 7


@pytest.mark.parametrize("mode", [0, 1])
def test_used_bits_bounds_every_set_bit(oracle, mode):
    """device.used_bits (the search's K-step hint, engine.cpp used_bits) is an upper bound of
    the highest descriptor bit the transform sets, for every n of both modes (ADVICE r02:
    LIMITED n = 2 sets 4 bits, descriptor_transform.hpp:62-68)."""
    from libbicos_amd.device import used_bits
    for n in range(2, 66 if mode == 0 else 17):
        s = random_stack(n, 16, 64, seed=1000 + n)
        d = oracle.transform(s, mode, 8)
        hi = -1
        for w in range(8):
            nz = d[..., w] != 0
            if nz.any():
                hi = 32 * w + int(np.max(np.floor(np.log2(d[..., w][nz].astype(np.float64)))))
        assert hi < used_bits(n, mode), (n, mode, hi)


@pytest.mark.parametrize("n", [2, 3, 4, 8, 10, 16])
def test_full_bit_count(oracle, n):
    s = random_stack(n, 64, 64, seed=100 + n)
    d = oracle.transform(s, 1, 8)
    bits = n * n - 2 * n + 3
    words = d.view(np.uint32)
    hi = np.zeros(d.shape[:2], np.int64)
    for w in range(8):
        nz = words[..., w] != 0
        hi[nz] = 32 * w + np.floor(np.log2(words[..., w][nz].astype(np.float64))).astype(np.int64)
    assert hi.max() <= bits - 1


def test_dispatch(oracle):
    # src/impl/cpu.cpp:122-156
    assert oracle.required_bits(33, 0) == 125 and oracle.desc_words(33, 0) == 4
    assert oracle.desc_words(8, 0) == 1 and oracle.desc_words(17, 0) == 2
    assert oracle.desc_words(40, 0) == 8 and oracle.desc_words(65, 0) == 8
    assert oracle.desc_words(66, 0) == -1
    assert oracle.desc_words(16, 1) == 8 and oracle.desc_words(17, 1) == -1
    with pytest.raises(oracle.OracleError):
        s = random_stack(66, 2, 8)
        oracle.match(s, s)
    with pytest.raises(oracle.OracleError):
        s = random_stack(1, 2, 8)
        oracle.match(s, s)


# ------------------------------------------------ SURVEY Appendix A behaviours
def test_subpixel_x_sequence():
    # Appendix A item 10: accumulated float x; step 0.1 -> 20 steps ending 0.900000155
    xs = N.x_steps(0.1)
    assert len(xs) == 20 and abs(float(xs[-1]) - 0.900000155) < 1e-9
    assert len(N.x_steps(0.25)) == 9 and float(N.x_steps(0.25)[-1]) == 1.0
    assert len(N.x_steps(0.05)) == 40
    assert len(N.x_steps(0.01)) == 201


def test_narrowing_wraps_through_int32():
    # Appendix A item 10: (TInput)roundevenf(v) wraps: -32 -> 224, 300 -> 44 (u8), 65504 (u16)
    assert list(N._narrow(np.array([-32.0, 300.0, 2.5, 3.5], np.float32), np.uint8)) == [224, 44, 2, 4]
    assert int(N._narrow(np.array([-32.0], np.float32), np.uint16)[0]) == 65504


def test_nan_correlation_passes_threshold(oracle):
    # Appendix A item 7: a constant right pixel gives 0/0 = NaN, which passes `nxc < thr`
    n, H, W = 8, 1, 16
    s0 = random_stack(n, H, W, seed=5)
    s1 = random_stack(n, H, W, seed=6)
    s1[:, 0, 3] = 77
    disp = np.full((H, W), -32768, np.int16)
    disp[0, 5] = 2    # col1 = 3: constant
    disp[0, 9] = 20   # col1 = -11: out of range -> invalid
    d, corr = oracle.agree(disp, s0, s1, 0.9, None)
    assert d[0, 5] == 2 and np.isnan(corr[0, 5])
    assert d[0, 9] == -32768 and np.isnan(corr[0, 9])
    d, corr = oracle.agree(disp, s0, s1, 0.9, 1.0 * n)   # min-variance -> -1 -> rejected
    assert d[0, 5] == -32768 and corr[0, 5] == -1.0


# ---------------------------------------------------- C vs numpy cross-check
CASES = [
    (2, 4, 40, np.uint8, 0), (3, 4, 40, np.uint8, 0), (4, 6, 50, np.uint8, 1),
    (8, 12, 96, np.uint8, 0), (9, 6, 70, np.uint16, 0), (17, 8, 90, np.uint16, 0),
    (33, 8, 120, np.uint8, 0), (40, 6, 70, np.uint8, 0), (16, 6, 64, np.uint8, 1),
    (10, 6, 64, np.uint16, 1), (65, 4, 50, np.uint8, 0),
]
CFGS = [
    dict(nxcorr_threshold=None),
    dict(nxcorr_threshold=0.5),
    dict(nxcorr_threshold=0.8, min_variance=2.0),
    dict(nxcorr_threshold=0.5, subpixel_step=0.1),
    dict(nxcorr_threshold=0.3, subpixel_step=0.25, min_variance=1.0),
    dict(variant=1, max_lr_diff=1, nxcorr_threshold=None),
    dict(variant=1, max_lr_diff=3, no_dupes=True, nxcorr_threshold=0.5),
    dict(variant=1, max_lr_diff=0, nxcorr_threshold=0.2, subpixel_step=0.2),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_%dx%d_%s_m%d" % (
    c[0], c[1], c[2], np.dtype(c[3]).name, c[4]))
def test_c_oracle_matches_numpy_restatement(oracle, case):
    n, H, W, dt, mode = case
    L, R = stereo_stack(n, H, W, dt, dmin=2, drange=8)
    for cfg in CFGS:
        c = dict(cfg, mode=mode)
        a = oracle.match(L, R, oracle.OracleConfig(**c), nthreads=2)
        b = N.match(L, R, **c)
        assert _eq(a[0], b[0]) and _eq(a[1], b[1]), (case, cfg)


@pytest.mark.parametrize("dt", [np.uint8, np.uint16])
def test_c_oracle_matches_numpy_on_random_stacks(oracle, dt):
    # unstructured data: many duplicate minima, wide subpixel overshoots (wrap path)
    for n in (4, 12):
        L = random_stack(n, 6, 48, dt, seed=11, maxval=15)
        R = random_stack(n, 6, 48, dt, seed=12, maxval=15)
        for cfg in CFGS:
            a = oracle.match(L, R, oracle.OracleConfig(**cfg), nthreads=2)
            b = N.match(L, R, **cfg)
            assert _eq(a[0], b[0]) and _eq(a[1], b[1]), (n, dt, cfg)


def test_wrap_path_is_exercised():
    L = random_stack(12, 6, 48, np.uint8, seed=11)
    R = random_stack(12, 6, 48, np.uint8, seed=12)
    y0, y1, y2 = (R[:, :, 0:-2].astype(np.float32), R[:, :, 1:-1].astype(np.float32),
                  R[:, :, 2:].astype(np.float32))
    A = 0.5 * ((y0 - 2 * y1) + y2)
    B = 0.5 * (y2 - y0)
    v = A * 0.25 + B * 0.5 + y1   # x = 0.5
    assert (np.rint(v) < 0).any() or (np.rint(v) > 255).any()


def test_oracle_recovers_planted_disparity(oracle):
    n, H, W = 33, 32, 512
    L, R = stereo_stack(n, H, W)
    d, _ = oracle.match(L, R, oracle.OracleConfig(nxcorr_threshold=None))
    truth = (16 + (48 * np.arange(H)) // H)[:, None]
    valid = d != -32768
    assert valid.mean() > 0.95
    assert (d == truth)[valid].mean() > 0.9


def test_row_band_invariance(oracle):
    # every stage is row-local: matching a band of rows equals the same rows of the frame
    L, R = stereo_stack(17, 24, 96, dmin=2, drange=8)
    cfg = oracle.OracleConfig(nxcorr_threshold=0.5, subpixel_step=0.1, variant=1)
    full, fc = oracle.match(L, R, cfg, nthreads=3)
    band, bc = oracle.match(L[:, 5:13], R[:, 5:13], cfg)
    assert _eq(full[5:13].copy(), band) and _eq(fc[5:13].copy(), bc)


def test_v3_build_is_bit_identical(oracle):
    L, R = stereo_stack(33, 8, 256)
    cfg = oracle.OracleConfig(nxcorr_threshold=0.5, subpixel_step=0.1, min_variance=1.0)
    a = oracle.match(L, R, cfg)
    b = oracle.match(L, R, cfg, variant="v3")
    assert _eq(a[0], b[0]) and _eq(a[1], b[1])
