"""Host-side checks of the one-launch Consistency search's key arithmetic (search_mx.hip
search_lr_kernel): the FP4 digit encoding of |a| (lr_abs_digits, restated
here as the kernel computes it), and the float32 exactness of the keys the products form,

    D = ham + (col1 % 32) * 2^-12 + col0_offset * 2^-15        (reverse keys, per block)
    D = ham + (col1 - B) * 2^-12 + c0w * 2^-15                  (forward running minimum)

with the decodings the kernel applies to them. The GPU parity tests check the kernel itself;
these pin the arithmetic it relies on, for every value it can meet."""
import numpy as np

FP4 = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0]   # e2m1 codes 0..7
ABS_CONST = [1, 6, 6, 6, 6, 6]                   # right-operand constants of the six elements


def lr_code(u):
    return u if u <= 4 else (5 if u == 6 else (6 if u == 8 else 7))


def lr_abs_digits(n):
    """Mirror of search_mx.hip lr_abs_digits: the left FP4 codes of the six |a| elements."""
    if n < 0:
        return [7] * 6
    v0, q = n % 3, n // 3
    a = min(4, q // 12)
    r = q - 12 * a
    cq = 0
    for i in range(a):
        cq |= 7 << (4 * i)
    if a == 4:
        cq |= lr_code(r) << 16
    else:
        r1 = 8 if r >= 8 else (6 if r == 7 else (4 if r == 5 else r))
        cq |= lr_code(r1) << (4 * a)
        cq |= lr_code(r - r1) << (4 * a + 4)
    b1 = (2 * v0) | ((cq & 0xF) << 4)
    b2 = (cq >> 4) & 0xFF
    b3 = (cq >> 12) & 0xFF
    return [b1 & 0xF, b1 >> 4, b2 & 0xF, b2 >> 4, b3 & 0xF, b3 >> 4]


def test_abs_digits_encode_every_popcount():
    for n in range(0, 155):  # <= 154 used bits
        codes = lr_abs_digits(n)
        assert all(0 <= c <= 7 for c in codes)
        assert sum(k * FP4[c] for k, c in zip(ABS_CONST, codes)) == n, n
    # the past-the-image column: larger than any distance
    assert sum(k * FP4[c] for k, c in zip(ABS_CONST, lr_abs_digits(-1))) == 186 > 154


def test_reverse_keys_exact_and_decodable():
    ham = np.arange(155, dtype=np.float64)[:, None, None]
    c1d = np.arange(32, dtype=np.float64)[None, :, None]
    c0 = np.arange(0, 2048, 7, dtype=np.float64)[None, None, :]
    exact = ham + c1d * 2.0 ** -12 + c0 * 2.0 ** -15
    d32 = exact.astype(np.float32)
    assert np.array_equal(d32.astype(np.float64), exact)  # no rounding anywhere
    k = (d32 * np.float32(32768.0)).astype(np.uint32)      # the epilogue's decoding
    assert np.array_equal((k & 0x7FFF).astype(np.int64) - 8 * c1d.astype(np.int64),
                          np.broadcast_to(c0.astype(np.int64), k.shape))
    assert np.array_equal(k >> 15, np.broadcast_to(ham.astype(np.uint32), k.shape))
    # for a fixed col1 the bits order by (ham, col0): the reverse search's first minimum
    flat = d32[:, 5, :].reshape(-1).view(np.uint32)
    assert np.all(np.diff(flat.astype(np.int64)) > 0)


def test_forward_running_minimum_exact_and_decodable():
    ham = np.arange(0, 155, 3, dtype=np.float64)[:, None, None]
    rel = np.arange(-2047, 32, 5, dtype=np.float64)[None, :, None]   # col1 - B
    c0w = np.arange(128, dtype=np.float64)[None, None, :]             # 4 j + t
    exact = ham + rel * 2.0 ** -12 + c0w * 2.0 ** -15
    d32 = exact.astype(np.float32)
    assert np.array_equal(d32.astype(np.float64), exact)
    v = d32 - (c0w * 2.0 ** -15).astype(np.float32)                   # exact
    r = np.rint(v)
    assert np.array_equal(r, np.broadcast_to(ham, r.shape).astype(np.float32))
    assert np.array_equal(((v - r) * np.float32(4096.0)).astype(np.int64),
                          np.broadcast_to(rel.astype(np.int64), v.shape))
