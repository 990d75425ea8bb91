"""bicos-cli (libbicos_amd/cli, reference src/cli.cpp:55-253, src/fileutils.cpp:30-154,
include/fileutils.hpp:44-89).

CPU: the file layer (tests/cpp/imageio_check) against independent Python encoders and
decoders -- PNG of every colour type / bit depth / filter, PGM, TIFF, the Q matrix from
YAML and XML FileStorage files, reprojection to .xyz. GPU: the CLI end to end on a folder
of PNGs, its raw TIFF disparity and correlation maps bit-exact against the CPU oracle, and
the point cloud against numpy's reprojection of the oracle disparity.
"""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "tests", "cpp", "imageio_check")
CLI = os.path.join(ROOT, "libbicos_amd", "bicos-cli")


def _built():
    if not os.path.exists(CHECK):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True,
                       capture_output=True)
    if not os.path.exists(CLI):
        subprocess.run(["make", "-C", os.path.join(ROOT, "libbicos_amd", "cli")], check=True,
                       capture_output=True)


# ------------------------------------------------------------ independent helpers
def png_bytes(samples, ctype, depth, filt=0, palette=None):
    """PNG encoder (test side): samples [h, w, ch] integers; filt = 0..4 for every row."""
    h, w = samples.shape[:2]
    ch = samples.shape[2] if samples.ndim == 3 else 1
    s = samples.reshape(h, w * ch).astype(np.int64)
    rows = []
    for r in range(h):
        if depth == 16:
            raw = b"".join(struct.pack(">H", int(v)) for v in s[r])
        elif depth == 8:
            raw = bytes(int(v) for v in s[r])
        else:
            bits = "".join(format(int(v), "0%db" % depth) for v in s[r])
            bits += "0" * (-len(bits) % 8)
            raw = bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))
        rows.append(bytearray(raw))
    bpp = max(1, ch * depth // 8)
    out = bytearray()
    prev = bytearray(len(rows[0]))
    for raw in rows:
        f = bytearray(len(raw))
        for i in range(len(raw)):
            a = raw[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            if filt == 0:
                p = 0
            elif filt == 1:
                p = a
            elif filt == 2:
                p = b
            elif filt == 3:
                p = (a + b) // 2
            else:
                q = a + b - c
                pa, pb, pc = abs(q - a), abs(q - b), abs(q - c)
                p = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
            f[i] = (raw[i] - p) & 0xFF
        out += bytes([filt]) + f
        prev = raw

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
    if palette is not None:
        png += chunk(b"PLTE", bytes(palette.astype(np.uint8).ravel()))
    png += chunk(b"IDAT", zlib.compress(bytes(out))) + chunk(b"IEND", b"")
    return png


def gray_of(rgb):
    """libpng png_set_rgb_to_gray(0.299, 0.587) as OpenCV's PNG reader asks for it."""
    r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
    return (9798 * r + 19235 * g + 3735 * b + 16384) >> 15


def decode(path, keep16, tmp):
    out = os.path.join(tmp, "dec.raw")
    r = subprocess.run([CHECK, "decode", path, str(int(keep16)), out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    raw = open(out, "rb").read()
    rows, cols, typ = struct.unpack("<iii", raw[:12])
    return np.frombuffer(raw[12:], np.uint16 if typ == 2 else np.uint8).reshape(rows, cols), typ


def read_tiff(path):
    """Baseline TIFF reader (test side): one strip, one channel, little-endian."""
    b = open(path, "rb").read()
    assert b[:4] == b"II*\x00"
    off = struct.unpack("<I", b[4:8])[0]
    n = struct.unpack("<H", b[off:off + 2])[0]
    tags = {}
    for i in range(n):
        t, ty, cnt, v = struct.unpack("<HHII", b[off + 2 + 12 * i: off + 14 + 12 * i])
        tags[t] = v & 0xFFFF if ty == 3 else v
    w, h, bits, fmt = tags[256], tags[257], tags[258], tags.get(339, 1)
    assert tags[259] == 1 and tags[277] == 1
    dt = {(8, 1): np.uint8, (16, 1): np.uint16, (16, 2): np.int16, (32, 3): np.float32,
          (64, 3): np.float64}[(bits, fmt)]
    data = b[tags[273]: tags[273] + tags[279]]
    return np.frombuffer(data, dt).reshape(h, w)


# ------------------------------------------------------------------- CPU tests
@pytest.mark.parametrize("ctype,depth,ch", [(0, 8, 1), (0, 16, 1), (0, 1, 1), (0, 2, 1), (0, 4, 1),
                                            (2, 8, 3), (2, 16, 3), (4, 8, 2), (6, 8, 4), (6, 16, 4),
                                            (3, 8, 1), (3, 4, 1)])
@pytest.mark.parametrize("filt", [0, 1, 2, 3, 4])
def test_png_decode(tmp_path, ctype, depth, ch, filt):
    _built()
    rng = np.random.default_rng(ctype * 100 + depth * 10 + filt)
    h, w = 7, 13
    hi = (1 << depth) - 1
    palette = None
    if ctype == 3:
        palette = rng.integers(0, 256, size=(1 << depth, 3))
    s = rng.integers(0, hi + 1, size=(h, w, ch))
    p = tmp_path / "x.png"
    p.write_bytes(png_bytes(s, ctype, depth, filt, palette))
    for keep16 in (False, True):
        got, typ = decode(str(p), keep16, str(tmp_path))
        v = s.astype(np.int64)
        if depth == 16 and not keep16:
            v = v >> 8
        if ctype == 3:
            want = gray_of(palette[v[..., 0]])
        elif ctype in (0, 4):
            want = v[..., 0] * 255 // hi if depth < 8 else v[..., 0]
        else:
            want = gray_of(v)
        assert typ == (2 if depth == 16 and keep16 else 0)
        np.testing.assert_array_equal(got.astype(np.int64), want)


def test_pgm_decode(tmp_path):
    _built()
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, size=(5, 9)).astype(np.uint8)
    p = tmp_path / "a.pgm"
    p.write_bytes(b"P5\n# comment\n9 5\n255\n" + a.tobytes())
    got, typ = decode(str(p), True, str(tmp_path))
    assert typ == 0
    np.testing.assert_array_equal(got, a)
    b16 = rng.integers(0, 4096, size=(4, 6)).astype(">u2")
    p.write_bytes(b"P5 6 4 4095\n" + b16.tobytes())
    got, typ = decode(str(p), True, str(tmp_path))
    assert typ == 2
    np.testing.assert_array_equal(got, b16.astype(np.uint16))
    got, typ = decode(str(p), False, str(tmp_path))
    np.testing.assert_array_equal(got, (b16.astype(np.uint16) >> 8).astype(np.uint8))


def test_bad_inputs_are_errors(tmp_path):
    _built()
    p = tmp_path / "x.png"
    png = bytearray(png_bytes(np.zeros((2, 2, 1), np.int64), 0, 8))
    png[-20] ^= 0xFF  # corrupt a chunk -> CRC mismatch
    p.write_bytes(bytes(png))
    r = subprocess.run([CHECK, "decode", str(p), "1", str(tmp_path / "o")], capture_output=True, text=True)
    assert r.returncode == 1 and "error" in r.stderr
    p.write_bytes(b"GIF89a....")
    r = subprocess.run([CHECK, "decode", str(p), "1", str(tmp_path / "o")], capture_output=True, text=True)
    assert r.returncode == 1 and "unsupported" in r.stderr


@pytest.mark.parametrize("dt,typ", [(np.int16, 3), (np.float32, 5), (np.float64, 6), (np.uint8, 0),
                                    (np.uint16, 2)])
def test_tiff_roundtrip(tmp_path, dt, typ):
    _built()
    rng = np.random.default_rng(typ)
    a = (rng.standard_normal((6, 11)) * 1000).astype(dt)
    if dt == np.float32:
        a[0, 0] = np.nan
    raw = tmp_path / "a.raw"
    raw.write_bytes(a.tobytes())
    out = tmp_path / "a.tiff"
    r = subprocess.run([CHECK, "tiff", str(raw), "6", "11", str(typ), str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    back = read_tiff(str(out))
    assert back.dtype == a.dtype
    assert np.array_equal(back.view(np.uint8), a.view(np.uint8))


def test_png_encode_roundtrip(tmp_path):
    _built()
    a = np.arange(5 * 7, dtype=np.uint8).reshape(5, 7) * 7
    raw = tmp_path / "a.raw"
    raw.write_bytes(a.tobytes())
    out = tmp_path / "a.png"
    r = subprocess.run([CHECK, "png", str(raw), "5", "7", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got, typ = decode(str(out), True, str(tmp_path))
    np.testing.assert_array_equal(got, a)


def test_colorize_normalises_valid_pixels(tmp_path):
    """cv::normalize(NORM_MINMAX) under the validity mask, then the colour map; invalid
    pixels black (reference src/fileutils.cpp:30-46)."""
    _built()
    d = np.array([[-32768, 10, 20], [30, 40, -32768]], np.int16)
    raw = tmp_path / "d.raw"
    raw.write_bytes(d.tobytes())
    out = tmp_path / "d.rgb"
    for cmap in (0, 1):
        r = subprocess.run([CHECK, "colorize", str(raw), "2", "3", "3", str(cmap), str(out)],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        rgb = np.frombuffer(out.read_bytes(), np.uint8).reshape(2, 3, 3)
        assert (rgb[0, 0] == 0).all() and (rgb[1, 2] == 0).all()
        levels = [rgb[0, 1], rgb[0, 2], rgb[1, 0], rgb[1, 1]]  # 0, 85, 170, 255 of the map
        assert len({tuple(x) for x in levels}) == 4
    f = np.full((2, 2), np.nan, np.float32)
    f[0, 1] = 3.5
    raw.write_bytes(f.tobytes())
    r = subprocess.run([CHECK, "colorize", str(raw), "2", "2", "5", "0", str(out)], capture_output=True, text=True)
    assert r.returncode == 0
    rgb = np.frombuffer(out.read_bytes(), np.uint8).reshape(2, 2, 3)
    assert (rgb[0, 0] == 0).all() and rgb[0, 1].any()   # flat image: level 0 of the map


Q = np.array([[1, 0, 0, -320.5], [0, 1, 0, -240.25], [0, 0, 0, 800.0], [0, 0, 1 / 0.12, 0]])
YAML = """%YAML:1.0
---
K: !!opencv-matrix
   rows: 3
   cols: 3
   dt: d
   data: [ 1., 0., 0., 0., 1., 0., 0., 0., 1. ]
Q: !!opencv-matrix
   rows: 4
   cols: 4
   dt: d
   data: [ {} ]
"""
XML = """<?xml version="1.0"?>
<opencv_storage>
<Q type_id="opencv-matrix">
  <rows>4</rows>
  <cols>4</cols>
  <dt>d</dt>
  <data>
    {}</data></Q>
</opencv_storage>
"""


@pytest.mark.parametrize("fmt", ["yaml", "xml"])
def test_q_matrix(tmp_path, fmt):
    _built()
    p = tmp_path / ("q." + fmt)
    nums = [repr(float(v)) for v in Q.ravel()]
    p.write_text(YAML.format(", ".join(nums)) if fmt == "yaml" else XML.format(" ".join(nums)))
    r = subprocess.run([CHECK, "matrix", str(p), "Q"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    np.testing.assert_array_equal(np.array([float(x) for x in r.stdout.split()]), Q.ravel())


def reproject(d, q, allow_neg):
    """cv::reprojectImageTo3D + save_pointcloud (test side, numpy)."""
    lines = []
    for y in range(d.shape[0]):
        for x in range(d.shape[1]):
            v = float(d[y, x])
            if np.isnan(v) or (d.dtype == np.int16 and v == -32768):
                continue
            o = q @ np.array([x, y, v, 1.0])
            with np.errstate(divide="ignore", invalid="ignore"):
                p = (o[:3] * (1.0 / o[3])).astype(np.float32)
            if not np.isfinite(p).all() or (not allow_neg and p[2] < 0):
                continue
            lines.append(p)
    return np.array(lines, np.float32).reshape(-1, 3)


@pytest.mark.parametrize("dt,typ", [(np.int16, 3), (np.float32, 5)])
def test_xyz(tmp_path, dt, typ):
    _built()
    rng = np.random.default_rng(typ)
    d = rng.integers(-5, 60, size=(9, 12)).astype(dt)
    d[0, 0] = -32768 if dt == np.int16 else np.nan
    d[1, 1] = 0  # W = 0: non-finite
    raw = tmp_path / "d.raw"
    raw.write_bytes(d.tobytes())
    qf = tmp_path / "q.yml"
    qf.write_text(YAML.format(", ".join(repr(float(v)) for v in Q.ravel())))
    for allow in (0, 1):
        out = tmp_path / "p.xyz"
        r = subprocess.run([CHECK, "xyz", str(raw), "9", "12", str(typ), str(qf), str(allow), str(out)],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        got = np.loadtxt(out, dtype=np.float64).reshape(-1, 3)
        want = reproject(d, Q, allow)
        assert got.shape == want.shape
        np.testing.assert_allclose(got, want, rtol=1e-5)  # 6 significant digits in the file


def test_cli_usage_and_errors(tmp_path):
    _built()
    r = subprocess.run([CLI, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--lr-maxdiff" in r.stdout
    r = subprocess.run([CLI, "--frobnicate"], capture_output=True, text=True)
    assert r.returncode == 1 and "unknown option" in r.stderr
    (tmp_path / "in").mkdir()
    (tmp_path / "in" / "foo.png").write_bytes(png_bytes(np.zeros((2, 2, 1), np.int64), 0, 8))
    r = subprocess.run([CLI, str(tmp_path / "in")], capture_output=True, text=True)
    assert r.returncode == 1 and "NN_{left,right}" in r.stderr


# ------------------------------------------------------------------- GPU: end to end
def _write_folder(path, L, R, two_folders):
    os.makedirs(path, exist_ok=True)
    n = L.shape[0]
    depth = 16 if L.dtype == np.uint16 else 8
    for t in range(n):
        for side, a in (("left", L[t]), ("right", R[t])):
            png = png_bytes(a[..., None].astype(np.int64), 0, depth, filt=t % 5)
            if two_folders:
                d = os.path.join(path, side)
                os.makedirs(d, exist_ok=True)
                open(os.path.join(d, "%d.png" % t), "wb").write(png)
            else:
                open(os.path.join(path, "%d_%s.png" % (t, side)), "wb").write(png)


CLI_CASES = [
    ("default_full", 12, np.uint8, False, [], dict(nxcorr_threshold=0.75, mode=1)),
    ("limited_var_step_corr", 33, np.uint8, False, ["--limited", "-v", "2", "-s", "0.2", "--corrmap"],
     dict(nxcorr_threshold=0.75, mode=0, min_variance=2.0, subpixel_step=0.2)),
    ("two_folders_u16_lr", 16, np.uint16, True, ["--limited", "-m", "1", "-t", "0.9"],
     dict(nxcorr_threshold=0.9, mode=0, variant=1, max_lr_diff=1)),
    ("no_threshold_int16", 10, np.uint8, False, ["-t", "0", "-n", "9"],
     dict(nxcorr_threshold=None, mode=1)),
    ("corrmap_without_threshold", 8, np.uint8, False, ["-t", "0", "--corrmap"],
     dict(nxcorr_threshold=-1.0, mode=1)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CLI_CASES, ids=lambda c: c[0])
def test_cli_end_to_end(case, oracle, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    _built()
    from libbicos_amd.synthetic import stereo_stack
    name, n, dt, two, extra, cfg = case
    H, W = 40, 200
    L, R = stereo_stack(n, H, W, dt)
    src = str(tmp_path / "in")
    _write_folder(src, L, R, two)
    folders = [os.path.join(src, "left"), os.path.join(src, "right")] if two else [src]
    out = str(tmp_path / "out" / "disp.png")
    os.makedirs(os.path.dirname(out))
    qf = tmp_path / "q.yml"
    qf.write_text(YAML.format(", ".join(repr(float(v)) for v in Q.ravel())))
    r = subprocess.run([CLI] + folders + extra + ["-o", out, "-q", str(qf)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    if "-n" in extra:
        k = int(extra[extra.index("-n") + 1])
        L, R = L[:k], R[:k]
    rd, rc = oracle.match(L, R, oracle.OracleConfig(**cfg))
    disp = read_tiff(str(tmp_path / "out" / "disp.tiff"))
    assert disp.dtype == rd.dtype
    assert np.array_equal(disp.view(np.uint8), rd.view(np.uint8))
    assert os.path.getsize(str(tmp_path / "out" / "disp.png")) > 0
    if "--corrmap" in extra:
        corr = read_tiff(str(tmp_path / "out" / "disp-corrmap.tiff"))
        assert np.array_equal(corr.view(np.uint8), rc.view(np.uint8))
    got = np.loadtxt(str(tmp_path / "out" / "disp.xyz"), dtype=np.float64).reshape(-1, 3)
    want = reproject(rd, Q, False)
    assert len(want) > 0.3 * H * W  # most pixels have a valid positive disparity
    np.testing.assert_allclose(got, want, rtol=1e-5)
