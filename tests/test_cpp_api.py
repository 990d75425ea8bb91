"""The C++ API (include/bicos/match.hpp, hip.hpp, opencv.hpp) as a reference C++ caller
uses it (reference include/match.hpp:31-41, src/lib.cpp:31-49): tests/cpp/match_cpp runs
BICOS::match through every input branch -- host images with padded rows, device images
that form one planar buffer (zero-copy), device images in separate pitched allocations
(2-D staging), an OpenCV-shaped matrix type through bicos/opencv.hpp, and the
impl::hip::match backend seam -- and each branch's maps must equal the CPU oracle's bit
for bit.
"""
import os
import subprocess

import numpy as np
import pytest

from libbicos_amd.synthetic import stereo_stack

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "match_cpp")
BRANCHES = ("host", "dev_planar", "dev_staged", "mats", "seam")


def test_cpp_driver_is_built():
    """build() compiles the driver (hipcc, no GPU needed) against the in-tree library."""
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.dirname(EXE)], check=True, capture_output=True)
    assert os.access(EXE, os.X_OK)


CASES = [
    dict(n=8, H=37, W=300, dt=np.uint8, cfg=dict(nxcorr_threshold=0.9)),
    dict(n=33, H=24, W=515, dt=np.uint8, cfg=dict(nxcorr_threshold=0.96, min_variance=2.0,
                                                  subpixel_step=0.1)),
    dict(n=12, H=19, W=257, dt=np.uint16, cfg=dict(nxcorr_threshold=None)),
    dict(n=40, H=16, W=300, dt=np.uint8, cfg=dict(nxcorr_threshold=0.96, variant=1,
                                                  max_lr_diff=1)),
    dict(n=10, H=21, W=190, dt=np.uint8, cfg=dict(nxcorr_threshold=0.5, mode=1, variant=1,
                                                  max_lr_diff=2, no_dupes=True)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_%dx%d_%s" % (
    c["n"], c["H"], c["W"], np.dtype(c["dt"]).name))
def test_cpp_match_branches_bit_exact(case, oracle, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    test_cpp_driver_is_built()
    n, H, W, dt, cfg = case["n"], case["H"], case["W"], case["dt"], case["cfg"]
    L, R = stereo_stack(n, H, W, dt)
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(np.array([n, H, W, np.dtype(dt).itemsize], np.int32).tobytes())
        f.write(np.ascontiguousarray(L).tobytes())
        f.write(np.ascontiguousarray(R).tobytes())
    g = lambda k, d: cfg.get(k, d)  # noqa: E731
    nxc = g("nxcorr_threshold", None)
    args = [EXE, str(inp), str(tmp_path / "out"), str(-1 if nxc is None else nxc),
            str(g("subpixel_step", None) or -1), str(-1 if g("min_variance", None) is None
                                                     else cfg["min_variance"]),
            str(g("mode", 0)), str(g("variant", 0)), str(g("max_lr_diff", 1)),
            str(int(g("no_dupes", False))), "0"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = dict(l.split(" ", 1) for l in r.stdout.strip().splitlines())
    assert lines["error_case"] == "need at least two images"
    rd, rc = oracle.match(L, R, oracle.OracleConfig(**cfg))
    for b in BRANCHES:
        assert b in lines, r.stdout
        mem = "host" if b in ("host", "mats", "seam") else "device"
        assert lines[b].endswith("mem=" + mem), lines[b]
        d = np.fromfile(tmp_path / ("out.%s.disp" % b), dtype=rd.dtype).reshape(H, W)
        assert np.array_equal(d.view(np.uint8), rd.view(np.uint8)), b
        cpath = tmp_path / ("out.%s.corr" % b)
        if rc is None:
            assert not cpath.exists(), b
        else:
            c = np.fromfile(cpath, dtype=rc.dtype).reshape(H, W)
            assert np.array_equal(c.view(np.uint8), rc.view(np.uint8)), b
