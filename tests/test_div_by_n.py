"""nxc::div_by_n (libbicos_amd/csrc/nxc.hpp) replaces the correctly rounded division of the
per-step subpixel mean: the exhaustive CPU check over every (integer sum, n) it is used on
must find no difference from IEEE division."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_div_by_n_is_correctly_rounded(tmp_path):
    exe = str(tmp_path / "div_by_n_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tools", "div_by_n_check.c"), "-lm"], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
    assert out.strip().endswith("bad 0"), out


def test_agree_window_plane_division_is_exact():
    """agree_win_kernel (kernels.hip) splits a flat window index i over [plane][dword] with
    plane = (i * ceil(2^16 / nd)) >> 16: exact for every window width nd <= 20 and index
    i < 33 * 20 it is used with."""
    for nd in range(1, 21):
        rcp = (65536 + nd - 1) // nd
        for i in range(33 * 20):
            assert (i * rcp) >> 16 == i // nd, (nd, i)
