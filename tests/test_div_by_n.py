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

