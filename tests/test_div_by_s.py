"""div_by_S (pf_kernels.hpp, k_resample's normalised cumulative weights) equals IEEE fp64 division: the C restatement
in tests/div_by_s_check.c, built with gcc (-ffp-contract=off, libm fma), over 10^7 cases of the shapes k_resample
divides (quotients in [0, 1]; sums on the 2^-21 grid of fp32 scores; numerators just below S)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not found")
def test_div_by_s_matches_ieee(tmp_path):
    exe = tmp_path / "div_by_s_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(HERE, "div_by_s_check.c"), "-lm"],
                   check=True)
    r = subprocess.run([str(exe), "10000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
