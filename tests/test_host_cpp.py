"""Host-side unit tests of the device code's shared headers (CPU, no GPU):
the Stockham FFT core (incl. the composite radix-6/9 stages of the 270-point
plan) against a long-double DFT, fast_log / fast_exp against long double, and
the C-library float32 powf / logf emulation bit for bit against this libm."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "beta-sgp_amd", "csrc")


@pytest.mark.parametrize("src", ["fft_core_test.cpp", "math_test.cpp", "libmf_test.cpp"])
def test_host_cpp(src, tmp_path):
    exe = tmp_path / src.replace(".cpp", "")
    # -ffp-contract=off: the same rounding as the gfx950 build
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(ROOT, "tests", "cpp", src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all ok" in out.stdout
