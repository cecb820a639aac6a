"""The receiver back-end's lean fp64 sin/cos and atan2 (csrc/be_math.h, used by
rx_backend_fast_kernel in place of ocml's) against glibc, on the host: the header is compiled with
g++ and checked over the argument ranges the kernel sees (window tones up to |x| = pi·2^31, channel
estimates' phases) plus signed zeros and axes.  Bar: 1 ulp for atan2; for sin/cos 1.1e-16 absolute (2 ulp next to
a zero of sin/cos) (the kernel's end-to-end parity with the
oracle is tests/test_gpu_parity.py::test_receiver_backend_batched_vs_oracle)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_lean_sincos_atan2_within_one_ulp_of_libm(tmp_path):
    exe = tmp_path / "be_math_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "ofdm-sync-math_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "be_math_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    rows = [ln.split() for ln in out.strip().splitlines()]
    seen = set()
    for r in rows:
        seen.add(r[0])
        if r[0] == "sincos":
            assert float(r[2]) <= 2.0 and float(r[3]) <= 2.0, r      # 2 ulp only next to a zero of sin/cos
            assert float(r[4]) <= 2.3e-16 and float(r[5]) <= 2.3e-16, r
        else:
            assert float(r[2]) <= 1.0, r
    assert seen == {"sincos", "atan2", "atan2_special"}
