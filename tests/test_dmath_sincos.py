"""d_sincosf (rt_dmath.h) against d_sinf / d_cosf, bit for bit: the kernels' fused sin/cos must not change any
sample.  The device math is IEEE f32 without contraction, so tools/check_sincos.cpp builds it for
the host.  Here: every float within 2^16 ulps of the range-reduction boundaries (0, the octants k*pi/4 up to 2pi,
8192, inf, both signs) and every 97th bit pattern of the 2^32 (all of them took 5.5 minutes once: 0 mismatches)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sincos_matches_separate_calls(tmp_path):
    exe = str(tmp_path / "check_sincos")
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-DRT_DMATH_HOST_TEST",
                           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(ROOT, "tools", "check_sincos.cpp"), "-o", exe])
    out = subprocess.run([exe, "97"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().startswith("0 mismatches"), out.stdout
