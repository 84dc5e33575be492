"""The 8 kHz kernel's sqrt sequence (asterisk-tiresias_amd/csrc/tfp_split.hpp: sqrt_pair_cr), run by
tests/native/check_fast_sqrt.hip on this GPU over every non-negative finite float: bitwise equal to
the correctly rounded sqrtf (glibc / SSE sqrtss, pinned on a strided host sample) for x = 0 and
x in [2^-100, 2^100), and the kernel's rare-bin flag raised exactly for 0 < x < 2^-98."""
import os
import subprocess

import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu


def test_fast_sqrt_exhaustive():
    exe = os.path.join(PKG, "bin", "check_fast_sqrt")
    assert os.path.exists(exe), "build with make -C asterisk-tiresias_amd"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fast_mismatch 0, zero_bad 0, rare_missed 0, rare_spurious 0;" in r.stdout


def test_band_log_exhaustive():
    """The throughput kernel's band log (csrc/tfp_log.hpp: v_frexp reduction, 64-entry (invc, y0)
    table) == aubio_log10_fast (aubio's clamped glibc log10f, tests/native/check_math.cpp) on every
    non-negative finite float, both on this GPU (tests/native/check_log_fast.hip)."""
    exe = os.path.join(PKG, "bin", "check_log_fast")
    assert os.path.exists(exe), "build with make -C asterisk-tiresias_amd"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "aubio_log10_fast on 0\n" in r.stdout
