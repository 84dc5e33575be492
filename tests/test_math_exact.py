"""csrc/tfp_math.hpp (the exact log10f / log10 / %f used by the kernels) vs this host's glibc.

The same IEEE-only source runs on the GPU; here it is compiled for the host and compared with
glibc (what libaubio and fp_handler.c call) — sampled in CI, exhaustively by hand (the log of
the exhaustive run over all 2,139,095,039 positive floats is tests/native/check_math_exhaustive.log).
"""
import os
import subprocess

from conftest import REPO

NATIVE = os.path.join(REPO, "tests", "native")


def test_math_sampled(tmp_path):
    exe = str(tmp_path / "check_math")
    subprocess.run(["g++", "-O2", "-std=c++20", "-ffp-contract=off", "-fopenmp", os.path.join(NATIVE, "check_math.cpp"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe, "9973"], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert "0 fmt6 mismatches, 0 trunc mismatches" in out.stdout


def test_exhaustive_log_committed():
    log = open(os.path.join(NATIVE, "check_math_exhaustive.log")).read()
    assert "log10f_glibc vs glibc log10f : 0 / 2139095039 mismatches" in log
    assert "2139095039 floats" in log and "0 fmt6 mismatches, 0 trunc mismatches" in log
    assert "aubio_log10_fast vs aubio_log10_clamped : 0 / 2139095041 mismatches" in log
    assert log.strip().endswith("OK")


def test_logfix_sampled(tmp_path):
    """The frame values with the LogFix table == glibc's 10*log10|c| (sampled; the exhaustive
    run over every positive float is tests/native/check_logfix_exhaustive.log)."""
    exe = str(tmp_path / "check_logfix")
    subprocess.run(["g++", "-O2", "-std=c++20", "-ffp-contract=off", "-fno-builtin", "-fopenmp",
                    os.path.join(NATIVE, "check_logfix.cpp"),
                    os.path.join(REPO, "asterisk-tiresias_amd", "csrc", "tfp_tables.cpp"), "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe, "997"], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0 and out.stdout.strip().endswith("OK"), out.stdout
    assert "hashed LogFix vs sorted over the 2^24 key domain: 0 mismatches" in out.stdout


def test_logfix_exhaustive_log_committed():
    log = open(os.path.join(NATIVE, "check_logfix_exhaustive.log")).read()
    assert "10*log10|c| with LogFix vs glibc : 0 / 2139095039 mismatches" in log
    assert log.strip().endswith("OK")
