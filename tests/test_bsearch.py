"""csrc/tfp_bsearch.hpp (the coefs=2 sweep's bucket searches, tfp_scan.hip find_ab: both ends of a
bucket read with the first probe) vs std::lower_bound / std::upper_bound, compiled for the host."""
import os
import subprocess

from conftest import REPO


def test_bucket_searches(tmp_path):
    exe = str(tmp_path / "check_bsearch")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(REPO, "tests", "native", "check_bsearch.cpp"), "-o", exe],
                   check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert " 0 / " in out.stdout and out.stdout.strip().endswith("OK")
