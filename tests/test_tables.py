"""The product's host-built DSP tables (csrc/tfp_tables.cpp) equal the oracle's, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO


@pytest.mark.parametrize("sr", [8000, 16000, 44100])
def test_product_tables_equal_oracle(oracle, tmp_path, sr):
    exe = str(tmp_path / "dump")
    src = os.path.join(REPO, "tests", "native", "dump_tables.cpp")
    tab = os.path.join(REPO, "asterisk-tiresias_amd", "csrc", "tfp_tables.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin", src, tab, "-o", exe], check=True)
    out = str(tmp_path / "t.bin")
    sizes = subprocess.run([exe, str(sr), out], check=True, capture_output=True, text=True).stdout.split()
    raw = open(out, "rb").read()
    nt = int(sizes[0])
    f = np.frombuffer(raw[:nt], np.uint8)
    window = np.frombuffer(f[:2048].tobytes(), np.float32)
    o = 2048
    tw256_re = np.frombuffer(f[o:o + 1024].tobytes(), np.float32); o += 1024
    tw256_im = np.frombuffer(f[o:o + 1024].tobytes(), np.float32); o += 1024
    tw512_re = np.frombuffer(f[o:o + 1028].tobytes(), np.float32); o += 1028
    tw512_im = np.frombuffer(f[o:o + 1028].tobytes(), np.float32); o += 1028
    dct = np.frombuffer(f[o:o + 320].tobytes(), np.float32).reshape(2, 40)
    mel = np.frombuffer(raw[nt:], np.float32).reshape(40, 257)

    t = oracle.tables(sr)
    as_ = lambda a: np.ctypeslib.as_array(a).view(np.uint32)
    assert np.array_equal(window.view(np.uint32), as_(t.window))
    assert np.array_equal(tw256_re.view(np.uint32), as_(t.tw256_re))
    assert np.array_equal(tw256_im.view(np.uint32), as_(t.tw256_im))
    assert np.array_equal(tw512_re.view(np.uint32), as_(t.tw512_re))
    assert np.array_equal(tw512_im.view(np.uint32), as_(t.tw512_im))
    assert np.array_equal(dct.view(np.uint32), np.ctypeslib.as_array(t.dct).reshape(2, 40).view(np.uint32))
    assert np.array_equal(mel.view(np.uint32), np.ctypeslib.as_array(t.mel).reshape(40, 257).view(np.uint32))


def test_frame_pair_schedule_8k(tmp_path):
    """The throughput kernel's frame-pair filterbank schedule (csrc/tfp_tables.cpp
    build_fb_schedule) rebuilds every 8 kHz filter's dense row bit for bit, one job per filter."""
    exe = str(tmp_path / "fb")
    src = os.path.join(REPO, "tests", "native", "check_fb_schedule.cpp")
    tab = os.path.join(REPO, "asterisk-tiresias_amd", "csrc", "tfp_tables.cpp")
    inc = os.path.join(REPO, "asterisk-tiresias_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin", "-I", inc, src, tab, "-o", exe],
                   check=True)
    r = subprocess.run([exe, "8000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK: 34 filters")
