"""include/tiresias_fp.h from plain C: tests/native/abi_c_consumer.c builds with
`gcc -std=c99 -pedantic -Wall -Werror` against the header and links libtiresias_fp.so, the way
the reference's fp_handler.c shim would. Host entry points run anywhere; the
GPU run enrols, fingerprints and searches through the C-ABI and is checked against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

SRC = os.path.join(REPO, "tests", "native", "abi_c_consumer.c")
LIBDIR = os.path.join(REPO, "asterisk-tiresias_amd", "lib")


def _build(tmp_path, tfp_lib):
    exe = str(tmp_path / "abi_c_consumer")
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O1",
                    "-I" + os.path.join(REPO, "include"), SRC, "-o", exe, "-L" + LIBDIR, "-ltiresias_fp",
                    "-Wl,-rpath," + LIBDIR], check=True)
    return exe


def test_c99_consumer_builds_and_runs_host_calls(tmp_path, tfp_lib):
    exe = _build(tmp_path, tfp_lib)
    out = subprocess.run([exe, "host"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    first = int(out.stdout.split("first sample")[1])
    assert first == int(tfp_lib.synth_pcm(7, [3], 1024)[0, 0])


@pytest.mark.gpu
def test_c99_consumer_end_to_end_matches_oracle(tmp_path, tfp_lib, oracle):
    exe = _build(tmp_path, tfp_lib)
    binf = str(tmp_path / "out.bin")
    out = subprocess.run([exe, "gpu", binf], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    raw = open(binf, "rb").read()
    nq = int(np.frombuffer(raw[:8], np.int64)[0])
    frames = np.frombuffer(raw[8:8 + 32 * nq], tfp_lib.FRAME_DTYPE)
    res = raw[8 + 32 * nq:]
    found, match_count, frame_count, clip_id = np.frombuffer(res[:16], np.int32)
    uuid = res[16:80].split(b"\0")[0].decode()

    nclips, ns, qn, qoff = 8, 8000 * 6, 8000 * 3, 4096
    pcm = tfp_lib.synth_pcm(0xC0FFEE, range(nclips), ns)
    q = pcm[5, qoff:qoff + qn]
    _, qdb, qmicro = oracle.fingerprint(q)
    assert np.array_equal(frames["m1"], qmicro[:, 0]) and np.array_equal(frames["m2"], qmicro[:, 1])
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * ns, want_db=False)
    nf = (ns + 255) // 256
    uuids = ["00000000-0000-4000-8000-%012d" % c for c in range(nclips)]
    ok, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], np.repeat(np.arange(nclips), nf), uuids,
                                  qdb[:, 0], qdb[:, 1], 1, 0.5)
    assert (bool(found), int(frame_count)) == (ok, fc)
    if ok:
        assert (uuid, int(match_count)) == (uuids[w], mc)
