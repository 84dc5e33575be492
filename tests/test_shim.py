"""The compiled Asterisk-side shim (shim/fp_handler_tfp.c): the reference's facade
src/fp_handler.h:13-38 over the C-ABI, built with -pedantic -Werror against test stubs of the
Asterisk headers (tests/native/asterisk_stub) and driven from C by tests/native/shim_harness.c the
way the dialplan application calls it (src/application_handler.c:180-236): enrolment, a duplicate
file, FOUND / NOTFOUND, bad coefs, a NULL context, delete, and a restart that reloads the index
from the backup. Results equal the oracle's search over the same rows."""
import json
import os
import subprocess
import wave

import numpy as np
import pytest

from conftest import PKG, REPO

SHIM_SRC = [os.path.join(REPO, "shim", "fp_handler_tfp.c"), os.path.join(REPO, "tests", "native", "shim_harness.c")]
INC = ["-I" + os.path.join(REPO, d) for d in ("shim", "include", "tests/native/asterisk_stub")]


def _build(tmp_path, tfp_lib):
    lib = os.path.dirname(tfp_lib.LIB_PATH)
    exe = str(tmp_path / "shim_driver")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", *INC, "-c", SHIM_SRC[0], "-o",
                    str(tmp_path / "shim.o")], check=True)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", *INC, *SHIM_SRC, "-o", exe, "-L" + lib,
                    "-ltiresias_fp", "-Wl,-rpath," + lib], check=True)
    return exe


def test_shim_compiles_and_links(tmp_path, tfp_lib):
    """-pedantic -Werror C99 build of the shim; every C-ABI symbol it calls resolves."""
    exe = _build(tmp_path, tfp_lib)
    out = subprocess.run(["nm", "-u", exe], capture_output=True, text=True, check=True).stdout
    used = {l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("tfp_")}
    assert {"tfp_engine_create", "tfp_search_pcm_batch", "tfp_fingerprint_pcm", "tfp_index_add",
            "tfp_wav_read"} <= used
    assert used <= set(tfp_lib.header_symbols())


def _write_wav(path, pcm, channels=1, rate=8000):
    with wave.open(path, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(np.ascontiguousarray(pcm, np.int16).tobytes())


def _uuid(seq):
    return "%08x-0000-4000-8000-%012d" % ((seq * 2654435761) & 0xFFFFFFFF, seq)


def _run(exe, snap, *cmd):
    r = subprocess.run([exe, snap, *cmd], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return [json.loads(l) for l in r.stdout.splitlines()]


@pytest.mark.gpu
def test_shim_end_to_end_vs_oracle(tmp_path, tfp_lib, oracle):
    exe = _build(tmp_path, tfp_lib)
    snap = str(tmp_path / "snapshot.txt")
    n, nclips = 8000 * 8, 6
    pcm = tfp_lib.synth_pcm(0x7153A1, range(nclips), n)
    files = []
    for c in range(nclips):
        f = str(tmp_path / ("clip%d.wav" % c))
        if c == 5:  # stereo: the fp32 path (aubio's channel mean)
            st = np.stack([pcm[c], (pcm[c] // 2).astype(np.int16)], 1)
            _write_wav(f, st.reshape(-1), channels=2)
        else:
            _write_wav(f, pcm[c])
        files.append(f)
    # queries: excerpts of clips 2, 4, 5 and unrelated audio
    q = {"q2": pcm[2, 256 * 40: 256 * 40 + 24000], "q4": pcm[4, 256 * 10 + 77: 256 * 10 + 77 + 24000],
         "q5": pcm[5, 256 * 3: 256 * 3 + 24000],
         "qn": tfp_lib.synth_pcm(0x7153B2, [9], 24000)[0]}
    qf = {}
    for k, v in q.items():
        qf[k] = str(tmp_path / (k + ".wav"))
        _write_wav(qf[k], v)
    # oracle rows of what the shim enrols (the stereo file through aubio's fp32 channel mean)
    rows = {}
    for c in range(nclips):
        if c == 5:
            x = oracle.wav_mono_f32(np.stack([pcm[c], (pcm[c] // 2).astype(np.int16)], 1), 16)
            rows[c] = oracle.fingerprint_f32(x)[2]
        else:
            rows[c] = oracle.fingerprint(pcm[c])[2]

    def expect(live, key, tol):
        uu = [_uuid(c) for c in live]
        m1 = np.concatenate([rows[c][:, 0] for c in live])
        m2 = np.concatenate([rows[c][:, 1] for c in live])
        clip = np.concatenate([np.full(len(rows[c]), i) for i, c in enumerate(live)])
        _, qdb, _ = oracle.fingerprint(q[key])
        found, w, mc, fc = oracle.search(m1, m2, clip, uu, qdb[:, 0], qdb[:, 1], 1, tol, -1, -1)
        if not found:
            return {"TIRSTATUS": "NOTFOUND"}
        c = live[w]
        return {"TIRSTATUS": "FOUND", "TIRFRAMECOUNT": fc, "TIRMATCHCOUNT": mc, "TIRFILEUUID": _uuid(c),
                "TIRFILENAME": "clip%d.wav" % c, "TIRCONTEXT": "ctx"}

    cmd = ["init"]
    for f in files:
        cmd += ["enroll", "ctx", f]
    cmd += ["enroll", "ctx", files[0]]  # already enrolled: true, nothing added
    for k in ("q2", "q4", "q5", "qn"):
        cmd += ["search", "ctx", qf[k], "1", "0.45", "-1", "-1"]
    cmd += ["search", "ctx", qf["q2"], "1", "-1", "-1", "-1"]      # dialplan default tolerance
    cmd += ["search", "ctx", qf["q2"], "3", "0.45", "-1", "-1"]    # bad coefs -> NULL
    cmd += ["search", "NULL", qf["q2"], "1", "0.45", "-1", "-1"]   # NULL context -> NULL
    cmd += ["search", "ctx", str(tmp_path / "missing.wav"), "1", "0.45", "-1", "-1"]
    cmd += ["delete", _uuid(4), "search", "ctx", qf["q4"], "1", "0.45", "-1", "-1", "term"]
    out = _run(exe, snap, *cmd)
    assert out[0] == {"init": True}
    assert all(o["ok"] for o in out[1:8]) and len(out[1:8]) == 7
    s = [o for o in out if "TIRSTATUS" in o]
    live = list(range(nclips))

    def sub(o):
        return {k: v for k, v in o.items() if k not in ("file", "TIRFILEHASH")}
    assert sub(s[0]) == expect(live, "q2", 0.45)
    assert sub(s[1]) == expect(live, "q4", 0.45)
    assert sub(s[2]) == expect(live, "q5", 0.45)
    assert sub(s[3]) == expect(live, "qn", 0.45)
    assert sub(s[4]) == expect(live, "q2", 0.001)
    assert s[5]["TIRSTATUS"] == s[6]["TIRSTATUS"] == s[7]["TIRSTATUS"] == "NOTFOUND"
    assert {"delete": _uuid(4), "ok": True} in out
    assert sub(s[8]) == expect([0, 1, 2, 3, 5], "q4", 0.45)
    assert s[0]["TIRSTATUS"] == "FOUND"  # (which clip wins is the oracle's call, above)
    assert out[-1] == {"term": True}
    # restart: fp_init rebuilds the GPU index from the backup
    out2 = _run(exe, snap, "init", "search", "ctx", qf["q2"], "1", "0.45", "-1", "-1", "search", "ctx", qf["q5"],
                "1", "0.45", "-1", "-1", "term")
    assert out2[0] == {"init": True}
    assert sub(out2[1]) == sub(s[0])
    assert sub(out2[2]) == expect([0, 1, 2, 3, 5], "q5", 0.45)
