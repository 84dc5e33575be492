"""The compiled Asterisk-side shim: shim/fp_handler_tfp.c (hot half, over the C-ABI) +
shim/fp_catalog.c (the reference's SQLite catalog and audio_recongition.db backup), together the
reference's facade src/fp_handler.h:13-38, built with -pedantic -Werror against test stubs of the
Asterisk headers (tests/native/asterisk_stub) and driven from C by tests/native/shim_harness.c the
way the module calls it (application_handler.c:180-236, app_tiresias.c:365-424): enrolment, a
duplicate file, FOUND / NOTFOUND, bad coefs, a NULL context, delete, a restart that reloads the
index from the backup file; batched directory enrolment == the reference's file-by-file loop; and
backup files interchangeable with tiresias_amd/dbio.py's in both directions. Results equal the
oracle's search over the same rows."""
import json
import os
import subprocess
import wave

import numpy as np
import pytest

from conftest import PKG, REPO

SHIM_SRC = [os.path.join(REPO, "shim", "fp_handler_tfp.c"), os.path.join(REPO, "shim", "fp_catalog.c"),
            os.path.join(REPO, "tests", "native", "shim_harness.c")]
INC = ["-I" + os.path.join(REPO, d) for d in ("shim", "include", "tests/native/asterisk_stub")] + \
    ["-idirafter", "/opt/conda/include"]  # sqlite3.h (the image has libsqlite3.so.0 but no dev package)
LIBS = ["-l:libsqlite3.so.0", "-lcrypto", "-lm"]


def _build(tmp_path, tfp_lib):
    lib = os.path.dirname(tfp_lib.LIB_PATH)
    exe = str(tmp_path / "shim_driver")
    for src in SHIM_SRC[:2]:
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", *INC, "-c", src, "-o",
                        str(tmp_path / (os.path.basename(src) + ".o"))], check=True)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", *INC, *SHIM_SRC, "-o", exe, "-L" + lib,
                    "-ltiresias_fp", "-Wl,-rpath," + lib, *LIBS, "-lpthread"], check=True)
    return exe


def test_shim_compiles_and_links(tmp_path, tfp_lib):
    """-pedantic -Werror C99 build of the shim; every C-ABI symbol it calls resolves."""
    exe = _build(tmp_path, tfp_lib)
    out = subprocess.run(["nm", "-u", exe], capture_output=True, text=True, check=True).stdout
    used = {l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("tfp_")}
    assert {"tfp_group_create", "tfp_group_search_pcm_batch", "tfp_group_fingerprint_batch", "tfp_group_index_add",
            "tfp_group_index_add_batch", "tfp_wav_read", "tfp_host_alloc"} <= used
    assert used <= set(tfp_lib.header_symbols())


def _write_wav(path, pcm, channels=1, rate=8000):
    with wave.open(path, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(np.ascontiguousarray(pcm, np.int16).tobytes())


def _run(exe, snap, *cmd):
    r = subprocess.run([exe, snap, *cmd], capture_output=True, text=True, timeout=300)
    print(r.stderr[-4000:])  # (the module's ast_log lines, in the test's captured output)
    assert r.returncode == 0, r.stderr
    return [json.loads(l) for l in r.stdout.splitlines()]


@pytest.mark.gpu
def test_shim_end_to_end_vs_oracle(tmp_path, tfp_lib, oracle):
    exe = _build(tmp_path, tfp_lib)
    snap = str(tmp_path / "audio_recongition.db")
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

    uid = {}  # clip -> the uuid the module generated for it (random v4, fp_handler.c:1097-1109)

    def expect(live, key, tol):
        uu = [uid[c] for c in live]
        m1 = np.concatenate([rows[c][:, 0] for c in live])
        m2 = np.concatenate([rows[c][:, 1] for c in live])
        clip = np.concatenate([np.full(len(rows[c]), i) for i, c in enumerate(live)])
        _, qdb, _ = oracle.fingerprint(q[key])
        found, w, mc, fc = oracle.search(m1, m2, clip, uu, qdb[:, 0], qdb[:, 1], 1, tol, -1, -1)
        if not found:
            return {"TIRSTATUS": "NOTFOUND"}
        c = live[w]
        return {"TIRSTATUS": "FOUND", "TIRFRAMECOUNT": fc, "TIRMATCHCOUNT": mc, "TIRFILEUUID": uid[c],
                "TIRFILENAME": "clip%d.wav" % c, "TIRCONTEXT": "ctx"}

    cmd = ["init"]
    for f in files:
        cmd += ["enroll", "ctx", f]
    cmd += ["enroll", "ctx", files[0]]  # already enrolled: true, nothing added
    out = _run(exe, snap, *(cmd + ["lists", "term"]))
    assert out[0] == {"init": True}
    assert all(o["ok"] for o in out[1:8]) and len(out[1:8]) == 7
    lists = out[8]["audio_lists"]
    assert len(lists) == nclips and all(a["context"] == "ctx" for a in lists)
    for a in lists:
        uid[int(a["name"][4:-4])] = a["uuid"]
    cmd = ["init"]
    for k in ("q2", "q4", "q5", "qn"):
        cmd += ["search", "ctx", qf[k], "1", "0.45", "-1", "-1"]
    cmd += ["search", "ctx", qf["q2"], "1", "-1", "-1", "-1"]      # dialplan default tolerance
    cmd += ["search", "ctx", qf["q2"], "3", "0.45", "-1", "-1"]    # bad coefs -> NULL
    cmd += ["search", "NULL", qf["q2"], "1", "0.45", "-1", "-1"]   # NULL context -> NULL
    cmd += ["search", "ctx", str(tmp_path / "missing.wav"), "1", "0.45", "-1", "-1"]
    cmd += ["delete", uid[4], "search", "ctx", qf["q4"], "1", "0.45", "-1", "-1", "term"]
    out = _run(exe, snap, *cmd)
    assert out[0] == {"init": True}
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
    assert {"delete": uid[4], "ok": True} in out
    assert sub(s[8]) == expect([0, 1, 2, 3, 5], "q4", 0.45)
    assert s[0]["TIRSTATUS"] == "FOUND"  # (which clip wins is the oracle's call, above)
    assert s[0]["TIRFILEHASH"] == __import__("hashlib").md5(open(files[int(s[0]["TIRFILENAME"][4:-4])], "rb")
                                                            .read()).hexdigest()
    assert out[-1] == {"term": True}
    # restart: fp_init rebuilds the GPU index from the backup
    out2 = _run(exe, snap, "init", "search", "ctx", qf["q2"], "1", "0.45", "-1", "-1", "search", "ctx", qf["q5"],
                "1", "0.45", "-1", "-1", "term")
    assert out2[0] == {"init": True}
    assert sub(out2[1]) == expect([0, 1, 2, 3, 5], "q2", 0.45)
    assert sub(out2[2]) == expect([0, 1, 2, 3, 5], "q5", 0.45)


def _db_rows_by_name(path):
    """{audio_list name: (context, hash, [(m1 REAL or None, m2 REAL or None) in frame order])}"""
    import sqlite3
    con = sqlite3.connect(path)
    out = {}
    for uuid, name, ctx, h in con.execute("select uuid, name, context, hash from audio_list"):
        rows = con.execute("select max1, max2 from audio_fingerprint where audio_uuid = ? order by frame_idx",
                           (uuid,)).fetchall()
        out[name] = (ctx, h, rows)
    con.close()
    return out


@pytest.mark.gpu
def test_shim_batched_directory_enrolment_equals_per_file(tmp_path, tfp_lib, oracle):
    """app_tiresias.c:365-424's scan of a context directory (alphasort): fp_create_audio_list_infos
    (one GPU batch per sample format, on a 3-engine device group) leaves the same catalog and
    audio_fingerprint rows and gives the oracle's search results, as fp_craete_audio_list_info file
    by file on one engine does, including a repeated file
    (already enrolled), a non-audio file (not enrolled), stereo (fp32 path) and 16 kHz audio."""
    exe = _build(tmp_path, tfp_lib)
    d = tmp_path / "dir"
    d.mkdir()
    n = 8000 * 6
    pcm = tfp_lib.synth_pcm(0x7153A1, range(7), n)
    for c in range(5):
        _write_wav(str(d / ("c%02d.wav" % c)), pcm[c])
    _write_wav(str(d / "c05_copy.wav"), pcm[1])                       # same bytes as c01: deduplicated
    st = np.stack([pcm[5], (pcm[5] // 3).astype(np.int16)], 1)
    _write_wav(str(d / "c06_stereo.wav"), st.reshape(-1), channels=2)
    _write_wav(str(d / "c07_16k.wav"), tfp_lib.synth_pcm(0x7153A1, [6], 16000 * 5)[0], rate=16000)
    (d / "c08_notes.txt").write_text("not audio")
    q = str(tmp_path / "q.wav")
    _write_wav(q, pcm[3, 256 * 30: 256 * 30 + 16000])
    res = {}
    for mode in ("enrolldir", "enrolldir1"):
        db = str(tmp_path / (mode + ".db"))
        # the batched run on a 3-engine group (shards on GPU 0), the per-file run on one engine
        devs = "0,0,0" if mode == "enrolldir" else "0"
        out = _run(exe, db, "devices", devs, "init", mode, "ctx", str(d), "search", "ctx", q, "1", "0.45", "-1", "-1",
                   "search", "ctx", q, "1", "0.001", "-1", "-1", "term")[1:]
        assert out[0] == {"init": True} and out[-1] == {"term": True}
        res[mode] = (out[1], [o for o in out if "TIRSTATUS" in o], _db_rows_by_name(db))
    b, f = res["enrolldir"], res["enrolldir1"]
    assert b[0]["ok"] == f[0]["ok"] == [True] * 8 + [False]
    assert b[0]["enrolled"] == 7
    # each run's searches == the oracle over the rows and (random) uuids that run's backup holds
    _, qdb, _ = oracle.fingerprint(np.asarray(pcm[3, 256 * 30: 256 * 30 + 16000]))
    for mode, tol, k in (("enrolldir", 0.45, 0), ("enrolldir", 0.001, 1), ("enrolldir1", 0.45, 0),
                         ("enrolldir1", 0.001, 1)):
        import sqlite3
        con = sqlite3.connect(str(tmp_path / (mode + ".db")))
        al = con.execute("select uuid, name from audio_list order by uuid").fetchall()
        m1, m2, cl = [], [], []
        for i, (u, _) in enumerate(al):
            for a, c in con.execute("select max1, max2 from audio_fingerprint where audio_uuid = ? order by frame_idx",
                                    (u,)):
                m1.append(-(2**31) if a is None else round(a * 1e6))
                m2.append(-(2**31) if c is None else round(c * 1e6))
                cl.append(i)
        con.close()
        found, w, mc, fc = oracle.search(np.array(m1), np.array(m2), np.array(cl), [u for u, _ in al], qdb[:, 0],
                                         qdb[:, 1], 1, tol, -1, -1)
        o = res[mode][1][k]
        assert (o["TIRSTATUS"] == "FOUND") == found
        if found:
            assert (o["TIRFILEUUID"], o["TIRFILENAME"], o["TIRMATCHCOUNT"], o["TIRFRAMECOUNT"]) == \
                (al[w][0], al[w][1], mc, fc), mode
    assert b[1][0]["TIRSTATUS"] == f[1][0]["TIRSTATUS"] == "FOUND"
    assert b[2] == f[2] and sorted(b[2]) == ["c%02d.wav" % c for c in range(5)] + ["c06_stereo.wav", "c07_16k.wav"]
    # the stored rows are the oracle's "%f" values
    _, _, micro = oracle.fingerprint(pcm[2])
    rows = b[2]["c02.wav"][2]
    assert len(rows) == len(micro)
    assert all((None if m == -(2**31) else round(r * 1e6)) == (None if m == -(2**31) else int(m))
               for (r, _), m in zip(rows, micro[:, 0]))


@pytest.mark.gpu
def test_shim_backup_interchangeable_with_dbio(tmp_path, tfp_lib):
    """A backup the C module writes (fp_term) loads through the Python mirror (FpHandler ->
    dbio.load_backup) with the same search results, and one the mirror writes loads through the
    C module (fp_init) with the same results."""
    exe = _build(tmp_path, tfp_lib)
    n = 8000 * 6
    pcm = tfp_lib.synth_pcm(0x7153A1, range(6), n)
    files = []
    for c in range(6):
        files.append(str(tmp_path / ("w%d.wav" % c)))
        _write_wav(files[-1], pcm[c])
    qs = []
    for i, c in enumerate((0, 2, 4, 5)):
        qs.append(str(tmp_path / ("q%d.wav" % i)))
        _write_wav(qs[-1], pcm[c, 256 * (5 + 7 * i): 256 * (5 + 7 * i) + 16000])

    def searches_c(db, enrol):
        cmd = ["init"]
        for f in enrol:
            cmd += ["enroll", "ctx", f]
        for q in qs:
            cmd += ["search", "ctx", q, "1", "0.45", "-1", "-1", "search", "ctx", q, "2", "0.3", "-1", "-1"]
        out = _run(exe, db, *(cmd + ["term"]))
        return [{k: v for k, v in o.items() if k != "file"} for o in out if "TIRSTATUS" in o]

    def searches_py(db, enrol):
        h = tfp_lib.FpHandler(0, backup_path=db)
        assert h.fp_init()
        for f in enrol:
            assert h.fp_craete_audio_list_info("ctx", f)
        out = []
        for q in qs:
            for coefs, tol in ((1, 0.45), (2, 0.3)):
                r = h.fp_search_fingerprint_info("ctx", q, coefs, tol, -1, -1)
                out.append({"TIRSTATUS": "NOTFOUND"} if r is None else
                           {"TIRSTATUS": "FOUND", "TIRFRAMECOUNT": r["frame_count"], "TIRMATCHCOUNT": r["match_count"],
                            "TIRFILEUUID": r["uuid"], "TIRFILENAME": r["name"], "TIRCONTEXT": r["context"],
                            "TIRFILEHASH": r["hash"]})
        assert h.fp_term()
        return out

    c_db = str(tmp_path / "c.db")
    c_first = searches_c(c_db, files)
    assert sum(o["TIRSTATUS"] == "FOUND" for o in c_first) >= 4
    assert searches_py(c_db, []) == c_first          # C writes, Python reads
    py_db = str(tmp_path / "py.db")
    py_first = searches_py(py_db, files)
    py_uuids = {o["TIRFILENAME"]: o["TIRFILEUUID"] for o in py_first if o["TIRSTATUS"] == "FOUND"}
    assert searches_c(py_db, []) == py_first         # Python writes, C reads
    assert py_uuids  # (the two enrolments drew different random uuids, so their tie-breaks may differ)


@pytest.mark.gpu
def test_shim_64_channel_threads_equal_serial(tmp_path, tfp_lib):
    """The module's channel threads (application_handler.c:66 runs tiresias_exec per channel; each
    calls fp_search_fingerprint_info, :180) on one shared module (fp_handler.c:1161-1169): 64 threads
    x 6 searches at once through the shim on a 3-engine group ("0,0,0"), over 12 recordings, at the
    dialplan's coefs 1 and at coefs 2. Every result == the same file's serial search, and the calls
    ran coalesced (fewer GPU batches than calls: tfp_group_search_pcm_batch's coalescer)."""
    exe = _build(tmp_path, tfp_lib)
    db = str(tmp_path / "p.db")
    n = 8000 * 8
    pcm = tfp_lib.synth_pcm(0x7153A1, range(16), n)
    files = []
    for c in range(16):
        files.append(str(tmp_path / ("e%02d.wav" % c)))
        _write_wav(files[-1], pcm[c])
    qf = []
    for i in range(12):
        qf.append(str(tmp_path / ("q%02d.wav" % i)))
        q = pcm[i % 16, 256 * (3 + 5 * i): 256 * (3 + 5 * i) + 24000] if i % 4 != 3 else \
            tfp_lib.synth_pcm(0x7153B2, [i], 24000)[0]
        _write_wav(qf[-1], q)
    cmd = ["devices", "0,0,0", "init"]
    for f in files:
        cmd += ["enroll", "ctx", f]
    for coefs, tol in ((1, "0.45"), (2, "0.3")):
        for f in qf:
            cmd += ["search", "ctx", f, str(coefs), tol, "-1", "-1"]
        cmd += ["psearch", "64", "6", "ctx", str(coefs), tol, "-1", "-1", str(len(qf)), *qf]
    out = _run(exe, db, *(cmd + ["term"]))
    serial = [o for o in out if "TIRSTATUS" in o]
    par = [o for o in out if "psearch" in o]
    assert len(serial) == 24 and len(par) == 2
    for k, ps in enumerate(par):
        want = {}
        for i, o in enumerate(serial[12 * k: 12 * k + 12]):
            want[i] = (o["TIRSTATUS"] == "FOUND", o.get("TIRFILEUUID", ""), o.get("TIRMATCHCOUNT", 0),
                       o.get("TIRFRAMECOUNT", 0))
        assert sum(v[0] for v in want.values()) >= 6
        assert len(ps["results"]) == 64 * 6
        for fi, found, uuid, mc, fc in ps["results"]:
            assert (bool(found), uuid, mc, fc) == want[fi], (k, fi)
        assert ps["calls"] == 64 * 6 and ps["batches"] < ps["calls"], ps  # coalesced


@pytest.mark.gpu
def test_shim_live_channel_equals_recorded_file_search(tmp_path, tfp_lib, oracle):
    """fp_channel_* (the dialplan's record loop, application_handler.c:248-312, without the /tmp
    WAV): a call's audio pushed as 160-sample SLIN frames (plus a 7-sample tail frame), then searched,
    == fp_search_fingerprint_info on the recorded file (application_handler.c:180) == the oracle
    over the enrolled rows; a ring kept shorter than the call (max_ms 2000 of a 3.02 s call) == the
    search of a file holding its last 2 s."""
    exe = _build(tmp_path, tfp_lib)
    db = str(tmp_path / "c.db")
    n = 8000 * 8
    pcm = tfp_lib.synth_pcm(0x7153A1, range(8), n)
    files = []
    for c in range(8):
        files.append(str(tmp_path / ("e%d.wav" % c)))
        _write_wav(files[-1], pcm[c])
    calls, tails = [], []
    for i in range(5):
        src = pcm[i % 8, 256 * (4 + 9 * i): 256 * (4 + 9 * i) + 24167] if i != 4 else \
            tfp_lib.synth_pcm(0x7153B2, [3], 24167)[0]
        calls.append(str(tmp_path / ("call%d.wav" % i)))
        _write_wav(calls[-1], src)
        tails.append(str(tmp_path / ("tail%d.wav" % i)))
        _write_wav(tails[-1], src[-16000:])
    cmd = ["init"]
    for f in files:
        cmd += ["enroll", "ctx", f]
    for f, t in zip(calls, tails):
        for coefs, tol in (("1", "0.45"), ("2", "0.3"), ("1", "-1")):
            cmd += ["search", "ctx", f, coefs, tol, "-1", "-1", "chan", "ctx", f, "160", "3500", coefs, tol, "-1", "-1"]
        cmd += ["search", "ctx", t, "1", "0.45", "-1", "-1", "chan", "ctx", f, "160", "2000", "1", "0.45", "-1", "-1"]
    out = _run(exe, db, *(cmd + ["lists", "term"]))
    res = [o for o in out if "TIRSTATUS" in o]
    assert len(res) == 5 * 8
    for k in range(0, len(res), 2):
        a, b = dict(res[k]), dict(res[k + 1])
        assert b.pop("file").startswith("chan:") and a.pop("file")
        assert a == b, (k, a, b)
    assert sum(o["TIRSTATUS"] == "FOUND" for o in res) >= 10
    # the oracle on the first call at coefs 1, tolerance 0.45
    lists = next(o for o in out if "audio_lists" in o)["audio_lists"]
    uid = {int(a["name"][1:-4]): a["uuid"] for a in lists}
    rows = [oracle.fingerprint(pcm[c])[2] for c in range(8)]
    _, qdb, _ = oracle.fingerprint(pcm[0, 256 * 4: 256 * 4 + 24167])
    found, w, mc, fc = oracle.search(np.concatenate([r[:, 0] for r in rows]), np.concatenate([r[:, 1] for r in rows]),
                                     np.repeat(np.arange(8), len(rows[0])), [uid[c] for c in range(8)], qdb[:, 0],
                                     qdb[:, 1], 1, 0.45, -1, -1)
    o = res[1]
    assert (o["TIRSTATUS"] == "FOUND") == found
    if found:
        assert (o["TIRFILEUUID"], o["TIRMATCHCOUNT"], o["TIRFRAMECOUNT"]) == (uid[w], mc, fc)
