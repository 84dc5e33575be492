"""The catalog half of the shim (shim/fp_catalog.c) on the CPU: the reference's SQLite catalog and
audio_recongition.db backup (src/fp_handler.c:68-108, :479-530, :559-571, :673-756, :758-805,
:832-855, :912-1095; src/db_ctx_handler.c:413-556, :673-772), driven from C by
tests/native/catalog_harness.c.

  * the backup file holds the reference's DDL text, byte for byte;
  * audio_fingerprint rows are REALs parsed from the "%f" text (NULL for absent keys), so the
    file equals what the reference's per-frame INSERTs write;
  * fp_create_hash == MD5 of the file; per-context dedup; basename as the audio_list name;
  * files written by the C catalog load through tiresias_amd/dbio.py and the reverse, row for row;
  * context delete removes the context's audio lists and their fingerprint rows.
"""
import json
import hashlib
import os
import sqlite3
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO

import sys
sys.path.insert(0, PKG)
from tiresias_amd import dbio  # noqa: E402

NULL = -(2**31)


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cat") / "catalog_driver")
    inc = ["-I" + os.path.join(REPO, d) for d in ("shim", "include", "tests/native", "tests/native/asterisk_stub")]
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", *inc, "-idirafter", "/opt/conda/include",
                    "-c", os.path.join(REPO, "shim", "fp_catalog.c"), "-o", out + ".o"], check=True)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", *inc, "-idirafter", "/opt/conda/include",
                    os.path.join(REPO, "shim", "fp_catalog.c"), os.path.join(REPO, "tests", "native", "catalog_harness.c"),
                    "-o", out, "-l:libsqlite3.so.0", "-lcrypto", "-lm"], check=True)
    return out


def run(driver, db, *cmd):
    r = subprocess.run([driver, db, *cmd], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return [json.loads(l) for l in r.stdout.splitlines()]


def rows_bin(path, m1, m2):
    np.concatenate([np.asarray(m1, np.int32), np.asarray(m2, np.int32)]).tofile(path)
    return path


def _clip_rows(rng, n):
    m1 = rng.integers(-40_000_000, 40_000_000, n).astype(np.int32)
    m2 = rng.integers(-40_000_000, 40_000_000, n).astype(np.int32)
    m1[rng.random(n) < 0.05] = NULL
    m2[rng.random(n) < 0.05] = NULL
    m1[:4] = [0, -1, 999_999, -1_000_001]  # zero, -0.000001, rounding digits
    m2[:4] = [1, 17_000_000, NULL, -999_999]
    return m1, m2


def test_backup_file_is_the_reference_schema_and_rows(driver, tmp_path):
    rng = np.random.default_rng(3)
    db = str(tmp_path / "audio_recongition.db")
    files = []
    for k in range(3):
        f = tmp_path / ("f%d.wav" % k)
        f.write_bytes(rng.bytes(1000 + k))
        files.append(str(f))
    clips = {("u%d" % k): _clip_rows(rng, 50 + 10 * k) for k in range(3)}
    cmd = ["init", "ctx", "sales", str(tmp_path)]
    for k, f in enumerate(files):
        cmd += ["create", "sales", f, "u%d" % k]
    cmd += ["create", "sales", files[1], "dup"]   # same hash, same context: already enrolled
    cmd += ["create", "other", files[1], "u9"]    # another context: a new row
    for u, (m1, m2) in clips.items():
        cmd += ["store", "sales", u, rows_bin(str(tmp_path / (u + ".bin")), m1, m2)]
    cmd += ["term"]
    out = run(driver, db, *cmd)
    assert [o.get("create") for o in out if "create" in o] == [1, 1, 1, 0, 1]
    assert all(o["store"] for o in out if "store" in o) and out[-1] == {"term": True}

    con = sqlite3.connect(db)
    ddl = [r[0] for r in con.execute("select sql from sqlite_master where sql is not null order by rowid")]
    # the reference's statements (fp_handler.c:686-753) as SQLite keeps them
    assert ddl == [s.rstrip(";").replace("create table", "CREATE TABLE").replace("create index", "CREATE INDEX")
                   for s in dbio.SCHEMA]
    al = con.execute("select uuid, name, context, hash from audio_list order by rowid").fetchall()
    md5 = [hashlib.md5(open(f, "rb").read()).hexdigest() for f in files]
    assert al == [("u0", "f0.wav", "sales", md5[0]), ("u1", "f1.wav", "sales", md5[1]),
                  ("u2", "f2.wav", "sales", md5[2]), ("u9", "f1.wav", "other", md5[1])]
    for u, (m1, m2) in clips.items():
        got = con.execute("select frame_idx, typeof(max1), max1, typeof(max2), max2, context from audio_fingerprint"
                          " where audio_uuid = ? order by rowid", (u,)).fetchall()
        assert [g[0] for g in got] == list(range(len(m1)))
        for (fi, t1, v1, t2, v2, ctx), a, b in zip(got, m1, m2):
            assert ctx == "sales"
            for t, v, m in ((t1, v1, a), (t2, v2, b)):
                if m == NULL:
                    assert t == "null" and v is None
                else:  # the REAL SQLite parses from the reference's "%f" literal
                    lit = con.execute("select %s" % dbio.micro_text(m)).fetchone()[0]
                    assert t == "real" and v == lit, (u, fi, m, v, lit)
    con.close()

    # fp_init of that file: the same rows back, grouped by clip
    out = run(driver, db, "init", "load", "close")
    loaded = {c["uuid"]: (c["m1"], c["m2"]) for c in out[1]["clips"]}
    assert set(loaded) == set(clips)
    for u, (m1, m2) in clips.items():
        assert loaded[u] == (m1.tolist(), m2.tolist())


class _Rows:
    """The part of the engine dbio.py talks to: index_add_batch / index_rows."""

    def __init__(self, rows=None):
        self.rows = dict(rows or {})

    def index_add_batch(self, uuids, foff, m1, m2):
        for i, u in enumerate(uuids):
            self.rows[u] = (np.asarray(m1[foff[i]:foff[i + 1]]).tolist(), np.asarray(m2[foff[i]:foff[i + 1]]).tolist())

    def index_rows(self, uuid):
        return self.rows[uuid]


def test_interop_with_dbio_both_ways(driver, tmp_path):
    rng = np.random.default_rng(4)
    clips = {("%08x-0000-4000-8000-%012d" % (k * 7919, k)): _clip_rows(rng, 40 + k) for k in range(5)}
    # C catalog writes -> dbio loads
    db1 = str(tmp_path / "c.db")
    cmd = ["init", "ctx", "c", str(tmp_path)]
    for k, (u, (m1, m2)) in enumerate(clips.items()):
        f = tmp_path / ("a%d.wav" % k)
        f.write_bytes(rng.bytes(500))
        cmd += ["create", "c", str(f), u, "store", "c", u, rows_bin(str(tmp_path / ("r%d.bin" % k)), m1, m2)]
    run(driver, db1, *(cmd + ["term"]))
    mem = sqlite3.connect(":memory:")
    dbio.create_catalog(mem)
    eng = _Rows()
    n = dbio.load_backup(mem, eng, db1)
    assert n["clips"] == 5 and n["audios"] == 5 and n["contexts"] == 1
    assert eng.rows == {u: (m1.tolist(), m2.tolist()) for u, (m1, m2) in clips.items()}
    # dbio writes -> C catalog loads (and keeps the catalog rows)
    db2 = str(tmp_path / "py.db")
    dbio.write_backup(mem, eng, db2)
    out = run(driver, db2, "init", "load", "lists", "close")
    assert {c["uuid"]: (c["m1"], c["m2"]) for c in out[1]["clips"]} == eng.rows
    assert sorted(a["uuid"] for a in out[2]["audio_lists"]) == sorted(clips)
    assert out[2]["context_lists"] == [{"name": "c", "directory": str(tmp_path)}]


def test_delete_and_context_delete(driver, tmp_path):
    rng = np.random.default_rng(5)
    db = str(tmp_path / "d.db")
    cmd = ["init", "ctx", "a", str(tmp_path), "ctx", "b", str(tmp_path)]
    for k, ctx in enumerate(["a", "a", "b"]):
        f = tmp_path / ("x%d.wav" % k)
        f.write_bytes(rng.bytes(300 + k))
        m1, m2 = _clip_rows(rng, 20)
        cmd += ["create", ctx, str(f), "v%d" % k, "store", ctx, "v%d" % k, rows_bin(str(tmp_path / ("x%d.bin" % k)), m1, m2)]
    cmd += ["delete", "v0", "delete", "v0", "ctxdel", "b", "ctxdel", "zz", "lists", "load", "term"]
    out = run(driver, db, *cmd)
    dels = [o for o in out if "delete" in o or "ctxdel" in o]
    assert dels == [{"delete": True}, {"delete": False}, {"ctxdel": True}, {"ctxdel": False}]
    lists = [o for o in out if "audio_lists" in o][0]
    assert [a["uuid"] for a in lists["audio_lists"]] == ["v1"]
    assert [c["name"] for c in lists["context_lists"]] == ["a"]
    assert [c["uuid"] for c in [o for o in out if "load" in o][0]["clips"]] == ["v1"]


def test_hash_and_uuid(driver, tmp_path):
    f = tmp_path / "h.bin"
    f.write_bytes(bytes(range(256)) * 300)
    out = run(driver, str(tmp_path / "n.db"), "hash", str(f), "hash", str(tmp_path / "missing"), "uuid", "uuid")
    assert out[0]["hash"] == hashlib.md5(f.read_bytes()).hexdigest()
    assert out[1]["hash"] == ""
    import uuid
    us = [uuid.UUID(o["uuid"]) for o in out[2:]]
    assert all(u.version == 4 and u.variant == uuid.RFC_4122 for u in us) and us[0] != us[1]
    assert all(str(u) == o["uuid"] for u, o in zip(us, out[2:]))


def test_json_shaped_text_reads_back_as_the_reference_does(driver, tmp_path):
    """db_ctx_get_record (db_ctx_handler.c:311-333) loads every TEXT column with
    ast_json_load_string (jansson json_loads, flags 0: an array or object at the top) and keeps an
    array / object / string result, else the text as a string. A context whose name and directory
    are JSON text come back in the listings as the parsed values; other text, a JSON string literal
    included, comes back as the text itself."""
    db = str(tmp_path / "j.db")
    out = run(driver, db, "init", "ctx", '{"a": [1, "x"]}', '["d1", "d2"]', "ctx", '"quoted"', "plain dir",
              "ctx", "[1, 2", "{}", "lists", "term")
    ctx = [o for o in out if "context_lists" in o][0]["context_lists"]
    byname = {json.dumps(c["name"], sort_keys=True): c for c in ctx}
    assert set(byname) == {json.dumps({"a": [1, "x"]}, sort_keys=True), json.dumps('"quoted"'), json.dumps("[1, 2")}
    assert byname[json.dumps({"a": [1, "x"]}, sort_keys=True)]["directory"] == ["d1", "d2"]
    assert byname[json.dumps('"quoted"')]["directory"] == "plain dir"
    assert byname[json.dumps("[1, 2")]["directory"] == {}
