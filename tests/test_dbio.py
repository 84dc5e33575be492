"""audio_recongition.db snapshot load/backup (dbio.py; fp_init/fp_term, fp_handler.c:68-108).

CPU tests drive the host logic with a stub engine: a DB written by the reference's own
INSERT path (oracle/sql_oracle.py restates it string for string) must load into exactly the
stored micro-unit rows, and a backup must hold the same REAL/NULL values the reference
would have stored. The GPU test closes the loop through the device index: enrol, back up,
reload in a fresh handler, and every search equals the reference SQL run on the file.
"""
import os
import sqlite3

import numpy as np
import pytest

from tiresias_amd import dbio
from tiresias_amd._lib import NULL_MICRO

from sql_oracle import SqlFingerprintDB  # noqa: E402  (oracle/ on sys.path via conftest)


class StubEngine:
    def __init__(self):
        self.clips = {}

    def index_add_batch(self, uuids, foff, m1, m2):
        for i, u in enumerate(uuids):
            assert u not in self.clips
            self.clips[u] = (np.array(m1[foff[i]:foff[i + 1]]), np.array(m2[foff[i]:foff[i + 1]]))

    def index_rows(self, uuid):
        if uuid not in self.clips:
            from tiresias_amd import TfpError
            raise TfpError(-4, uuid)
        return self.clips[uuid]


def _random_clips(rng, n):
    clips = {}
    for c in range(n):
        nf = int(rng.integers(0, 40))
        m1 = rng.integers(-450_000_000, 200_000_000, nf).astype(np.int32)
        m2 = rng.integers(-450_000_000, 200_000_000, nf).astype(np.int32)
        m1[rng.random(nf) < 0.1] = NULL_MICRO
        m2[rng.random(nf) < 0.1] = NULL_MICRO
        m1[rng.random(nf) < 0.05] = 0
        clips["%08x-0000-4000-8000-%012d" % (int(rng.integers(2**32)), c)] = (m1, m2)
    return clips


def _reference_file(path, clips):
    """What the reference's fp_term would leave: catalog + audio_fingerprint via its INSERTs."""
    ref = SqlFingerprintDB()
    for ddl in dbio.SCHEMA[:2]:
        ref.db.execute(ddl)
    ref.db.execute("insert into context_list values ('ctx', '/tmp/ctx')")
    for u, (m1, m2) in clips.items():
        ref.db.execute("insert into audio_list values (?, ?, 'ctx', 'h')", (u, u[:8] + ".wav"))
        ref.insert_rows("ctx", u, m1, m2)
    ref.db.commit()
    dst = sqlite3.connect(path)
    ref.db.backup(dst)  # page copy, like db_ctx_backup
    dst.close()


def _fp_rows(path):
    db = sqlite3.connect(path)
    rows = db.execute("select context, audio_uuid, frame_idx, max1, typeof(max1), max2, typeof(max2)"
                      " from audio_fingerprint order by audio_uuid, frame_idx").fetchall()
    db.close()
    return rows


def test_micro_text_roundtrips_through_sqlite_real_affinity():
    rng = np.random.default_rng(5)
    vals = np.concatenate([rng.integers(-(2**31) + 1, 2**31 - 1, 20000), [0, 1, -1, 999999, -999999, 10**6, -10**6]])
    db = sqlite3.connect(":memory:")
    db.execute("create table t(i integer, x real)")
    db.executemany("insert into t values (?, ?)", ((i, dbio.micro_text(v)) for i, v in enumerate(vals)))
    got = np.array(db.execute("select %s from t order by i" % dbio._MICRO_SQL.format(c="x")).fetchall())[:, 0]
    assert (got == vals).all()
    assert dbio.micro_text(NULL_MICRO) is None


def test_load_reference_written_file(tmp_path):
    rng = np.random.default_rng(11)
    clips = _random_clips(rng, 60)
    path = str(tmp_path / "audio_recongition.db")
    _reference_file(path, clips)
    cat = sqlite3.connect(":memory:")
    dbio.create_catalog(cat)
    eng = StubEngine()
    out = dbio.load_backup(cat, eng, path)
    nonempty = {u for u, (m1, _) in clips.items() if len(m1)}
    assert out["clips"] == len(nonempty) and out["audios"] == len(clips) and out["contexts"] == 1
    assert out["rows"] == sum(len(m1) for m1, _ in clips.values())
    assert set(eng.clips) == nonempty
    for u in nonempty:
        assert (eng.clips[u][0] == clips[u][0]).all() and (eng.clips[u][1] == clips[u][1]).all()
    assert cat.execute("select count(*) from audio_list").fetchone()[0] == len(clips)


def test_backup_equals_reference_file(tmp_path):
    rng = np.random.default_rng(12)
    clips = _random_clips(rng, 40)
    ref_path = str(tmp_path / "ref.db")
    _reference_file(ref_path, clips)
    cat = sqlite3.connect(":memory:")
    dbio.create_catalog(cat)
    eng = StubEngine()
    dbio.load_backup(cat, eng, ref_path)
    ours = str(tmp_path / "ours.db")
    out = dbio.write_backup(cat, eng, ours)
    assert out["rows"] == sum(len(m1) for m1, _ in clips.values())
    a, b = _fp_rows(ref_path), _fp_rows(ours)
    assert a == b  # same REAL bits, same NULLs, same frame_idx/context
    db = sqlite3.connect(ours)
    names = {r[0] for r in db.execute("select name from sqlite_master")}
    assert {"context_list", "audio_list", "audio_fingerprint", "idx_audio_fingerprint_max1"} <= names
    # second backup over an existing file replaces it
    dbio.write_backup(cat, eng, ours)
    assert _fp_rows(ours) == a


def test_missing_file_loads_nothing(tmp_path):
    cat = sqlite3.connect(":memory:")
    dbio.create_catalog(cat)
    assert dbio.load_backup(cat, StubEngine(), str(tmp_path / "none.db"))["rows"] == 0
    assert not os.path.exists(tmp_path / "none.db")


def test_non_numeric_rows_rejected(tmp_path):
    path = str(tmp_path / "bad.db")
    db = sqlite3.connect(path)
    for ddl in dbio.SCHEMA:
        db.execute(ddl)
    db.execute("insert into audio_fingerprint values ('c', 'u', 0, 'abc', 1.0)")
    db.commit()
    db.close()
    cat = sqlite3.connect(":memory:")
    dbio.create_catalog(cat)
    with pytest.raises(ValueError):
        dbio.load_backup(cat, StubEngine(), path)


@pytest.mark.gpu
def test_backup_reload_search_matches_reference_sql(oracle, tfp_lib, tmp_path):
    from tiresias_amd import FpHandler
    from tiresias_amd.fp_handler import write_wav_mono16
    nclips, n = 12, 8000 * 4
    pcm = tfp_lib.synth_pcm(0x5EED, range(nclips), n)
    path = str(tmp_path / "audio_recongition.db")
    h = FpHandler(backup_path=path)
    assert h.fp_init()
    assert h.fp_create_context_list_info("ctx", str(tmp_path), False)
    for c in range(nclips):
        f = str(tmp_path / f"clip{c}.wav")
        write_wav_mono16(f, pcm[c])
        assert h.fp_craete_audio_list_info("ctx", f)
    assert h.fp_term()

    # the backup holds exactly what the reference stores for these clips
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n, nthreads=4, want_db=False)
    db = sqlite3.connect(path)
    nf = (n + 255) // 256
    for u, name in db.execute("select uuid, name from audio_list").fetchall():
        c = int(name[len("clip"):-len(".wav")])
        rows = db.execute("select %s, %s from audio_fingerprint where audio_uuid = ? order by frame_idx"
                          % (dbio._MICRO_SQL.format(c="max1"), dbio._MICRO_SQL.format(c="max2")), (u,)).fetchall()
        assert (np.array(rows, np.int64).reshape(-1, 2) == micro[c * nf:(c + 1) * nf]).all(), name
    db.close()

    # reload into a fresh engine; search == the reference SQL over the same file
    h2 = FpHandler(backup_path=path)
    assert h2.fp_init()
    assert len(h2.fp_get_audio_lists_all()) == nclips
    ref = SqlFingerprintDB()
    src = sqlite3.connect(path)
    src.backup(ref.db)
    src.close()
    qs = [pcm[3][4096:4096 + 16000], pcm[7][:12000], tfp_lib.synth_pcm(0xABC, [0], 16000)[0]]
    for i, q in enumerate(qs):
        f = str(tmp_path / f"q{i}.wav")
        write_wav_mono16(f, q)
        _, qdb, _ = oracle.fingerprint(q)
        for coefs, tol in ((1, 0.001), (2, 0.5), (1, 2.0)):
            exp = ref.search([None if not np.isfinite(v) else float(v) for v in qdb[:, 0]],
                             [None if not np.isfinite(v) else float(v) for v in qdb[:, 1]], coefs, tol, -1, -1)
            got = h2.fp_search_fingerprint_info("ctx", f, coefs, tol, -1, -1)
            if exp is None:
                assert got is None, (i, coefs)
            else:
                assert got is not None and (got["uuid"], got["match_count"], got["frame_count"]) == \
                    (exp["audio_uuid"], exp["match_count"], exp["frame_count"]), (i, coefs)
    h2.fp_term(); os.remove(path)  # noqa: E702
