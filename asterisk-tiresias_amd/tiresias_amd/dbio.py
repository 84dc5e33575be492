"""audio_recongition.db snapshot load / backup straight to and from the GPU index.

The reference keeps its whole state in an in-memory SQLite DB (fp_handler.c:30,680) that
fp_init fills from the backup file (db_ctx_load_db_data, db_ctx_handler.c:750-772: ATTACH,
then `insert into main.T select * from backup.T` for every table, :827-841) and fp_term
page-copies back to it (db_ctx_backup, db_ctx_handler.c:673-717). Here the control-plane
tables (context_list, audio_list) stay in SQLite, and audio_fingerprint rows move between
the file and the engine's device index:

  * load: every stored max1/max2 REAL is the parse of the "%f" text the reference inserted
    (db_ctx_handler.c:478-481), so round(x * 1e6) recovers the exact micro-unit value the
    engine keys on; SQL NULL (a non-finite dB — jansson refuses the real, the column is
    left out of the INSERT, fp_handler.c:651) becomes TFP_NULL_MICRO.
  * backup: rows are written back as the same "%f" text into REAL-affinity columns, so
    SQLite parses them exactly as it parsed the reference's INSERT literals; the schema is
    the one init_database creates (fp_handler.c:686-753), so the file round-trips through
    the unmodified reference module as well.

Both directions are bulk: one tfp_index_add_batch upload for the whole table on load, one
tfp_index_rows read-back per clip on backup.
"""
from __future__ import annotations

import os
import sqlite3

import numpy as np

from ._lib import NULL_MICRO

DEF_BACKUP_DATABASE = "/var/lib/asterisk/third-party/tiresias/audio_recongition.db"  # fp_handler.c:31

# init_database (fp_handler.c:686-753) with DEF_AUBIO_COEFS = 2
SCHEMA = (
    "create table context_list(   name        varchar(255),   directory   varchar(1023),   primary key(name));",
    "create table audio_list(   uuid           varchar(255),   name           varchar(255),"
    "   context        varchar(255),\thash           varchar(1023));",
    "create table audio_fingerprint( context        varchar(255), audio_uuid     varchar(255),"
    " frame_idx      integer, max1 real, max2 real);",
    "create index idx_audio_fingerprint_context on audio_fingerprint(context);",
    "create index idx_audio_fingerprint_max1 on audio_fingerprint(max1);",
    "create index idx_audio_fingerprint_max2 on audio_fingerprint(max2);",
)

_MICRO_SQL = "case when {c} is null then %d else cast(round({c} * 1000000.0) as integer) end" % NULL_MICRO


def micro_text(m: int) -> str | None:
    """printf("%f") text of a stored micro-unit value (None for NULL)."""
    m = int(m)
    if m == NULL_MICRO:
        return None
    a = abs(m)
    return "%s%d.%06d" % ("-" if m < 0 else "", a // 1_000_000, a % 1_000_000)


def create_catalog(db: sqlite3.Connection):
    """The two control-plane tables of init_database, in the engine's in-memory catalog."""
    for ddl in SCHEMA[:2]:
        db.execute(ddl)


def load_backup(db: sqlite3.Connection, engine, filename: str) -> dict:
    """db_ctx_load_db_data: catalog rows into `db`, fingerprint rows into the GPU index.

    A missing file loads nothing and succeeds (the reference's ATTACH creates an empty DB).
    Returns counts; raises ValueError for rows the reference could not have written
    (non-numeric max columns) and TfpError if a uuid is already indexed.
    """
    out = {"contexts": 0, "audios": 0, "clips": 0, "rows": 0}
    if not os.path.exists(filename):
        return out
    src = sqlite3.connect("file:%s?mode=ro" % filename, uri=True)
    try:
        tables = {r[0] for r in src.execute("select name from sqlite_master where type='table'")}
        for t, key in (("context_list", "contexts"), ("audio_list", "audios")):
            if t in tables:
                rows = src.execute("select * from %s" % t).fetchall()
                if rows:
                    db.executemany("insert into %s values (%s)" % (t, ",".join("?" * len(rows[0]))), rows)
                out[key] = len(rows)
        if "audio_fingerprint" not in tables:
            return out
        bad = src.execute("select count(*) from audio_fingerprint where typeof(max1) not in ('real','integer','null')"
                          " or typeof(max2) not in ('real','integer','null')").fetchone()[0]
        if bad:
            raise ValueError(f"{bad} audio_fingerprint rows hold non-numeric max1/max2")
        uuids = [r[0] for r in src.execute("select distinct audio_uuid from audio_fingerprint"
                                           " where audio_uuid is not null order by audio_uuid")]
        src.execute("create temp table uid(u text primary key, id integer)")
        src.executemany("insert into temp.uid values (?, ?)", [(u, i) for i, u in enumerate(uuids)])
        cur = src.execute("select m.id, %s, %s from audio_fingerprint f join temp.uid m on m.u = f.audio_uuid"
                          " order by m.id, f.rowid" % (_MICRO_SQL.format(c="f.max1"), _MICRO_SQL.format(c="f.max2")))
        parts = []
        while True:
            chunk = cur.fetchmany(1 << 18)
            if not chunk:
                break
            parts.append(np.array(chunk, dtype=np.int64).reshape(-1, 3))
        rows = np.concatenate(parts) if parts else np.zeros((0, 3), np.int64)
    finally:
        src.close()
    vals = rows[:, 1:]
    if len(vals) and (vals.max() > 2**31 - 1 or vals[vals != NULL_MICRO].min(initial=0) < -(2**31) + 1):
        raise ValueError("audio_fingerprint max1/max2 outside the range any fingerprint can take")
    counts = np.bincount(rows[:, 0], minlength=len(uuids)) if len(uuids) else np.zeros(0, np.int64)
    foff = np.zeros(len(uuids) + 1, np.int64)
    np.cumsum(counts, out=foff[1:])
    engine.index_add_batch(uuids, foff, rows[:, 1].astype(np.int32), rows[:, 2].astype(np.int32))
    out["clips"], out["rows"] = len(uuids), int(len(rows))
    return out


def write_backup(db: sqlite3.Connection, engine, filename: str) -> dict:
    """db_ctx_backup: a file holding the reference schema, the catalog and every indexed row.

    Fingerprint rows are written for each audio_list uuid the engine holds, in frame order,
    with that audio's context (create_audio_fingerprint_info, fp_handler.c:559-566). The
    file is written beside the target and renamed over it, so a failed backup leaves the
    previous snapshot intact.
    """
    tmp = filename + ".tmp-%d" % os.getpid()
    if os.path.exists(tmp):
        os.remove(tmp)
    dst = sqlite3.connect(tmp)
    out = {"contexts": 0, "audios": 0, "rows": 0}
    try:
        for ddl in SCHEMA:
            dst.execute(ddl)
        ctx = db.execute("select * from context_list").fetchall()
        dst.executemany("insert into context_list values (?, ?)", ctx)
        aud = db.execute("select * from audio_list").fetchall()
        dst.executemany("insert into audio_list values (?, ?, ?, ?)", aud)
        out["contexts"], out["audios"] = len(ctx), len(aud)
        for uuid, _name, context, _hash in aud:
            try:
                m1, m2 = engine.index_rows(uuid)
            except Exception as e:  # not indexed (fingerprinting failed): catalog row only
                if getattr(e, "code", None) == -4:
                    continue
                raise
            dst.executemany("insert into audio_fingerprint(context, audio_uuid, frame_idx, max1, max2)"
                            " values (?, ?, ?, ?, ?)",
                            ((context, uuid, i, micro_text(a), micro_text(b)) for i, (a, b) in enumerate(zip(m1, m2))))
            out["rows"] += len(m1)
        dst.commit()
    except BaseException:
        dst.close()
        os.remove(tmp)
        raise
    dst.close()
    os.replace(tmp, filename)
    return out
