"""SQL ORACLE: the reference's search path executed by SQLite (test infrastructure only).

Restates, string for string, the SQL that /root/reference/src/fp_handler.c sends through
db_ctx_handler.c, and runs it with Python's sqlite3 (SQLite 3.37.2 in this image):

  DDL            fp_handler.c:713-753  (audio_fingerprint + indices on context/max1/max2)
  row insert     db_ctx_handler.c:413-556 — one INSERT per frame row, reals printed "%f",
                 keys whose json_real was NULL (±inf) are absent → column NULL
  temp table     fp_handler.c:857-893
  per frame      fp_handler.c:287-359  "insert into %s select * from audio_fingerprint where
                 max1 >= %f and max1 <= %f [and max2 >= %f and max2 <= %f] group by audio_uuid"
  result         fp_handler.c:367-374  "select *, count(*) from %s group by audio_uuid
                 order by count(*) DESC" → first row
  frame_count    fp_handler.c:286,403

This is the pin for the match semantics (tie-break, NULLs, truncation, inclusive bounds):
tests/golden/make_golden.py runs it to produce the committed fixtures, and the C oracle and
the GPU engine are both checked against those fixtures.
"""
from __future__ import annotations

import math
import sqlite3


def micro_str(m: int) -> str:
    """The "%f" text of a stored value given its micro-units (exact integer formatting)."""
    neg = m < 0
    a = -m if neg else m
    return ("-" if neg else "") + f"{a // 1000000}.{a % 1000000:06d}"


def _f(x: float) -> str:
    # C printf("%f"); Python's %-formatting is also exact round-half-even of the binary value.
    return "%f" % x


class SqlFingerprintDB:
    def __init__(self):
        self.db = sqlite3.connect(":memory:")
        c = self.db.cursor()
        c.execute("create table audio_fingerprint( context        varchar(255), audio_uuid     varchar(255),"
                  " frame_idx      integer, max1 real, max2 real);")
        c.execute("create index idx_audio_fingerprint_context on audio_fingerprint(context);")
        c.execute("create index idx_audio_fingerprint_max1 on audio_fingerprint(max1);")
        c.execute("create index idx_audio_fingerprint_max2 on audio_fingerprint(max2);")
        self.temp_seq = 0

    def insert_rows(self, context: str, uuid: str, m1s, m2s, null: int = -(2**31)):
        """create_audio_fingerprint_info: one INSERT per frame (fp_handler.c:559-571)."""
        c = self.db.cursor()
        for idx, (m1, m2) in enumerate(zip(m1s, m2s)):
            keys = ["frame_idx", "audio_uuid"]
            vals = ["%d" % idx, "'%s'" % uuid]
            if m1 != null:
                keys.append("max1"); vals.append(micro_str(int(m1)))
            if m2 != null:
                keys.append("max2"); vals.append(micro_str(int(m2)))
            keys.append("context"); vals.append("'%s'" % context)
            c.execute("insert into audio_fingerprint(%s) values (%s);" % (", ".join(keys), ", ".join(vals)))
        self.db.commit()

    def insert_rows_bulk(self, context: str, clips, null: int = -(2**31), per_stmt: int = 500):
        """The same rows as insert_rows (same "%f" literals, same NULL rule), loaded in one
        transaction with multi-row INSERT statements: for building large benchmark tables fast
        (the load is not what the baseline times). clips: iterable of (uuid, m1s, m2s)."""
        c = self.db.cursor()
        c.execute("begin")
        buf = []

        def lit(m):
            return "NULL" if m == null else micro_str(int(m))
        for uuid, m1s, m2s in clips:
            for idx, (m1, m2) in enumerate(zip(m1s, m2s)):
                buf.append("('%s','%s',%d,%s,%s)" % (context, uuid, idx, lit(m1), lit(m2)))
                if len(buf) == per_stmt:
                    c.execute("insert into audio_fingerprint(context, audio_uuid, frame_idx, max1, max2) values "
                              + ",".join(buf))
                    buf = []
        if buf:
            c.execute("insert into audio_fingerprint(context, audio_uuid, frame_idx, max1, max2) values " + ",".join(buf))
        self.db.commit()

    def search(self, q1s, q2s, coefs: int, tolerance: float, freq_ignore_low: int, freq_ignore_high: int):
        """fp_search_fingerprint_info on precomputed query fingerprints.

        q1s/q2s are the unrounded doubles of the query's JSON rows (None = absent key).
        Returns None (NOTFOUND/NULL) or dict(audio_uuid, match_count, frame_count)."""
        if coefs < 1 or coefs > 2:
            return None
        tole = tolerance
        if tole < 0:
            tole = 0.001
        self.temp_seq += 1
        table = "temp_%08d" % self.temp_seq
        c = self.db.cursor()
        c.execute("create table %s( context        varchar(255), audio_uuid     varchar(255),"
                  " frame_idx      integer, max1 real, max2 real);" % table)
        frame_count = len(q1s)
        for i in range(frame_count):
            v1 = q1s[i] if q1s[i] is not None else 0.0  # ast_json_real_get(NULL) == 0.0
            freq = float(int(v1))                       # (int) truncation, fp_handler.c:290
            if freq_ignore_low > 0 and freq < 10 * math.log10(freq_ignore_low):
                continue
            if freq_ignore_high > 0 and freq > 10 * math.log10(freq_ignore_high):
                continue
            sql = ("insert into %s select * from audio_fingerprint where  max1 >= %s  and max1 <= %s "
                   % (table, _f(freq - tole), _f(freq + tole)))
            for j in range(1, coefs):
                v = q2s[i] if q2s[i] is not None else 0.0
                if freq_ignore_low > 0 and v < 10 * math.log10(freq_ignore_low):
                    continue
                if freq_ignore_high > 0 and v > 10 * math.log10(freq_ignore_high):
                    continue
                sql = "%s and max%d >= %s and max%d <= %s" % (sql, j + 1, _f(v - tole), j + 1, _f(v + tole))
            sql = "%s group by audio_uuid" % sql
            try:
                c.execute(sql)
            except sqlite3.Error:
                pass  # db_ctx_exec logs and returns false; the loop goes on (fp_handler.c:357-359)
        row = c.execute("select *, count(*) from %s group by audio_uuid order by count(*) DESC" % table).fetchone()
        c.execute("drop table %s;" % table)
        if row is None:
            return None
        return {"audio_uuid": row[1], "match_count": int(row[5]), "frame_count": frame_count}
