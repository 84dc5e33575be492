"""Generate tests/golden/match_cases.json — golden vectors for the search semantics.

The reference has no tests or fixtures, so its behaviour is manufactured here:
every expected result below is what the reference's own SQL (restated verbatim in
oracle/sql_oracle.py, citing /root/reference/src/fp_handler.c:308-374) returns when SQLite
executes it on rows inserted the way db_ctx_insert does ("%f" reals, NULL for absent keys).

Fixture = data: DB rows (clip, max1/max2 micro-units or NULL), uuids, query frames (the
unrounded doubles; null = absent JSON key) and the expected (uuid, match_count, frame_count).

Run:  python tests/golden/make_golden.py      (deterministic; seed below)
"""
from __future__ import annotations

import json
import os
import sys
import uuid as uuidlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from sql_oracle import SqlFingerprintDB  # noqa: E402

NULL = -(2**31)
SEED = 0x7153A1


def rand_uuid(rng, prefix: str | None = None) -> str:
    u = str(uuidlib.UUID(bytes=rng.bytes(16), version=4))
    if prefix:
        u = prefix + u[len(prefix):]
    return u


def draw_values(rng, n, null_p):
    """Micro-unit values clustered near integer dB keys so the trunc±tol windows hit."""
    kind = rng.random(n)
    base = rng.integers(-40, 40, n).astype(np.int64) * 1_000_000
    near = base + rng.integers(-2500, 2501, n)
    wide = rng.integers(-60_000_000, 45_000_000, n)
    exact = base + rng.choice([-1000, 1000, -999, 999, 0, -1001, 1001], n)
    v = np.where(kind < 0.45, near, np.where(kind < 0.6, exact, wide))
    v = np.where(rng.random(n) < null_p, NULL, v)
    return v.astype(np.int64)


def draw_query(rng, n, rows_m1, rows_m2):
    """Query doubles: some copied from DB rows (self-match), some near integers, some NULL."""
    q1 = []
    q2 = []
    for _ in range(n):
        r = rng.random()
        if r < 0.3 and len(rows_m1):
            j = int(rng.integers(len(rows_m1)))
            a = rows_m1[j] / 1e6 if rows_m1[j] != NULL else None
            b = rows_m2[j] / 1e6 if rows_m2[j] != NULL else None
            jit = float(rng.normal(0, 3e-7))
            q1.append(None if a is None else a + jit)
            q2.append(None if b is None else b + float(rng.normal(0, 3e-4)))
        elif r < 0.9:
            q1.append(float(rng.integers(-40, 40)) + float(rng.random()) * (1 if rng.random() < 0.5 else -1))
            q2.append(float(rng.integers(-40, 40)) + float(rng.random()))
        else:
            q1.append(None if rng.random() < 0.5 else float(rng.normal(0, 30)))
            q2.append(None)
    return q1, q2


PARAMS = [
    (1, 0.001, -1, -1), (1, 0.001, -1, -1), (1, 0.01, -1, -1), (1, 0.1, -1, -1), (1, 0.45, -1, -1),
    (1, -1.0, -1, -1), (1, 0.0, -1, -1), (1, 1.5, -1, -1), (1, 0.0078125, -1, -1), (1, 0.001, 100, 3400),
    (2, 0.001, -1, -1), (2, 0.01, -1, -1), (2, 0.45, -1, -1), (2, 0.1, 100, 3400), (2, 2.0, 2, 1000),
    (1, 0.05, 5, -1), (2, 0.3, -1, 20), (0, 0.001, -1, -1), (3, 0.001, -1, -1), (1, float("nan"), -1, -1),
]


def make_scenario(rng, name, nclips, max_frames, null_p, nqueries, prefix_share=False):
    uuids = []
    pref = rand_uuid(rng)[:20] if prefix_share else None
    for _ in range(nclips):
        uuids.append(rand_uuid(rng, pref if prefix_share and rng.random() < 0.5 else None))
    clip, m1, m2 = [], [], []
    for c in range(nclips):
        nf = int(rng.integers(1, max_frames + 1))
        clip += [c] * nf
        m1 += draw_values(rng, nf, null_p).tolist()
        m2 += draw_values(rng, nf, null_p).tolist()
    db = SqlFingerprintDB()
    for c in range(nclips):
        idx = [i for i, x in enumerate(clip) if x == c]
        db.insert_rows("ctx%d" % (c % 3), uuids[c], [m1[i] for i in idx], [m2[i] for i in idx])
    queries = []
    for qi in range(nqueries):
        nq = int(rng.integers(0, 60)) if qi else 0
        q1, q2 = draw_query(rng, nq, m1, m2)
        coefs, tol, low, high = PARAMS[qi % len(PARAMS)] if qi else (1, 0.001, -1, -1)
        res = db.search(q1, q2, coefs, tol, low, high)
        queries.append({"q1": q1, "q2": q2, "coefs": coefs, "tol": tol, "low": low, "high": high,
                        "frame_count": len(q1), "expect": res})
    return {"name": name, "uuids": uuids, "clip": clip, "m1": m1, "m2": m2, "queries": queries}


def make_tie_scenario(rng, nclips=2000):
    """Every clip ties: SQLite must return the greatest audio_uuid."""
    uuids = [rand_uuid(rng) for _ in range(nclips)]
    clip = list(range(nclips)) * 2
    m1 = [24_000_500] * nclips + [7_000_000] * nclips
    m2 = [1_000_000] * (2 * nclips)
    db = SqlFingerprintDB()
    for c in range(nclips):
        db.insert_rows("ctx", uuids[c], [24_000_500, 7_000_000], [1_000_000, 1_000_000])
    queries = []
    for q1 in ([24.3], [24.3, 7.9], [7.2, 24.9, 99.0], [-7.5]):
        res = db.search(q1, [1.0] * len(q1), 1, 0.001, -1, -1)
        queries.append({"q1": q1, "q2": [1.0] * len(q1), "coefs": 1, "tol": 0.001, "low": -1, "high": -1,
                        "frame_count": len(q1), "expect": res})
    assert queries[0]["expect"]["audio_uuid"] == max(uuids)
    return {"name": "tie_2000", "uuids": uuids, "clip": clip, "m1": m1, "m2": m2, "queries": queries}


def main():
    rng = np.random.default_rng(SEED)
    scen = []
    for s in range(24):
        scen.append(make_scenario(rng, "rand_%02d" % s, int(rng.integers(1, 30)), 60,
                                  0.03 if s % 3 else 0.2, 40, prefix_share=(s % 4 == 0)))
    scen.append(make_scenario(rng, "empty_db", 0, 1, 0.0, 10))
    scen.append(make_tie_scenario(rng))
    n_q = sum(len(s["queries"]) for s in scen)
    n_found = sum(1 for s in scen for q in s["queries"] if q["expect"])
    out = {"generator": "tests/golden/make_golden.py", "seed": SEED, "sqlite": __import__("sqlite3").sqlite_version,
           "scenarios": scen}
    path = os.path.join(HERE, "match_cases.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path, "scenarios", len(scen), "queries", n_q, "found", n_found,
          "bytes", os.path.getsize(path))


if __name__ == "__main__":
    main()
