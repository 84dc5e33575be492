"""The coefs = 2 clip-set caches (round 6): built from the clip order (the index rows ordered by
nearest-integer key, column and max2: a filter per tolerance, no sort), kept for four tolerances
(the active one and three others, least recently used out) and carried through index merges with the
clip order itself (tfp_index.hip launch_order_merge); an index delta gets a cache of its own rows,
swept beside the main one (no merge per enrolment). The dialplan passes the tolerance per call
(application_handler.c:114-122) and every enrolment's rows are searchable at once
(fp_handler.c:559-571): callers alternating coefs = 2 tolerances between enrolments and removals get
the oracle's answer (fp_handler.c:318-353) at every step."""
import numpy as np
import pytest

from test_gpu_index import Mirror, _dense_db, _engine_with, _frames, _uuids

pytestmark = pytest.mark.gpu


def _queries(rng, data, sources, nfr=30, jitter=0):
    q = []
    for c in sources:
        if c < 0:  # unrelated frames
            q.append(np.stack([rng.uniform(10, 25, nfr), rng.uniform(0, 30, nfr)], axis=1))
            continue
        m1, m2 = data[c]
        sel = rng.integers(0, len(m1), nfr)
        q.append(np.stack([m1[sel] / 1e6 + 0.0004, (m2[sel] + rng.integers(-jitter, jitter + 1, nfr)) / 1e6], axis=1))
    return np.concatenate(q), np.arange(len(sources) + 1, dtype=np.int64) * nfr


def _check(eng, oracle, tfp_lib, mir, qdb, qoff, p, step):
    exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
    res, _ = eng.search_batch(_frames(tfp_lib, qdb), qoff, p)
    got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
    assert got == exp, (step, p.tolerance, [i for i in range(len(exp)) if got[i] != exp[i]][:5])
    return sum(e is not None for e in exp)


def _clustered_db(rng, nclips, nrow):
    """_dense_db's max1 keys with max2 values in runs a few micro-units apart (clusters cut at every
    tolerance's gap) and repeated values (equal points)."""
    data = _dense_db(rng, nclips, nrow)
    out = []
    for m1, m2 in data:
        base = rng.integers(0, 3_000_000, nrow // 5)
        m2 = (np.repeat(base, 5)[:nrow] + rng.integers(0, 6, nrow) * rng.integers(1, 2500, nrow)).astype(np.int32)
        m2[::7] = m2[0]
        out.append((m1, m2))
    return out


@pytest.mark.parametrize("delta", ["1", "0"])
def test_coefs2_tolerance_alternation_with_enrolments_and_removals(tfp_lib, oracle, delta):
    """coefs = 2 batches alternating tolerances 0.001 / 0.45 / 0.01 / 0.1 / 0.3 (served by the clip
    order and the cache LRU) and 0.7 (above 0.49: the boxes' rows sorted, the delta merged first)
    between adds (with the index delta: swept from the delta's own cache beside the main one) and
    removals: every batch == the oracle over the live rows; the clip order is built once and merged through every later update,
    and revisited tolerances are LRU hits."""
    rng = np.random.default_rng(6060)
    data = _clustered_db(rng, 470, 40)
    uu = _uuids(rng, 470)
    uu[455] = "00000000-0000-4000-8000-000000000003"  # sorts first
    uu[456] = "ffffffff-ffff-4fff-bfff-fffffffffff0"  # sorts last
    eng = _engine_with(tfp_lib, {"TFP_INDEX_DELTA": delta})
    mir = Mirror()
    tols = [0.001, 0.45, 0.001, 0.45, 0.01, 0.1, 0.3, 0.7, 0.45, 0.001]
    try:
        for c in range(420):
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]
        eng.index_commit()
        live = list(range(420))
        found = 0
        ops = ["-", "add", "remove", "add", "add", "-", "remove", "add", "remove", "add", "add", "-"]
        nxt = 420
        for step, op in enumerate(ops):
            if op == "remove":
                c = live.pop(int(rng.integers(len(live))))
                eng.index_remove(uu[c])
                del mir.rows[uu[c]]
            elif op == "add":
                c = nxt if step not in (3, 9) else (455 if step == 3 else 456)
                nxt += 1
                eng.index_add(uu[c], *data[c])
                mir.rows[uu[c]] = data[c]
                live.append(c)
            for tol in tols[step % 3:] + tols[:step % 3]:
                src = [int(live[int(x)]) for x in rng.integers(0, len(live), 6)] + [-1, live[-1]]
                qdb, qoff = _queries(rng, data, src, jitter=3)
                found += _check(eng, oracle, tfp_lib, mir, qdb, qoff, tfp_lib.params(2, tol), (step, op))
        st = eng.index_cache_stats()
        assert found > 300, found
        assert st["hits"] > 0 and st["from_order"] > 0, st
        assert st["order_merges"] > 0, st          # the order carried through the merges ...
        assert st["order_builds"] <= 2, st         # ... instead of re-sorted (one more after a full build at most)
        if delta == "1":
            assert st["delta_sweeps"] > 0 and st["delta_builds"] > 0, st
    finally:
        eng.close()


def test_cache_from_order_equals_sorted_boxes(tfp_lib, oracle):
    """The cache built from the clip order (tolerances <= 0.49) and the one built by sorting the
    boxes' rows answer alike: the same batches at tol 0.49 (order) and through an engine whose
    clip order is fresh, at the order's edge keys (max1 values a micro-unit inside and outside the
    0.49 boxes, negative keys), coefs = 2 with the ignore filter (frames without a max2 condition
    hit every group of their key) == the oracle."""
    rng = np.random.default_rng(707)
    data = []
    for c in range(300):
        k = rng.choice([-3, -2, 16, 17], 40)
        off = rng.choice([-490_000, -489_999, -490_001, 489_999, 490_000, 490_001, 0, 1], 40)
        m1 = (k * 1_000_000 + off + rng.integers(-5, 6, 40) * (rng.random(40) < 0.3)).astype(np.int32)
        m2 = rng.integers(-2_000_000, 2_000_000, 40).astype(np.int32)
        data.append((m1, m2))
    uu = _uuids(rng, 300)
    eng = tfp_lib.Engine(0)
    mir = Mirror()
    try:
        for c in range(300):
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]
        eng.index_commit()
        found = 0
        for tol in (0.49, 0.489999, 0.001, 0.0):
            for low, high in ((-1, -1), (50, 60)):
                src = [int(x) for x in rng.integers(0, 300, 10)]
                qdb, qoff = _queries(rng, data, src, jitter=2)
                qdb[:, 0] = np.round(qdb[:, 0] - 0.0004, 6)  # the rows' own max1 values
                p = tfp_lib.params(2, tol, low, high)
                found += _check(eng, oracle, tfp_lib, mir, qdb, qoff, p, ("edge", tol, low))
        assert found > 20
        assert eng.index_cache_stats()["from_order"] >= 4
    finally:
        eng.close()


@pytest.mark.parametrize("tol", [0.001, 0.3])
def test_coefs2_delta_sweep_without_merge(tfp_lib, oracle, tol):
    """Enrolments followed by coefs = 2 searches (round 6): the new clips stay in the index delta and
    the sweep runs over the delta's own clip-set cache beside the main one (the main caches and the
    index untouched: no merge, no cache rebuild), as the reference's INSERT makes a clip searchable
    for the cost of its rows (fp_handler.c:559-571). Covered: a delta copy of a main clip's rows under
    a greater uuid (wins the tie) and one under a smaller uuid (loses it), a clip in keys the main
    index lacks, one with only NULL max1 rows, one without rows; then a tolerance above 0.49 merges
    the delta first. Every batch == the oracle over the live rows."""
    rng = np.random.default_rng(9090 + int(tol * 1000))
    data = _clustered_db(rng, 300, 40)
    uu = _uuids(rng, 300)
    eng = _engine_with(tfp_lib, {"TFP_INDEX_DELTA": "1"})
    mir = Mirror()
    try:
        for c in range(300):
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]
        eng.index_commit()
        p = tfp_lib.params(2, tol)
        src = [int(x) for x in rng.integers(0, 300, 8)]
        qdb, qoff = _queries(rng, data, src, jitter=2)
        _check(eng, oracle, tfp_lib, mir, qdb, qoff, p, "main")  # the main caches at this tolerance
        fb0, mg0 = eng.index_build_stats()
        st0 = eng.index_cache_stats()
        # the delta: copies of clips x (greater uuid) and y (smaller uuid), new keys, NULL rows, no rows
        x = next(c for c in range(300) if uu[c][-1] not in "f9")
        y = next(c for c in range(300) if c != x and uu[c][-1] not in "0a")
        bump = lambda u, d: u[:-1] + "%x" % (int(u[-1], 16) + d)
        m1n = (rng.integers(40, 44, 40) * 1_000_000 + rng.integers(-400_000, 400_000, 40)).astype(np.int32)
        adds = [(bump(uu[x], 1), data[x]), (bump(uu[y], -1), data[y]),
                ("7" * 8 + "-0000-4000-8000-000000000040", (m1n, rng.integers(0, 3_000_000, 40).astype(np.int32))),
                ("7" * 8 + "-0000-4000-8000-000000000041", (np.full(40, tfp_lib.NULL_MICRO, np.int32),
                                                           rng.integers(0, 3_000_000, 40).astype(np.int32))),
                ("7" * 8 + "-0000-4000-8000-000000000042", (np.zeros(0, np.int32), np.zeros(0, np.int32)))]
        found = 0
        for u, rows in adds:
            eng.index_add(u, *rows)
            mir.rows[u] = rows
            qd, qo = _queries(rng, data + [data[x], data[y], adds[2][1]], [x, y, 300, 301, 302] +
                              [int(v) for v in rng.integers(0, 300, 3)] + [-1], jitter=1)
            found += _check(eng, oracle, tfp_lib, mir, qd, qo, p, ("delta", u))
        assert found > 20
        st1 = eng.index_cache_stats()
        assert eng.index_build_stats() == (fb0, mg0), "an enrolment + coefs = 2 search merged the index"
        assert st1["builds"] == st0["builds"] and st1["delta_sweeps"] - st0["delta_sweeps"] >= len(adds), (st0, st1)
        assert eng.index_delta_stats()[1] == len(adds)
        # above the order's tolerances the delta is merged first (the boxes' rows of the merged index)
        _check(eng, oracle, tfp_lib, mir, qdb, qoff, tfp_lib.params(2, 0.7), "merged")
        assert eng.index_build_stats()[1] == mg0 + 1 and eng.index_delta_stats()[1] == 0
        _check(eng, oracle, tfp_lib, mir, qdb, qoff, p, "after the merge")
    finally:
        eng.close()
