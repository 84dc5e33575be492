"""Incremental maintenance of the device index (csrc/tfp_index.hip) on the GPU.

The reference's enrolment INSERTs a clip's rows into audio_fingerprint, whose max1 B-tree makes
them searchable at once (src/fp_handler.c:559-571, :745-753); a delete removes them
(:115-159). After the first build the engine merges adds and removals into its m1-sorted index in
one pass (the new rows alone are sorted; columns renumbered around the inserted / removed uuids)
instead of re-sorting every staged row. Every step below is searched on all paths (batch vote,
batch-1 small path, coefs = 2 general path) and must equal the oracle over the live rows
(count(*) DESC, ties to the greatest audio_uuid, :367-374) and an engine that rebuilds fully
(TFP_INDEX_FULL=1); the merge count proves no full sort ran.

Each test runs twice: with the index delta (round 4, the default: clips enrolled since the last
merge searched beside the sorted index by the coefs = 1 paths, merged before a coefs = 2 search or a
removal of an indexed clip) and with TFP_INDEX_DELTA=0 (every update a merge).

Also the staging compaction's failure path (advisor finding, round 2): an allocation failure
inside compact_staging must leave every clip's rows readable and the next build correct."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_DB, SEED_Q = 0x7153A1, 0x7153B2
HOP = 256


def _engine_with(tfp_lib, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return tfp_lib.Engine(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _uuids(rng, n):
    out = []
    for _ in range(n):
        h = "%032x" % int.from_bytes(rng.bytes(16), "little")
        out.append("%s-%s-4%s-a%s-%s" % (h[:8], h[8:12], h[13:16], h[17:20], h[20:32]))
    return out


class Mirror:
    """The live audio_fingerprint rows (uuid -> (m1, m2)) the engines should hold."""

    def __init__(self):
        self.rows = {}

    def search(self, oracle, q1, q2, qoff, p):
        uu = sorted(self.rows)
        m1 = np.concatenate([self.rows[u][0] for u in uu]) if uu else np.zeros(0, np.int32)
        m2 = np.concatenate([self.rows[u][1] for u in uu]) if uu else np.zeros(0, np.int32)
        clip = np.concatenate([np.full(len(self.rows[u][0]), i, np.int32) for i, u in enumerate(uu)]) if uu else \
            np.zeros(0, np.int32)
        # the sorted-index oracle (checked against the reference SQL in test_oracle.py); uu is in
        # uuid order, so the tie key of clip i is i
        idx = oracle.SortedIndex(m1, m2, clip, np.arange(max(len(uu), 1), dtype=np.int32))
        w, mc = idx.search_batch(q1, q2, qoff, p.coefs, p.tolerance, p.freq_ignore_low, p.freq_ignore_high,
                                 nthreads=16)
        return [(uu[w[i]], int(mc[i])) if w[i] >= 0 else None for i in range(len(qoff) - 1)]


def _frames(tfp_lib, qdb):
    fr = np.zeros(len(qdb), tfp_lib.FRAME_DTYPE)
    fr["q1"], fr["q2"] = qdb[:, 0], qdb[:, 1]
    return fr


@pytest.mark.parametrize("delta", ["1", "0"])
def test_incremental_updates_equal_oracle_and_full_build(tfp_lib, oracle, delta):
    rng = np.random.default_rng(31)
    n, nclips = 8000 * 10, 420
    nf = (n + HOP - 1) // HOP
    pcm = tfp_lib.synth_pcm(SEED_DB, range(nclips), n)
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n, nthreads=16, want_db=False)
    rows = [(micro[c * nf:(c + 1) * nf, 0].copy(), micro[c * nf:(c + 1) * nf, 1].copy()) for c in range(nclips)]
    uuids = _uuids(rng, nclips)
    uuids[410] = "00000000-0000-4000-8000-000000000000"  # sorts before every other uuid
    uuids[411] = "ffffffff-ffff-4fff-bfff-ffffffffffff"  # ... and after
    # queries: 3 s excerpts of clips (enrolled at various steps) and unrelated audio
    qn = 8000 * 3
    qsrc = [int(rng.integers(nclips)) if i % 4 != 3 else -1 for i in range(40)]
    qsrc[:6] = [300, 305, 410, 411, 2, 415]
    qpcm = np.stack([tfp_lib.synth_pcm(SEED_DB, [c], qn, offsets=[256 * int(rng.integers(0, 150))])[0] if c >= 0
                     else tfp_lib.synth_pcm(SEED_Q, [i], qn)[0] for i, c in enumerate(qsrc)])
    qdb = np.concatenate([oracle.fingerprint(q)[1] for q in qpcm])
    nfq = (qn + HOP - 1) // HOP
    qoff = np.arange(len(qpcm) + 1, dtype=np.int64) * nfq
    frames = _frames(tfp_lib, qdb)

    inc = _engine_with(tfp_lib, {"TFP_INDEX_DELTA": delta})
    full = _engine_with(tfp_lib, {"TFP_INDEX_FULL": "1"})
    mir = Mirror()
    engines = (inc, full)

    def add(cs, uu=None):
        uu = uu or [uuids[c] for c in cs]
        fo = np.concatenate([[0], np.cumsum([len(rows[c][0]) for c in cs])])
        for e in engines:
            if len(cs) == 1:
                e.index_add(uu[0], rows[cs[0]][0], rows[cs[0]][1])
            else:
                e.index_add_batch(uu, fo, np.concatenate([rows[c][0] for c in cs]),
                                  np.concatenate([rows[c][1] for c in cs]))
        for u, c in zip(uu, cs):
            mir.rows[u] = rows[c]

    def remove(u):
        for e in engines:
            e.index_remove(u)
        del mir.rows[u]

    def check(step):
        # batch-1 (small path) on the first queries, first: with the delta, before the coefs = 2
        # search below merges it
        p = tfp_lib.params(1, 0.001)
        exp = mir.search(oracle, qdb[:6 * nfq, 0], qdb[:6 * nfq, 1], qoff[:7], p)
        for i in range(6):
            r, _ = inc.search(frames[qoff[i]:qoff[i + 1]], p)
            assert (None if r is None else (r["audio_uuid"], r["match_count"])) == exp[i], (step, i)
        found = 0
        for p in (tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.3), tfp_lib.params(2, 0.05)):
            exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
            found = max(found, sum(x is not None for x in exp))
            for e in engines:
                res, fcs = e.search_batch(frames, qoff, p)
                got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
                assert got == exp, (step, p.coefs, p.tolerance, [i for i in range(len(exp)) if got[i] != exp[i]][:5])
                assert all(f == nfq for f in fcs)
        return found

    add(list(range(300)))
    for e in engines:
        e.index_commit()
    assert inc.index_build_stats() == (1, 0)
    check("initial")
    steps = 0
    add([300]); steps += 1
    check("one clip")
    add([301]); steps += 1
    check("another clip")
    add(list(range(302, 340))); steps += 1
    check("batch of 38")
    for c in (0, 17, 150, 299):
        remove(uuids[c])
    steps += 1
    check("4 removed")
    remove(uuids[301]); steps += 1
    check("a merged clip removed")
    add([17], [uuids[17]])                      # a removed uuid re-enrolled (same rows)
    add([340], [uuids[0]]); steps += 1          # ... and one with other rows (one build for both)
    check("re-added")
    add([410]); add([411]); steps += 1
    check("first and last uuid")
    add([412]); remove(uuids[412]); add([413]); steps += 1   # added and removed between builds
    check("transient clip")
    for c in range(341, 356):                   # one clip per build (enrol, commit: searchable at once)
        add([c]); steps += 1
        for e in engines:
            e.index_commit()
        if c % 5 == 0:
            check("stream of adds %d" % c)
    assert check("final") > 10
    fb, merges = inc.index_build_stats()
    if delta == "0":
        assert fb == 1 and merges == steps, (fb, merges, steps)   # no full sort after the first build
    else:  # updates went to the delta (swept beside the main index by coefs = 2), merged by the removals
        nd, _ = inc.index_delta_stats()
        assert fb == 1 and nd >= 10 and 1 <= merges <= steps, (fb, merges, nd, steps)
    assert full.index_build_stats()[1] == 0
    for e in engines:
        assert e.index_stats() == (sum(len(r[0]) for r in mir.rows.values()), len(mir.rows))
        e.close()


def test_compaction_failure_leaves_index_intact(tfp_lib, oracle):
    """compact_staging fails (injected allocation failure) after many removals: the call returns
    TFP_E_NOMEM, every live clip's rows read back unchanged, and the next commit succeeds and
    searches equal the oracle (the advisor's round-2 finding at tfp_engine.cpp:453)."""
    rng = np.random.default_rng(5)
    n, nclips = 8000 * 30, 200
    nf = (n + HOP - 1) // HOP
    pcm = tfp_lib.synth_pcm(SEED_DB, range(nclips), n)
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n, nthreads=16, want_db=False)
    uuids = _uuids(rng, nclips)
    eng = _engine_with(tfp_lib, {"TFP_TEST_FAIL_COMPACT": "1"})
    eng.index_add_batch(uuids, np.arange(nclips + 1) * nf, micro[:, 0], micro[:, 1])
    eng.index_commit()
    mir = Mirror()
    for c in range(nclips):
        mir.rows[uuids[c]] = (micro[c * nf:(c + 1) * nf, 0], micro[c * nf:(c + 1) * nf, 1])
    for c in range(0, nclips, 4):   # interleaved live / dead runs
        for k in range(3):
            if c + k < nclips:
                eng.index_remove(uuids[c + k])
                del mir.rows[uuids[c + k]]
    with pytest.raises(tfp_lib.TfpError) as ei:
        eng.index_commit()  # dead rows > 1/4 of the live ones: compaction, which fails
    assert ei.value.code == -3
    for u, (m1, m2) in mir.rows.items():
        g1, g2 = eng.index_rows(u)
        assert np.array_equal(g1, m1) and np.array_equal(g2, m2), u
    eng.index_commit()
    for u, (m1, m2) in mir.rows.items():
        g1, g2 = eng.index_rows(u)
        assert np.array_equal(g1, m1) and np.array_equal(g2, m2), u
    qn = 8000 * 3
    live = [c for c in range(nclips) if uuids[c] in mir.rows]
    qpcm = np.stack([tfp_lib.synth_pcm(SEED_DB, [live[i * 7 % len(live)]], qn, offsets=[256 * 40])[0]
                     for i in range(12)])
    qdb = np.concatenate([oracle.fingerprint(q)[1] for q in qpcm])
    nfq = (qn + HOP - 1) // HOP
    qoff = np.arange(len(qpcm) + 1, dtype=np.int64) * nfq
    p = tfp_lib.params(1, 0.001)
    res, _ = eng.search_batch(_frames(tfp_lib, qdb), qoff, p)
    got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
    exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
    assert got == exp
    assert sum(x is not None for x in exp) >= 5
    eng.close()


@pytest.mark.parametrize("delta", ["0", "1"])
def test_key_bits_carried_across_merges(tfp_lib, oracle, delta):
    """The small path's key bitsets are carried across single-clip merges (a zero column at each
    breakpoint, then the new rows' bits; tfp_index.hip key_bits_*), and rebuilt where the row width
    changes (384 -> 385 clips: 12 -> 16 words) or a clip was removed. Every step's batch-1 searches
    (the small path reads the bitsets) == the oracle; new uuids sort first, last and in between."""
    rng = np.random.default_rng(77)
    nrow = 60

    def rows_of():  # each clip's rows in two of 30 keys' boxes: a query's own clip outscores the rest
        k = rng.choice(rng.choice(np.arange(10, 40), 2, replace=False), nrow)
        m1 = (k * 1_000_000 + rng.integers(0, 250_000, nrow)).astype(np.int32)
        m2 = rng.integers(0, 30_000_000, nrow).astype(np.int32)
        return m1, m2

    uu = _uuids(rng, 400)
    uu[385] = "00000000-0000-4000-8000-000000000001"  # sorts first
    uu[386] = "ffffffff-ffff-4fff-bfff-fffffffffffe"  # sorts last
    data = [rows_of() for _ in range(400)]
    eng = _engine_with(tfp_lib, {"TFP_INDEX_DELTA": delta})
    mir = Mirror()
    p = tfp_lib.params(1, 0.3)

    def check(step, sources):
        q = []
        for c in sources:
            m1, m2 = data[c]
            sel = rng.integers(0, nrow, 40)
            q.append(np.stack([m1[sel] / 1e6 + 0.001, m2[sel] / 1e6], axis=1))
        qdb = np.concatenate(q)
        qoff = np.arange(len(sources) + 1, dtype=np.int64) * 40
        exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
        fr = _frames(tfp_lib, qdb)
        for i in range(len(sources)):
            r, _ = eng.search(fr[qoff[i]:qoff[i + 1]], p)  # batch-1: the small path over the bitsets
            assert (None if r is None else (r["audio_uuid"], r["match_count"])) == exp[i], (step, i)
        return sum(e is not None for e in exp)

    try:
        for c in range(380):
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]
        eng.index_commit()
        found = check("initial", [0, 5, 100, 379])
        for c in list(range(380, 393)) + ["remove", 393, 394]:
            if c == "remove":
                eng.index_remove(uu[7])
                del mir.rows[uu[7]]
            else:
                eng.index_add(uu[c], *data[c])
                mir.rows[uu[c]] = data[c]
            eng.index_commit()
            found += check(c, [int(x) for x in rng.integers(0, 380, 2)] + ([c] if c != "remove" else [8]))
        assert found > 20
        fb, merges = eng.index_build_stats()
        if delta == "0":
            assert fb == 1 and merges == 16, (fb, merges)
        else:  # every add a delta update; the removal of an indexed clip merged the delta once
            nd, _ = eng.index_delta_stats()
            assert fb == 1 and merges == 1 and nd == 15, (fb, merges, nd)
    finally:
        eng.close()


@pytest.mark.parametrize("delta", ["0", "1"])
def test_add_only_updates_empty_and_null_rows(tfp_lib, oracle, delta):
    """Updates that only add take the engine's host fast path (no pass over every clip; the
    column map from the new uuids' insertion points, csrc/tfp_engine.cpp live_order) and merge every
    staged row with the rows that cannot match (NULL max1: the reference's max1 >= ... never holds
    for them, fp_handler.c:339-347) sorted past the new row count. Covered: a clip without rows that
    sorts first (the columns still shift), clips with some and with only NULL max1 rows, a clip
    added and removed between builds (still add-only), more new uuids before old ones than the
    column map holds, a removal (the general path) and an add after it. Every step, batch and
    batch-1 searches == the oracle over the live rows."""
    rng = np.random.default_rng(123)
    nrow = 60

    def rows_of():
        k = rng.choice(rng.choice(np.arange(10, 40), 2, replace=False), nrow)
        m1 = (k * 1_000_000 + rng.integers(0, 250_000, nrow)).astype(np.int32)
        m2 = rng.integers(0, 30_000_000, nrow).astype(np.int32)
        return m1, m2

    uu = _uuids(rng, 260)
    uu[200] = "00000000-0000-4000-8000-000000000002"  # sorts first
    for i in range(240, 252):                          # sort before most old uuids
        uu[i] = "0%07x-0000-4000-8000-000000000000" % (i * 997)
    data = [rows_of() for _ in range(260)]
    data[200] = (np.zeros(0, np.int32), np.zeros(0, np.int32))
    m1 = data[201][0].copy()
    m1[::2] = tfp_lib.NULL_MICRO
    data[201] = (m1, data[201][1])
    data[202] = (np.full(nrow, tfp_lib.NULL_MICRO, np.int32), data[202][1])
    eng = _engine_with(tfp_lib, {"TFP_INDEX_DELTA": delta})
    mir = Mirror()
    params = (tfp_lib.params(1, 0.3), tfp_lib.params(2, 0.05))

    def check(step, sources):
        q = []
        for c in sources:
            m1, m2 = data[c]
            sel = rng.integers(0, nrow, 40)
            q.append(np.stack([m1[sel] / 1e6 + 0.001, m2[sel] / 1e6], axis=1))
        qdb = np.concatenate(q)
        qoff = np.arange(len(sources) + 1, dtype=np.int64) * 40
        fr = _frames(tfp_lib, qdb)
        found = 0
        for p in params:
            exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
            res, _ = eng.search_batch(fr, qoff, p)
            got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
            assert got == exp, (step, p.coefs)
            found += sum(e is not None for e in exp)
        p = params[0]
        exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
        for i in range(len(sources)):
            r, _ = eng.search(fr[qoff[i]:qoff[i + 1]], p)  # batch-1: the small path
            assert (None if r is None else (r["audio_uuid"], r["match_count"])) == exp[i], (step, i)
        return found

    def check_delta(step, sources):  # coefs = 1 only (batch and batch-1): served with the delta
        q = []
        for c in sources:
            m1, m2 = data[c]
            sel = rng.integers(0, nrow, 40)
            q.append(np.stack([m1[sel] / 1e6 + 0.001, m2[sel] / 1e6], axis=1))
        qdb = np.concatenate(q)
        qoff = np.arange(len(sources) + 1, dtype=np.int64) * 40
        fr = _frames(tfp_lib, qdb)
        p = params[0]
        exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
        for i in range(len(sources)):
            r, _ = eng.search(fr[qoff[i]:qoff[i + 1]], p)
            assert (None if r is None else (r["audio_uuid"], r["match_count"])) == exp[i], (step, i)
        res, _ = eng.search_batch(fr, qoff, p)
        assert [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res] == exp, step

    def add(cs):
        for c in cs:
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]

    try:
        add(range(200))
        eng.index_commit()
        found = check("initial", [0, 50, 199])
        steps = [("empty clip first", [200], None), ("half NULL", [201], None), ("all NULL", [202], None),
                 ("batch + transient", [203, 204, 205], 206), ("12 before old uuids", list(range(240, 252)), None),
                 ("removal", [207], "remove"), ("after removal", [208], None), ("one more", [209], None)]
        for name, cs, extra in steps:
            if extra == "remove":
                eng.index_remove(uu[3])
                del mir.rows[uu[3]]
            add(cs)
            if isinstance(extra, int):  # added and removed before the build
                eng.index_add(uu[extra], *data[extra])
                eng.index_remove(uu[extra])
            eng.index_commit()
            srcs = [int(x) for x in rng.integers(4, 200, 2)] + [c for c in cs if c not in (200, 201, 202)]
            if delta == "1":
                check_delta(name, srcs)
            found += check(name, srcs)
        assert found > 20
        fb, merges = eng.index_build_stats()
        if delta == "0":
            assert fb == 1 and merges == len(steps), (fb, merges)
        else:  # each step's adds a delta update, which the coefs = 2 searches sweep beside the main
            # index (round 6: no merge); the removal of an indexed clip (uu[3]) merges at once
            nd, _ = eng.index_delta_stats()
            assert fb == 1 and merges == 1 and nd == len(steps) - 1, (fb, merges, nd)
            assert eng.index_cache_stats()["delta_sweeps"] > 0
        assert eng.index_stats() == (sum(len(r[0]) for r in mir.rows.values()), len(mir.rows))
    finally:
        eng.close()


def _dense_db(rng, nclips, nrow):
    """Clips whose rows crowd into keys 16-18 (fractions across the whole key, so the 0.45 boxes
    hold thousands of rows each and the 0.001 boxes a few): every key-bits path gets big pieces."""
    data = []
    for _ in range(nclips):
        k = rng.choice([16, 17, 17, 18], nrow)
        m1 = (k * 1_000_000 + rng.integers(-499_000, 499_000, nrow)).astype(np.int32)
        m1[: nrow // 10] = (k[: nrow // 10] * 1_000_000 + rng.integers(-900, 900, nrow // 10)).astype(np.int32)
        m2 = rng.integers(0, 30_000_000, nrow).astype(np.int32)
        data.append((m1, m2))
    return data


def _check_batch1(eng, oracle, tfp_lib, mir, data, sources, p, rng, step):
    q = []
    for c in sources:
        m1, m2 = data[c]
        sel = rng.integers(0, len(m1), 30)
        q.append(np.stack([m1[sel] / 1e6 + 0.0004, m2[sel] / 1e6], axis=1))
    qdb = np.concatenate(q)
    qoff = np.arange(len(sources) + 1, dtype=np.int64) * 30
    exp = mir.search(oracle, qdb[:, 0], qdb[:, 1], qoff, p)
    fr = _frames(tfp_lib, qdb)
    for i in range(len(sources)):
        r, _ = eng.search(fr[qoff[i]:qoff[i + 1]], p)  # batch-1: the small path over the key bitsets
        assert (None if r is None else (r["audio_uuid"], r["match_count"])) == exp[i], (step, p.tolerance, i)
    return sum(e is not None for e in exp)


@pytest.mark.parametrize("knobs", [{}, {"TFP_KEYBITS_WIN": "4"}, {"TFP_KEYBITS_DIRECT": "0"},
                                   {"TFP_KEYBITS_DIRECT": "1000000000"}, {"TFP_KEYBITS_WIN": "8", "TFP_KEYBITS_DIRECT": "0"}])
def test_key_bits_build_forms(tfp_lib, oracle, knobs):
    """launch_key_bits (round 5): the boxes' rows walked in chunks, each piece's bits set in an LDS
    copy of the key's row and ORed into memory once per word, small pieces with global atomics,
    rows wider than the LDS window window by window. Forced forms (windows of 4 / 8 words = 128 /
    256 columns over 700 clips; every piece through LDS; every piece direct) == the default ==
    the oracle, on boxes of thousands of rows (tol 0.45) and of a few (tol 0.001)."""
    rng = np.random.default_rng(5150)
    data = _dense_db(rng, 700, 50)
    uu = _uuids(rng, 700)
    eng = _engine_with(tfp_lib, knobs)
    mir = Mirror()
    try:
        for c in range(700):
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]
        eng.index_commit()
        found = 0
        for tol in (0.45, 0.001, 0.2, 1.5):
            found += _check_batch1(eng, oracle, tfp_lib, mir, data, [int(x) for x in rng.integers(0, 700, 6)],
                                   tfp_lib.params(1, tol), rng, "build")
        assert found > 10
    finally:
        eng.close()


@pytest.mark.parametrize("delta", ["0", "1"])
def test_tolerance_alternation_and_removals(tfp_lib, oracle, delta):
    """The dialplan passes the tolerance per call (application_handler.c:114-122): batch-1 searches
    alternating between tolerances (0.001 and 0.45, and two more, so the engine's cache of other
    tolerances' key ranges and bitsets evicts its least recently used entry) between adds and
    removals of indexed clips (the bitsets carried through the column renumbering, removed columns
    dropped, src/fp_handler.c:115-159): every search == the oracle over the live rows."""
    rng = np.random.default_rng(4242)
    data = _dense_db(rng, 460, 40)
    uu = _uuids(rng, 460)
    uu[450] = "00000000-0000-4000-8000-000000000002"  # sorts first
    eng = _engine_with(tfp_lib, {"TFP_INDEX_DELTA": delta})
    mir = Mirror()
    tols = [0.001, 0.45, 0.001, 0.45, 0.1, 0.3, 0.45, 0.001, 0.7, 0.45]
    try:
        for c in range(420):
            eng.index_add(uu[c], *data[c])
            mir.rows[uu[c]] = data[c]
        eng.index_commit()
        found = 0
        live = list(range(420))
        for step, op in enumerate(["-", "remove", "add", "-", "remove", "remove", "add", "add", "-", "remove"]):
            if op == "remove":
                c = live.pop(int(rng.integers(len(live))))
                eng.index_remove(uu[c])
                del mir.rows[uu[c]]
            elif op == "add":
                c = 420 + step if step != 6 else 450
                eng.index_add(uu[c], *data[c])
                mir.rows[uu[c]] = data[c]
                live.append(c)
            for tol in tols[step:] + tols[:step]:
                src = [int(live[int(x)]) for x in rng.integers(0, len(live), 2)]
                found += _check_batch1(eng, oracle, tfp_lib, mir, data, src, tfp_lib.params(1, tol), rng, (step, op))
        assert found > 50
    finally:
        eng.close()
