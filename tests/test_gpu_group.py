"""Device groups (tfp_group_*, csrc/tfp_group.cpp): the enrolled DB sharded over several engines
in one process, searched on all of them in parallel and combined on the host.

On this one-GPU box the group is three engines on device 0 (the same code path as three GPUs,
with device-to-device copies in place of xGMI peer copies). Every search — batch-1 (each shard
fingerprints the queries), a batch (each shard's vote), a query-sharded batch of >= 64 queries per
shard (fingerprint shares exchanged between shards) and coefs = 2 — and every stream tick (channels
split over the shards, or replicated) must equal the single engine over the same clips and the oracle (count(*) DESC, ties to the greatest
audio_uuid: src/fp_handler.c:367-374; clip-aligned shards: :353), including ties whose clips sit on
different shards."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_DB, SEED_Q = 0x7153A1, 0x7153B2
HOP = 256


def _uuids(rng, n):
    out = []
    for _ in range(n):
        h = "%032x" % int.from_bytes(rng.bytes(16), "little")
        out.append("%s-%s-4%s-a%s-%s" % (h[:8], h[8:12], h[13:16], h[17:20], h[20:32]))
    return out


def _oracle_search(oracle, live, q1, q2, qoff, p):
    uu = sorted(live)
    m1 = np.concatenate([live[u][0] for u in uu])
    m2 = np.concatenate([live[u][1] for u in uu])
    clip = np.concatenate([np.full(len(live[u][0]), i, np.int32) for i, u in enumerate(uu)])
    idx = oracle.SortedIndex(m1, m2, clip, np.arange(len(uu), dtype=np.int32))
    w, mc = idx.search_batch(q1, q2, qoff, p.coefs, p.tolerance, p.freq_ignore_low, p.freq_ignore_high, nthreads=16)
    return [(uu[w[i]], int(mc[i])) if w[i] >= 0 else None for i in range(len(qoff) - 1)]


def _pairs(res):
    return [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]


def test_group_of_three_equals_engine_and_oracle(tfp_lib, oracle):
    rng = np.random.default_rng(8)
    n, nsrc = 8000 * 10, 200
    nf = (n + HOP - 1) // HOP
    pcm = tfp_lib.synth_pcm(SEED_DB, range(nsrc), n)
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nsrc + 1) * n, nthreads=16, want_db=False)
    rows = [(micro[c * nf:(c + 1) * nf, 0].copy(), micro[c * nf:(c + 1) * nf, 1].copy()) for c in range(nsrc)]
    # 230 clips: 0..199 plus copies of 0..29 under other uuids (ties, likely on other shards)
    src = list(range(nsrc)) + list(range(30))
    uuids = _uuids(rng, len(src))
    g = tfp_lib.Group([0, 0, 0])
    e = tfp_lib.Engine(0)
    assert g.size() == 3
    live = {}
    fo = np.concatenate([[0], np.cumsum([nf] * 180)])
    for t in (g, e):
        t.index_add_batch(uuids[:180], fo, np.concatenate([rows[src[c]][0] for c in range(180)]),
                          np.concatenate([rows[src[c]][1] for c in range(180)]))
    for c in range(180, len(src)):
        for t in (g, e):
            t.index_add(uuids[c], rows[src[c]][0], rows[src[c]][1])
    for c in range(len(src)):
        live[uuids[c]] = rows[src[c]]
    for c in (3, 77, 181):
        for t in (g, e):
            t.index_remove(uuids[c])
        del live[uuids[c]]
    assert g.index_stats() == e.index_stats() == (len(live) * nf, len(live))
    per = g.engine_stats()
    assert sum(r for r, _ in per) == len(live) * nf and max(r for r, _ in per) - min(r for r, _ in per) <= 2 * nf
    for c in (0, 150, 229):
        a, b = g.index_rows(uuids[c])
        assert np.array_equal(a, rows[src[c]][0]) and np.array_equal(b, rows[src[c]][1])

    # fingerprinting split over the shards == one engine
    off = np.array([0, 5000, 5001, 24000, 24000, 80000, 80255, 160000], np.int64)
    flat = pcm[:2].reshape(-1)
    assert np.array_equal(g.fingerprint_batch(flat, off), e.fingerprint_batch(flat, off))

    # queries: 3 s excerpts (several of tied clips) and unrelated audio
    qn = 8000 * 3
    nq = 3 * 64  # >= 64 per shard: the query-sharded path
    qsrc = [int(rng.integers(nsrc)) if i % 4 != 3 else -1 for i in range(nq)]
    qsrc[:8] = [0, 1, 2, 3, 4, 150, 199, 29]
    qpcm = np.stack([tfp_lib.synth_pcm(SEED_DB, [c], qn, offsets=[256 * int(rng.integers(0, 150))])[0] if c >= 0
                     else tfp_lib.synth_pcm(SEED_Q, [i], qn)[0] for i, c in enumerate(qsrc)])
    _, qdb = oracle.fingerprint_batch(qpcm.reshape(-1), np.arange(nq + 1) * qn, nthreads=16)
    nfq = (qn + HOP - 1) // HOP
    qoff = np.arange(nq + 1, dtype=np.int64) * nfq
    soff = np.arange(nq + 1, dtype=np.int64) * qn
    frames = np.zeros(len(qdb), tfp_lib.FRAME_DTYPE)
    frames["q1"], frames["q2"] = qdb[:, 0], qdb[:, 1]
    found = 0
    for p in (tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.3), tfp_lib.params(2, 0.05)):
        exp = _oracle_search(oracle, live, qdb[:, 0], qdb[:, 1], qoff, p)
        found = max(found, sum(x is not None for x in exp))
        rs, fcs = g.search_pcm_batch(qpcm.reshape(-1), soff, p)          # query-sharded
        assert _pairs(rs) == exp and all(f == nfq for f in fcs), (p.coefs, p.tolerance)
        assert all(r is None or 0 <= r["clip_id"] < 3 for r in rs)
        assert _pairs(e.search_pcm_batch(qpcm.reshape(-1), soff, p)[0]) == exp
        rb, _ = g.search_batch(frames[:24 * nfq], qoff[:25], p)           # each shard's batch search
        assert _pairs(rb) == exp[:24]
        r1, _ = g.search_pcm_batch(qpcm[:4].reshape(-1), soff[:5], p)     # batch-1 path on every shard
        assert _pairs(r1) == exp[:4]
        for i in range(4):
            r, fc = g.search_pcm_batch(qpcm[i], [0, qn], p)
            assert _pairs(r) == exp[i:i + 1] and fc[0] == nfq
    assert found >= 40
    # ties across shards: a clip and its copy under another uuid, added one after the other to an
    # empty group (so they land on different shards, each the lightest at its turn): the query's
    # count ties and the greater uuid wins whichever shard holds it
    t = tfp_lib.Group([0, 0, 0])
    lo_u, hi_u = "10000000-0000-4000-8000-000000000000", "f0000000-0000-4000-8000-000000000000"
    for first, second in ((lo_u, hi_u), (hi_u, lo_u)):
        t.index_clear()
        t.index_add(first, rows[5][0], rows[5][1])
        t.index_add(second, rows[5][0], rows[5][1])
        t.index_add("80000000-0000-4000-8000-000000000000", rows[6][0], rows[6][1])
        assert sorted(r for r, _ in t.engine_stats()) == [nf, nf, nf]  # one clip per shard
        _, q5 = oracle.fingerprint_batch(pcm[5, :qn], np.array([0, qn]), nthreads=1)
        fr = np.zeros(len(q5), tfp_lib.FRAME_DTYPE)
        fr["q1"], fr["q2"] = q5[:, 0], q5[:, 1]
        for p in (tfp_lib.params(1, 0.45), tfp_lib.params(2, 0.45)):
            r, _ = t.search_batch(fr, [0, len(fr)], p)
            assert r[0] is not None and r[0]["audio_uuid"] == hi_u
            r2, _ = t.search_pcm_batch(pcm[5, :qn], [0, qn], p)
            assert r2[0] == r[0]
    t.close()

    # live channels: every tick == the single engine's stream == the oracle on the window, with the
    # channels split over the shards (13 channels: 5 / 4 / 4, the windows exchanged between shards)
    # and replicated on every shard (TFP_GROUP_STREAM=replicate); a channel reset mid-way (its
    # window not full again: no result, the others still matched), coefs = 2, invalid params
    nch, W, tick = 13, 24000, 160
    span = W + 4 * tick
    chs = [int(rng.integers(nsrc)) for _ in range(nch)]
    spcm = tfp_lib.synth_pcm(SEED_DB, chs, span, offsets=[256 * int(rng.integers(0, 100)) for _ in range(nch)])
    spcm[3] = tfp_lib.synth_pcm(SEED_Q + 5, [3], span)[0]
    nfw = (W + HOP - 1) // HOP
    for mode in ("split", "replicate"):
        os.environ["TFP_GROUP_STREAM"] = mode
        try:
            gs = tfp_lib.GroupStream(g, nch, W)
        finally:
            del os.environ["TFP_GROUP_STREAM"]
        es = tfp_lib.Stream(e, nch, W)
        for t in range(W // tick):
            blk = np.ascontiguousarray(spcm[:, t * tick:(t + 1) * tick])
            gs.push(blk)
            es.push(blk)
        for t, p in enumerate((tfp_lib.params(1, 0.001), tfp_lib.params(2, 0.05), tfp_lib.params(1, 0.45),
                               tfp_lib.params(3, 0.001))):
            s0 = W + t * tick
            if t == 2:  # channel 7 (shard 1 of 3 when split) starts over
                gs.reset(7)
                es.reset(7)
            blk = np.ascontiguousarray(spcm[:, s0:s0 + tick])
            rg = gs.push(blk, p)
            assert rg == es.push(blk, p), (mode, t)
            if p.coefs == 3:  # invalid: every channel NULL (fp_handler.c:247-250)
                assert rg == [None] * nch
                continue
            _, wdb = oracle.fingerprint_batch(np.ascontiguousarray(spcm[:, s0 + tick - W:s0 + tick]).reshape(-1),
                                              np.arange(nch + 1) * W, nthreads=16)
            exp = _oracle_search(oracle, live, wdb[:, 0], wdb[:, 1], np.arange(nch + 1) * nfw, p)
            if t >= 2:
                exp[7] = None
            assert _pairs(rg) == exp, (mode, t)
            assert all(r is None or r["frame_count"] == nfw for r in rg)
            assert sum(x is not None for x in exp) >= 6
        gs.reset()
        es.reset()
        blk = np.ascontiguousarray(spcm[:, :tick])
        assert gs.push(blk, tfp_lib.params(1, 0.45)) == [None] * nch  # every window empty again
        gs.close()
        es.close()
    # fewer channels than shards: shard 2 holds none (split)
    gs, es = tfp_lib.GroupStream(g, 2, W), tfp_lib.Stream(e, 2, W)
    for t in range(W // tick + 2):
        blk = np.ascontiguousarray(spcm[:2, t * tick:(t + 1) * tick])
        rg = gs.push(blk, tfp_lib.params(1, 0.45))
        assert rg == es.push(blk, tfp_lib.params(1, 0.45))
    assert rg[0] is not None
    gs.close()
    es.close()
    g.index_clear()
    assert g.index_stats() == (0, 0)
    g.close()
    e.close()


def test_group_add_batch_all_or_nothing(tfp_lib, oracle, monkeypatch):
    """A batch add on a group fails as a whole when one shard's engine fails (a device error,
    injected by TFP_TEST_FAIL_ADD_BATCH on the 5th engine call: the second group batch's middle
    shard call): the shards that took their part drop it again, so no clip stays on a GPU without
    a member (advisor r3: such an orphan could win a search the shim then reports as NOTFOUND and
    never be deleted). The group's clips, rows and every search stay as before the failed batch, and
    the next batch enrols normally."""
    n = 8000 * 4
    nf = (n + HOP - 1) // HOP
    pcm = tfp_lib.synth_pcm(SEED_DB, range(60), n)
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(61) * n, nthreads=16, want_db=False)
    uuids = _uuids(np.random.default_rng(31), 60)
    q = np.ascontiguousarray(pcm[:6, 256 * 10: 256 * 10 + 16000])
    p = tfp_lib.params(1, 0.45)

    def batch(g, a, b):
        fo = np.arange(b - a + 1, dtype=np.int64) * nf
        g.index_add_batch(uuids[a:b], fo, micro[a * nf:b * nf, 0], micro[a * nf:b * nf, 1])

    monkeypatch.setenv("TFP_TEST_FAIL_ADD_BATCH", "5")
    g = tfp_lib.Group([0, 0, 0])
    try:
        batch(g, 0, 30)  # engine calls 1-3
        before = (g.index_stats(), _pairs(g.search_pcm_batch(q.reshape(-1), np.arange(7) * 16000, p)[0]))
        with pytest.raises(tfp_lib.TfpError):
            batch(g, 30, 45)  # calls 4-6: the 5th fails
        assert g.index_stats() == before[0]
        assert sum(c for _, c in g.engine_stats()) == 30  # nothing of the failed batch left on any engine
        assert _pairs(g.search_pcm_batch(q.reshape(-1), np.arange(7) * 16000, p)[0]) == before[1]
        for u in uuids[30:45]:  # never members: removal reports them missing
            with pytest.raises(tfp_lib.TfpError):
                g.index_remove(u)
        batch(g, 30, 60)  # calls 7-9
        assert g.index_stats()[1] == 60
        live = {uuids[c]: (micro[c * nf:(c + 1) * nf, 0], micro[c * nf:(c + 1) * nf, 1]) for c in range(60)}
        _, qdb = oracle.fingerprint_batch(q.reshape(-1), np.arange(7) * 16000, nthreads=16)
        exp = _oracle_search(oracle, live, qdb[:, 0], qdb[:, 1], np.arange(7) * ((16000 + HOP - 1) // HOP), p)
        assert _pairs(g.search_pcm_batch(q.reshape(-1), np.arange(7) * 16000, p)[0]) == exp
    finally:
        g.close()


def test_group_enrolment_is_o_new_clips(oracle, tfp_lib):
    """Single-clip enrolments into a populated group (the shim's fp_craete_audio_list_info path,
    src/fp_handler.c:538-575 / src/app_tiresias.c:365-424; the clip is searchable at once,
    :559-571): each new clip takes the middle of its uuid neighbours' tie-key gap, so no other key
    changes and the shards get the new clips' keys only (tfp_index_update_tiebreak); their index
    delta updates do not re-send the main columns' keys. Every batch-1 search after an add, and after
    removals of an old and of a new clip, == the oracle over the live rows (ties to the greatest
    uuid across shards)."""
    import test_gpu_index as tgi
    rng = np.random.default_rng(9191)
    n0, nadd = 3000, 40
    data = tgi._dense_db(rng, n0 + nadd, 30)
    uu = _uuids(rng, n0 + nadd)
    uu[n0 + 5] = "00000000-0000-4000-8000-000000000001"  # a new first uuid
    uu[n0 + 6] = "ffffffff-ffff-4fff-bfff-ffffffffffff"  # a new last uuid
    uu[n0 + 7] = uu[10][:-1] + ("0" if uu[10][-1] != "0" else "1")  # a neighbour of an old uuid
    data[n0 + 8] = data[20]  # a copy of an old clip's rows: a tie decided by the uuid across shards
    old = os.environ.get("TFP_INDEX_DELTA")
    os.environ["TFP_INDEX_DELTA"] = "1"  # (test knob: the index delta at this DB size too)
    try:
        g = tfp_lib.Group([0, 0])
    finally:
        if old is None:
            del os.environ["TFP_INDEX_DELTA"]
        else:
            os.environ["TFP_INDEX_DELTA"] = old
    live = {}
    p = tfp_lib.params(1, 0.001)
    try:
        foff = np.concatenate([[0], np.cumsum([len(data[c][0]) for c in range(n0)])]).astype(np.int64)
        g.index_add_batch(uu[:n0], foff, np.concatenate([data[c][0] for c in range(n0)]),
                          np.concatenate([data[c][1] for c in range(n0)]))
        for c in range(n0):
            live[uu[c]] = data[c]
        g.index_commit()
        st0 = g.tiebreak_stats()
        found = 0

        def check(src):
            q = []
            for c in src:
                m1, m2 = data[c]
                sel = rng.integers(0, len(m1), 25)
                q.append(np.stack([m1[sel] / 1e6 + 0.0004, m2[sel] / 1e6], axis=1))
            qdb = np.concatenate(q)
            qoff = np.arange(len(src) + 1, dtype=np.int64) * 25
            exp = _oracle_search(oracle, live, qdb[:, 0], qdb[:, 1], qoff, p)
            fr = np.zeros(len(qdb), tfp_lib.FRAME_DTYPE)
            fr["q1"], fr["q2"] = qdb[:, 0], qdb[:, 1]
            for i in range(len(src)):
                res, _ = g.search_batch(fr[qoff[i]:qoff[i + 1]], [0, 25], p)  # batch-1
                got = None if res[0] is None else (res[0]["audio_uuid"], res[0]["match_count"])
                assert got == exp[i], (i, src[i])
            return sum(e is not None for e in exp)

        for j in range(nadd):
            c = n0 + j
            g.index_add(uu[c], *data[c])
            live[uu[c]] = data[c]
            found += check([c, int(rng.integers(n0)), 20])
        st = g.tiebreak_stats()
        # the first enrolment's respace only; one push of new keys per add; at most one full key
        # upload per shard (the first delta update widens the rows: a larger key buffer)
        assert st["respaces"] == st0["respaces"], (st0, st)
        assert st["partial_pushes"] - st0["partial_pushes"] >= nadd, (st0, st)
        assert st["shard_full_key_updates"] - st0["shard_full_key_updates"] <= 2, (st0, st)
        for u in (uu[33], uu[n0 + 3]):  # an old clip and a new one removed
            g.index_remove(u)
            del live[u]
        found += check([n0 + 4, 20, n0 + 8, int(rng.integers(n0))])
        assert found > nadd
    finally:
        g.close()
