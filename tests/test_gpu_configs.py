"""GPU parity at the BASELINE.json configs' own sizes.

Each test runs the device path the bench times, at the bench's size, and checks every result
against the CPU oracle (oracle/, the reference path restated; reference semantics
src/fp_handler.c:287-374 for the search, :577-671 for the fingerprint):

  configs[1]  1,024 x 30 s clips in one launch: every one of the 960,512 stored (m1, m2) rows,
              i.e. the persistent kernel's multi-tile loop (~29 tiles per wave) and its
              next-tile prefetch, which smaller batches never reach.
  configs[2]  the 100k-clip DB (93.8 M rows) and 5 s queries: the batch vote (class path and
              the Bt GEMM over 98 1,024-clip chunks) and the batch-1 path, against the oracle's
              sorted-index search over the same rows.
  vote chunks ties straddling 1,024-clip chunk boundaries (the GEMM's cross-chunk max), with
              the pattern-class vote and with the GEMM forced (TFP_VOTE_CLASS_MAX=-1).
  configs[4]  512 live channels: one tick's results on sampled channels vs the oracle on each
              channel's last window.
"""
import os

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

SEED_DB, SEED_Q = 0x7153A1, 0x7153B2
HOP = 256
ORACLE_THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _uuid_of(g: int) -> str:
    """bench.py's deterministic uuid per global clip id."""
    a = (g * 0x9E3779B97F4A7C15 + 0x7153A1) & (2**64 - 1)
    b = (a * 0xBF58476D1CE4E5B9 + g) & (2**64 - 1)
    s = "%032x" % ((a << 64) | b)
    s = s[:12] + "4" + s[13:16] + "89ab"[int(s[16], 16) & 3] + s[17:]
    return "%s-%s-%s-%s-%s" % (s[:8], s[8:12], s[12:16], s[16:20], s[20:32])


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


def test_configs1_full_batch_bit_exact(engine, oracle, torch_cuda):
    """configs[1] as bench.py runs it: 1,024 x 30 s clips synthesised in HBM, one plan, one
    tfp_fingerprint_device launch (+ finish_db). All 960,512 rows == the oracle's, bit for bit;
    the frame values (q1, q2) of a second launch with d_db equal glibc's bit for bit."""
    torch = torch_cuda
    nclips, n = 1024, 8000 * 30
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    pcm = torch.empty((nclips, n), dtype=torch.int16, device=dev)
    engine.synth_device(SEED_DB, range(nclips), n, pcm.data_ptr(), stream=stream)
    off = np.arange(nclips + 1, dtype=np.int64) * n
    plan = engine.plan(off)
    assert plan.nframes == 960512
    micro = torch.empty((plan.nframes, 2), dtype=torch.int32, device=dev)
    engine.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    host = pcm.cpu().numpy().reshape(-1)
    exp, db = oracle.fingerprint_batch(host, off, nthreads=ORACLE_THREADS)
    got = micro.cpu().numpy()
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert len(bad) == 0, ("frames differing", len(bad), bad[:10])
    # with the frame values (the query path's d_db)
    micro.fill_(0)
    qv = torch.empty((plan.nframes, 2), dtype=torch.float64, device=dev)
    engine.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), qv.data_ptr(), stream)
    torch.cuda.synchronize()
    assert np.array_equal(micro.cpu().numpy(), exp)
    q = qv.cpu().numpy()
    assert np.array_equal(q.view(np.uint64), db.view(np.uint64))  # glibc's 10*log10|c|, bit for bit


def _chunk_tie_index(eng, nclips, nkeys, seed):
    """nclips clips whose uuids sort like their numbers (column = uuid rank = clip number).
    Groups g = 0..3 are the column pairs (1024 (g+1) - 1, 1024 (g+1)) on either side of a
    1,024-clip vote chunk boundary, each with a row in every key's box but key g's; every other
    clip has rows in a random ~30 % of the keys' boxes, never in more than two of the boxes of
    keys 0..3 (so it cannot reach a group's count). Rows are added in shuffled order."""
    rng = np.random.default_rng(seed)
    uuids = ["%08x-0000-4000-8000-%012x" % (c, c) for c in range(nclips)]
    group = {}
    for g in range(4):
        group[1024 * (g + 1) - 1] = g
        group[1024 * (g + 1)] = g
    m1s, m2s, clips = [], [], []
    for c in range(nclips):
        if c in group:
            keys = [k for k in range(nkeys) if k != group[c]]
        else:
            drop = set(rng.choice(4, 2, replace=False).tolist())
            keys = [k for k in range(nkeys) if k not in drop and rng.random() < 0.3]
        keys = np.asarray(keys, np.int64)
        m1s.append((keys * 1000000 + rng.integers(-900, 901, len(keys))).astype(np.int32))
        m2s.append(rng.integers(-5000000, 5000000, len(keys)).astype(np.int32))
        clips.append(np.full(len(keys), c, np.int32))
    order = rng.permutation(nclips)
    eng.index_clear()
    fo = np.concatenate([[0], np.cumsum([len(m1s[c]) for c in order])])
    eng.index_add_batch([uuids[c] for c in order], fo, np.concatenate([m1s[c] for c in order]),
                        np.concatenate([m2s[c] for c in order]))
    return uuids, np.concatenate(m1s), np.concatenate(m2s), np.concatenate(clips)


@pytest.mark.parametrize("class_max", ["10", "-1"])
@pytest.mark.parametrize("nkeys", [6, 12])
def test_vote_ties_across_chunk_boundaries(oracle, tfp_lib, class_max, nkeys):
    """>= 4 GEMM chunks (4,200 clips). Query q has frames on every group key but e (0..3), so
    only group e reaches the query's full count: its two columns tie across the chunk boundary
    and the later one (greater uuid) must win. nkeys = 6 takes the pattern-class vote unless
    TFP_VOTE_CLASS_MAX=-1 forces the GEMM; nkeys = 12 always takes the GEMM."""
    eng = _engine_with(tfp_lib, {"TFP_VOTE_CLASS_MAX": class_max})
    try:
        nclips = 4200
        uuids, m1, m2, clip = _chunk_tie_index(eng, nclips, nkeys, 5 + nkeys)
        rng = np.random.default_rng(nkeys)
        q1s, qoff, expect_col = [], [0], []
        for i in range(48):
            e = i % 4 if i % 6 else int(rng.integers(4))
            keys = [k for k in range(nkeys) if k != e and (k < 4 or rng.random() < 0.8)]
            cnt = rng.integers(1, 6, len(keys))
            q = np.repeat(np.asarray(keys, np.float64), cnt) + rng.choice([0.2, 0.6], int(cnt.sum()))
            q1s.append(rng.permutation(q))
            qoff.append(qoff[-1] + len(q))
            expect_col.append(1024 * (e + 1))
        q1 = np.concatenate(q1s)
        q2 = np.zeros_like(q1)
        fr = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                         ("q1", "<f8"), ("q2", "<f8")]))
        fr["q1"], fr["q2"] = q1, q2
        res, fcs = eng.search_batch(fr, np.asarray(qoff), tfp_lib.params(1, 0.001))
        at_boundary = 0
        for i in range(len(qoff) - 1):
            a, b = qoff[i], qoff[i + 1]
            found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[a:b], q2[a:b], 1, 0.001, -1, -1)
            exp = (uuids[w], mc) if found else None
            got = None if res[i] is None else (res[i]["audio_uuid"], res[i]["match_count"])
            assert got == exp, (i, class_max, nkeys)
            assert fcs[i] == fc == b - a
            at_boundary += found and w == expect_col[i]
        assert at_boundary == len(qoff) - 1  # the construction put every winner on a boundary
    finally:
        eng.close()


def _enroll_db(eng, torch, dev, stream, ids, keep_rows=True, chunk=2048, oracle=None, check_every=0):
    """bench.py's enrolment (synth -> fingerprint_device -> index_add_device, 2,048 clips at a
    time) that also returns the rows it enrolled (host int32 [nclips * 938, 2]). With an oracle,
    every check_every-th clip's enrolled rows are compared with the oracle's fingerprints of the
    same PCM (copied back from the device buffer the kernel read). Returns (rows, clips checked)."""
    n_db = 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    buf = torch.empty((chunk, n_db), dtype=torch.int16, device=dev)
    micro = torch.empty((chunk * nf_db, 2), dtype=torch.int32, device=dev)
    rows = np.empty((len(ids) * nf_db, 2), np.int32) if keep_rows else None
    checked = 0
    eng.index_clear()
    for s in range(0, len(ids), chunk):
        part = ids[s:s + chunk]
        k = len(part)
        plan = eng.plan(np.arange(k + 1, dtype=np.int64) * n_db)
        eng.synth_device(SEED_DB, part, n_db, buf.data_ptr(), stream=stream)
        eng.fingerprint_device(plan, buf.data_ptr(), micro.data_ptr(), 0, stream)
        eng.index_add_device([_uuid_of(g) for g in part], np.arange(k + 1, dtype=np.int64) * nf_db, micro.data_ptr(),
                             stream)
        if keep_rows or check_every:
            torch.cuda.synchronize()
            got = micro[:k * nf_db].cpu().numpy()
            if keep_rows:
                rows[s * nf_db:(s + k) * nf_db] = got
            if check_every:
                sel = [i for i in range(k) if part[i] % check_every == 0]
                pcm = buf[torch.tensor(sel, device=dev)].cpu().numpy().reshape(-1)
                exp, _ = oracle.fingerprint_batch(pcm, np.arange(len(sel) + 1) * n_db, nthreads=ORACLE_THREADS,
                                                  want_db=False)
                g = np.concatenate([got[i * nf_db:(i + 1) * nf_db] for i in sel])
                bad = np.nonzero((g != exp).any(axis=1))[0]
                assert len(bad) == 0, ("enrolled rows differ from the oracle", s, len(bad))
                checked += len(sel)
    eng.index_commit()
    torch.cuda.synchronize()
    del buf, micro
    torch.cuda.empty_cache()
    return rows, checked


def _c3_queries(nq, db_clips, seed=SEED_Q):
    """bench.py's configs[2] query mix: 75 % 5 s excerpts of DB clips at 256-aligned offsets,
    25 % unrelated audio."""
    rng = np.random.default_rng(seed)
    n_db, qn = 8000 * 30, 8000 * 5
    spec = []
    for i in range(nq):
        if i % 4 != 3:
            spec.append((SEED_DB, int(rng.integers(db_clips)), 256 * int(rng.integers(0, (n_db - qn) // HOP))))
        else:
            spec.append((SEED_Q, i, 0))
    return spec


@pytest.fixture(scope="module")
def c3db(oracle, tfp_lib, torch_cuda):
    """configs[2]'s DB: 100,000 x 30 s clips (93.8 M rows) enrolled on the device as bench.py does
    (own engine), the rows of every 16th clip (6,250 clips, 5.9 M rows) checked against the
    oracle's fingerprints of the same PCM, a 64-clip sample of the host synthesiser's PCM against
    the device's, and the oracle's sorted index over the same rows (tie key = rank of the uuid
    among all clips)."""
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    eng = tfp_lib.Engine(0)
    db_clips, n_db = 100_000, 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    rows, checked = _enroll_db(eng, torch, dev, stream, list(range(db_clips)), oracle=oracle, check_every=16)
    assert checked == 6250
    nrows, nc = eng.index_stats()
    assert nc == db_clips and nrows == db_clips * nf_db
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(db_clips, 64, replace=False))
    pcm = tfp_lib.synth_pcm(SEED_DB, sample.tolist(), n_db)  # host synthesiser (the oracle's PCM above came from the device)
    exp, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(len(sample) + 1) * n_db, nthreads=ORACLE_THREADS,
                                      want_db=False)
    got = np.concatenate([rows[c * nf_db:(c + 1) * nf_db] for c in sample])
    assert np.array_equal(got, exp)
    uuids = [_uuid_of(g) for g in range(db_clips)]
    order = np.argsort(np.asarray(uuids))
    rank = np.empty(db_clips, np.int32)
    rank[order] = np.arange(db_clips, dtype=np.int32)
    idx = oracle.SortedIndex(rows[:, 0], rows[:, 1], np.repeat(np.arange(db_clips, dtype=np.int32), nf_db), rank)
    del rows
    yield {"eng": eng, "idx": idx, "uuids": uuids, "rank": rank, "db_clips": db_clips}
    eng.close()


def _c3_batch(c3db, tfp_lib, torch, nq, seed=SEED_Q):
    qn = 8000 * 5
    spec = _c3_queries(nq, c3db["db_clips"], seed)
    qpcm = np.stack([tfp_lib.synth_pcm(sd, [c], qn, offsets=[o])[0] for sd, c, o in spec])
    return qpcm, torch.from_numpy(qpcm).to("cuda")


def _oracle_q(oracle, qpcm):
    nfq = (qpcm.shape[1] + HOP - 1) // HOP
    qoff = np.arange(len(qpcm) + 1, dtype=np.int64) * nfq
    _, qdb = oracle.fingerprint_batch(np.ascontiguousarray(qpcm).reshape(-1), np.arange(len(qpcm) + 1) * qpcm.shape[1],
                                      nthreads=ORACLE_THREADS)
    return qdb, qoff


def _check_keys(c3db, tfp_lib, torch, qpcm, d_q, qdb, qoff, p, nthreads=ORACLE_THREADS):
    """The device path's key per query (search_device on the queries' PCM) == the oracle's over the
    same rows. coefs = 2 batches take the oracle's per-box form (oracle_boxes.c): at a wide tolerance
    one row scan per frame clause would read tens of millions of rows per frame."""
    eng, idx, rank = c3db["eng"], c3db["idx"], c3db["rank"]
    w, mc = idx.search_batch(qdb[:, 0], qdb[:, 1], qoff, p.coefs, p.tolerance, p.freq_ignore_low, p.freq_ignore_high,
                             nthreads=nthreads, method="boxes" if p.coefs == 2 else "scan")
    keys = torch.zeros(len(qpcm), dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    eng.search_device(eng.plan(np.arange(len(qpcm) + 1, dtype=np.int64) * qpcm.shape[1]), d_q.data_ptr(), p,
                      keys.data_ptr(), stream)
    torch.cuda.synchronize()
    k = keys.cpu().numpy().view(np.uint64)
    expk = np.where(w >= 0, (mc.astype(np.uint64) << np.uint64(32)) | rank[np.maximum(w, 0)].astype(np.uint64), 0)
    assert np.array_equal(k, expk.astype(np.uint64)), (p.coefs, p.tolerance, np.nonzero(k != expk)[0][:8])
    return w, mc


def test_configs2_full_db_vs_sorted_oracle(c3db, oracle, tfp_lib, torch_cuda):
    """configs[2]: 5 s queries against all 100,000 clips. The batch device path (vote; tol 0.001
    and 0.1) and the batch-1 host path, each (count, uuid rank) == the oracle's sorted-index
    search over the same 93.8 M rows."""
    torch = torch_cuda
    qpcm, d_q = _c3_batch(c3db, tfp_lib, torch, 96)
    qdb, qoff = _oracle_q(oracle, qpcm)
    for tol in (0.001, 0.1):
        w, _ = _check_keys(c3db, tfp_lib, torch, qpcm, d_q, qdb, qoff, tfp_lib.params(1, tol))
        assert (w >= 0).sum() >= len(qpcm) // 4
    # batch-1 (small path), host PCM in -> result out, as the dialplan application calls it
    w, mc = c3db["idx"].search_batch(qdb[:, 0], qdb[:, 1], qoff, 1, 0.001, nthreads=ORACLE_THREADS)
    nfq = int(qoff[1])
    for i in range(16):
        res, fc = c3db["eng"].search_pcm_batch(qpcm[i], [0, qpcm.shape[1]], tfp_lib.params(1, 0.001))
        got = None if res[0] is None else (res[0]["audio_uuid"], res[0]["match_count"])
        assert got == ((c3db["uuids"][w[i]], int(mc[i])) if w[i] >= 0 else None), i
        assert fc[0] == nfq


@pytest.mark.parametrize("coefs,tol,low,high,nq", [(2, 0.001, -1, -1, 512), (2, 0.01, -1, -1, 512), (2, 0.1, -1, -1, 512),
                                                   (2, 0.45, -1, -1, 512), (1, 0.45, -1, -1, 64),
                                                   (1, 0.01, 100, 3400, 64), (2, 0.1, 100, 3400, 512),
                                                   (2, 0.45, 100, 3400, 512), (1, 0.001, 50, 60, 64),
                                                   (2, 0.01, 50, 60, 512), (2, 0.45, 50, 60, 512)])
def test_configs2_sweeps_vs_sorted_oracle(c3db, oracle, tfp_lib, torch_cuda, coefs, tol, low, high, nq):
    """SURVEY §8(d)'s configs[2] sweeps at full DB size: coefs = 2 (the general path over the
    m2-ordered key segments, src/fp_handler.c:318-351), wider tolerances and the ignore filter
    (:293-306, :324-337) — every key == the oracle's. 100/3400 Hz drops ~92% of the synthetic
    frames (max1 ~17 dB < 20 dB) and matches nothing; 50/60 Hz (16.99/17.78 dB) keeps about a third
    and still matches, and drops the max2 condition of the frames whose max2 falls outside it (the
    case whose 16-bit count pairs once borrowed across the halves: round 3, golden rand_05), so the
    filter's kept/dropped split is exercised on both sides. Every coefs = 2 setting runs 512 queries:
    the 5 s queries have 157 frames (< 256), so the sweep takes 256-query chunks with four 8-bit
    counts per lane word, and 512 queries are two full chunks. At tolerance 0.45 every (key, clip)
    group of a chunk's keys is one long cluster of the clip-major sweep (bench.py times the coefs = 2
    settings on all 4,096)."""
    torch = torch_cuda
    qpcm, d_q = _c3_batch(c3db, tfp_lib, torch, nq, SEED_Q + coefs)
    qdb, qoff = _oracle_q(oracle, qpcm)
    w, _ = _check_keys(c3db, tfp_lib, torch, qpcm, d_q, qdb, qoff, tfp_lib.params(coefs, tol, low, high))
    if low == 50 or (low < 0 and tol >= 0.1):
        assert (w >= 0).sum() > 0  # the filter keeps frames that still match


def test_configs4_512_channels_one_tick(engine, oracle, tfp_lib, torch_cuda):
    """configs[4]: 512 live channels, 160-sample ticks, 3 s windows (94 frames). After the windows
    fill, each tick's result of 32 sampled channels == the oracle's search on that channel's last
    24,000 samples (the recording the dialplan application would have searched)."""
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    db_clips, n_db, W, tick = 3000, 8000 * 30, 24000, 160
    nf_db = (n_db + HOP - 1) // HOP
    rows, _ = _enroll_db(engine, torch, dev, stream, list(range(db_clips)))
    uuids = [_uuid_of(g) for g in range(db_clips)]
    order = np.argsort(np.asarray(uuids))
    rank = np.empty(db_clips, np.int32)
    rank[order] = np.arange(db_clips, dtype=np.int32)
    idx = oracle.SortedIndex(rows[:, 0], rows[:, 1], np.repeat(np.arange(db_clips, dtype=np.int32), nf_db), rank)
    nch, ticks = 512, 3
    rng = np.random.default_rng(44)
    span = W + ticks * tick
    src = [int(rng.integers(db_clips)) for _ in range(nch)]
    offs = [256 * int(rng.integers(0, (n_db - span) // HOP)) + int(rng.integers(0, 4)) * 40 for _ in range(nch)]
    pcm = tfp_lib.synth_pcm(SEED_DB, src, span, offsets=offs)
    for c in range(3, nch, 4):  # unrelated audio on every 4th channel
        pcm[c] = tfp_lib.synth_pcm(SEED_Q + 7, [c], span)[0]
    st = tfp_lib.Stream(engine, nch, W)
    p = tfp_lib.params(1, 0.001)
    for t in range(W // tick):
        st.push(np.ascontiguousarray(pcm[:, t * tick:(t + 1) * tick]))
    checked = found = 0
    for t in range(ticks):
        s0 = W + t * tick
        res = st.push(np.ascontiguousarray(pcm[:, s0:s0 + tick]), p)
        chans = rng.choice(nch, 32, replace=False)
        qdb = np.concatenate([oracle.fingerprint(pcm[c, s0 + tick - W:s0 + tick])[1] for c in chans])
        nfw = (W + HOP - 1) // HOP
        w, mc = idx.search_batch(qdb[:, 0], qdb[:, 1], np.arange(len(chans) + 1) * nfw, 1, 0.001,
                                 nthreads=ORACLE_THREADS)
        for i, c in enumerate(chans):
            exp = {"audio_uuid": uuids[w[i]], "match_count": int(mc[i]), "frame_count": nfw} if w[i] >= 0 else None
            assert res[c] == exp, (t, int(c))
            checked += 1
            found += w[i] >= 0
    assert checked == 96 and found > 20
    st.close()
    engine.index_clear()


def _bench_batch(c3db, torch, nq=4096):
    """The exact query batch bench.py times at configs[2] (bench.c3_queries), device and host."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    dev = torch.device("cuda", 0)
    d_q = bench.c3_queries(c3db["eng"], torch, dev, torch.cuda.current_stream().cuda_stream, nq, c3db["db_clips"])
    return d_q.cpu().numpy(), d_q


@pytest.mark.timeout(900)
def test_configs2_timed_batch_all_4096_vs_sorted_oracle(c3db, oracle, tfp_lib, torch_cuda):
    """The batch bench.py times (4,096 x 5 s queries, coefs = 1, tolerance 0.001, the vote path),
    every one of its keys == the oracle's sorted-index search over the same 93.8 M rows; and the
    bench's coefs = 2 sweeps of the same batch, all 4,096 queries (16 sweep chunks of 256 queries
    with 8-bit counts, src/fp_handler.c:318-351) at tolerance 0.001 and at 0.45 (its widest, the
    clip-major sweep's longest clusters), at full DB size."""
    torch = torch_cuda
    qpcm, d_q = _bench_batch(c3db, torch)
    qdb, qoff = _oracle_q(oracle, qpcm)
    w, _ = _check_keys(c3db, tfp_lib, torch, qpcm, d_q, qdb, qoff, tfp_lib.params(1, 0.001))
    assert (w >= 0).sum() >= 1000  # (the bench reports ~1,500 found)
    eng = c3db["eng"]
    for tol in (0.001, 0.45):
        st0 = eng.sweep_stats()
        w2, _ = _check_keys(c3db, tfp_lib, torch, qpcm, d_q, qdb, qoff, tfp_lib.params(2, tol))
        assert (w2 >= 0).sum() > 0
        # every batch of the check took the hand-written bin sort, none the library sort or a redo
        # (tfp_sweep_stats), and the silence-floor crowd was copied unsorted
        st = {k: v - st0[k] for k, v in eng.sweep_stats().items()}
        assert st["bins"] >= 1 and st["library"] == 0 and st["redone"] == 0 and st["crowd"] >= 1, (tol, st)


@pytest.mark.timeout(900)
def test_configs4_stream_ticks_against_the_100k_db(c3db, oracle, tfp_lib, torch_cuda):
    """configs[4] at the DB size bench.py times it against (src/application_handler.c:152-185,
    248-312: each channel's last 3 s searched every tick): 512 channels of 160-sample ticks over the
    100,000-clip DB, through tfp_stream on the DB's engine and through tfp_group_stream on a
    two-shard group (devices 0, 0: channels split over the shards, window frame values exchanged)
    holding the same clips. Each tick's results of 32 sampled channels == the oracle's sorted-index
    search (93.8 M rows) of that channel's last 24,000 samples."""
    torch = torch_cuda
    eng, idx, uuids, db_clips = c3db["eng"], c3db["idx"], c3db["uuids"], c3db["db_clips"]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    n_db, W, tick, nch, ticks = 8000 * 30, 24000, 160, 512, 3
    nf_db = (n_db + HOP - 1) // HOP
    nfw = (W + HOP - 1) // HOP
    rng = np.random.default_rng(4545)
    span = W + ticks * tick
    src = [int(rng.integers(db_clips)) for _ in range(nch)]
    offs = [256 * int(rng.integers(0, (n_db - span) // HOP)) + int(rng.integers(0, 4)) * 40 for _ in range(nch)]
    pcm = tfp_lib.synth_pcm(SEED_DB, src, span, offsets=offs)
    for c in range(3, nch, 4):  # unrelated audio on every 4th channel
        pcm[c] = tfp_lib.synth_pcm(SEED_Q + 9, [c], span)[0]
    p = tfp_lib.params(1, 0.001)

    def run(st, label):
        for t in range(W // tick):
            st.push(np.ascontiguousarray(pcm[:, t * tick:(t + 1) * tick]))
        checked = found = 0
        for t in range(ticks):
            s0 = W + t * tick
            res = st.push(np.ascontiguousarray(pcm[:, s0:s0 + tick]), p)
            chans = rng.choice(nch, 32, replace=False)
            qdb = np.concatenate([oracle.fingerprint(pcm[c, s0 + tick - W:s0 + tick])[1] for c in chans])
            w, mc = idx.search_batch(qdb[:, 0], qdb[:, 1], np.arange(len(chans) + 1) * nfw, 1, 0.001,
                                     nthreads=ORACLE_THREADS)
            for i, c in enumerate(chans):
                exp = {"audio_uuid": uuids[w[i]], "match_count": int(mc[i]), "frame_count": nfw} if w[i] >= 0 else None
                assert res[c] == exp, (label, t, int(c))
                checked += 1
                found += w[i] >= 0
        assert checked == 32 * ticks and found > 20, (label, found)

    st = tfp_lib.Stream(eng, nch, W)
    try:
        run(st, "engine")
    finally:
        st.close()
    # the same clips in a two-shard device group, enrolled from the DB engine's fingerprints
    g = tfp_lib.Group([0, 0])
    try:
        chunk = 2048
        buf = torch.empty((chunk, n_db), dtype=torch.int16, device=dev)
        micro = torch.empty((chunk * nf_db, 2), dtype=torch.int32, device=dev)
        for s0 in range(0, db_clips, chunk):
            ids = list(range(s0, min(db_clips, s0 + chunk)))
            k = len(ids)
            eng.synth_device(SEED_DB, ids, n_db, buf.data_ptr(), stream=stream)
            eng.fingerprint_device(eng.plan(np.arange(k + 1, dtype=np.int64) * n_db), buf.data_ptr(), micro.data_ptr(), 0,
                                   stream)
            torch.cuda.synchronize()
            rows = micro[:k * nf_db].cpu().numpy()
            g.index_add_batch([uuids[i] for i in ids], np.arange(k + 1, dtype=np.int64) * nf_db, rows[:, 0], rows[:, 1])
        del buf, micro
        torch.cuda.empty_cache()
        g.index_commit()
        assert sum(c for _, c in g.engine_stats()) == db_clips
        gs = tfp_lib.GroupStream(g, nch, W)
        try:
            run(gs, "group")
        finally:
            gs.close()
    finally:
        g.close()


def noise_clips(n, nsamples, seed=0x7153C3):
    """Full-scale white noise clips (int16): their max1 values sit at 16.19-16.25 dB, below every
    configs[2] DB row (>= 16.6 dB), so key 16's box at tolerance 0.45 ([15.55, 16.45] dB) holds
    only these clips' rows. A coefs = 1, tolerance 0.45 query cut from one can only be won by a
    noise clip (ties between them: the greatest uuid, src/fp_handler.c:367-374)."""
    rng = np.random.default_rng(seed)
    return rng.integers(-32768, 32768, (n, nsamples)).astype(np.int16)


def new_clip_uuid(i: int) -> str:
    """uuids above every _uuid_of(): the i-th enrolled noise clip sorts after all clips before it."""
    return "ffffffff-ffff-4fff-bfff-%012x" % i


@pytest.mark.timeout(900)
def test_updated_index_at_100k_clips_vs_full_build_and_oracle(c3db, oracle, tfp_lib, torch_cuda):
    """The enrolled index as single-clip enrolments leave it at configs[2] size (the reference's
    INSERTs into its max1 B-tree, src/fp_handler.c:559-571, :745-753: a clip is searchable at once):
    8 single-clip tfp_index_add calls and one removal of a clip the queries hit. The new clips are 7
    noise clips (noise_clips: after each add, a batch-1 search of an excerpt at coefs 1, tolerance
    0.45 must return the clip just added, which only its own rows can make win) and a copy of a DB
    clip's audio under a new uuid (a tie across old and new rows, decided by the uuid). Then a
    query batch (512 configs[2] queries + 32 excerpts of the new clips) at coefs 1 (vote) and 2
    (sweep): every key == an engine forced to full re-sorts (TFP_INDEX_FULL) over the same
    operations == the oracle's sorted index over the live rows. Runs last in the module: it changes
    the shared DB."""
    torch = torch_cuda
    eng, idx, db_clips = c3db["eng"], c3db["idx"], c3db["db_clips"]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    n_db, qn = 8000 * 30, 8000 * 5
    nf_db = (n_db + HOP - 1) // HOP
    assert int(idx.m1[(idx.m1 != oracle.NULL_MICRO) & (idx.m1 < 16_450_000)].size) == 0  # key 16's box at 0.45 is empty
    full = _engine_with(tfp_lib, {"TFP_INDEX_FULL": "1"})
    try:
        _enroll_db(full, torch, dev, stream, list(range(db_clips)), keep_rows=False)
        fb0, _ = eng.index_build_stats()
        spec = _c3_queries(512, db_clips, SEED_Q + 11)
        victim = spec[0][1]  # a DB clip the first query is an excerpt of
        copy_of = spec[1][1]
        new_pcm = np.concatenate([noise_clips(7, n_db), tfp_lib.synth_pcm(SEED_DB, [copy_of], n_db)])
        new_rows, _ = oracle.fingerprint_batch(new_pcm.reshape(-1), np.arange(9) * n_db, nthreads=ORACLE_THREADS,
                                               want_db=False)
        new_uuids = [new_clip_uuid(i) for i in range(7)] + [_uuid_of(10**7 + copy_of)]
        rows_m1, rows_m2, rows_clip = [idx.m1], [idx.m2], [idx.clip]
        uuids = list(c3db["uuids"])
        rng = np.random.default_rng(5)
        live = np.ones(db_clips + 8, bool)
        p1, p45 = tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.45)
        for i in range(8):
            m = new_rows[i * nf_db:(i + 1) * nf_db]
            for e in (eng, full):
                e.index_add(new_uuids[i], m[:, 0], m[:, 1])
            uuids.append(new_uuids[i])
            rows_m1.append(m[:, 0].copy())
            rows_m2.append(m[:, 1].copy())
            rows_clip.append(np.full(nf_db, db_clips + i, np.int32))
            if i == 4:
                for e in (eng, full):
                    e.index_remove(_uuid_of(victim))
                live[victim] = False
            # batch-1 searches of an excerpt of the new clip (the dialplan's call, application_handler.c:180)
            o = 256 * int(rng.integers(0, (n_db - qn) // HOP))
            q = np.ascontiguousarray(new_pcm[i, o:o + qn])
            for p in (p1, p45):
                got = [e.search_pcm_batch(q, [0, qn], p)[0][0] for e in (eng, full)]
                assert got[0] == got[1], (i, p.tolerance)
                if i < 7 and p is p45:
                    assert got[0] is not None and got[0]["audio_uuid"] == new_uuids[i], (i, got[0])
        assert eng.index_build_stats()[0] == fb0  # no full re-sort of the 100k-clip index
        r1, r2, rc = (np.concatenate(a) for a in (rows_m1, rows_m2, rows_clip))
        keep = live[rc]
        rank = np.full(len(uuids), -1, np.int32)
        for r, (_, c) in enumerate(sorted((u, c) for c, u in enumerate(uuids) if live[c])):
            rank[c] = r
        oidx = oracle.SortedIndex(r1[keep], r2[keep], rc[keep], rank)
        del r1, r2, rc, keep
        qpcm = [tfp_lib.synth_pcm(sd, [c], qn, offsets=[o])[0] for sd, c, o in spec]
        for i in range(8):
            for _ in range(4):
                o = 256 * int(rng.integers(0, (n_db - qn) // HOP))
                qpcm.append(new_pcm[i, o:o + qn])
        qpcm = np.stack(qpcm)
        d_q = torch.from_numpy(qpcm).to("cuda")
        qdb, qoff = _oracle_q(oracle, qpcm)
        plan_off = np.arange(len(qpcm) + 1, dtype=np.int64) * qn
        for p in (p1, p45, tfp_lib.params(2, 0.001), tfp_lib.params(2, 0.1)):
            w, mc = oidx.search_batch(qdb[:, 0], qdb[:, 1], qoff, p.coefs, p.tolerance, nthreads=ORACLE_THREADS,
                                      method="boxes" if p.coefs == 2 else "scan")
            expk = np.where(w >= 0, (mc.astype(np.uint64) << np.uint64(32)) | rank[np.maximum(w, 0)].astype(np.uint64), 0)
            for e in (eng, full):
                keys = torch.zeros(len(qpcm), dtype=torch.int64, device="cuda")
                e.search_device(e.plan(plan_off), d_q.data_ptr(), p, keys.data_ptr(), stream)
                torch.cuda.synchronize()
                k = keys.cpu().numpy().view(np.uint64)
                assert np.array_equal(k, expk.astype(np.uint64)), (e is full, p.coefs, p.tolerance,
                                                                    np.nonzero(k != expk)[0][:8])
            if p is p45:  # the noise excerpts: the newest noise clip (greatest uuid), the victim never
                assert all(w[512 + j] == db_clips + 6 for j in range(28)) and victim not in set(w.tolist())
        assert full.index_build_stats()[1] == 0  # the reference engine never merged
    finally:
        full.close()
