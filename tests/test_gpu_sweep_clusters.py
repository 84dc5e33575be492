"""The coefs=2 sweep over clusters of points (csrc/tfp_scan.hip, CellCache::c_lo/c_hi/c_beg).

A group's points closer than dgap = floor(2 tol 1e6) - 3 micro-units (the least max2 window width
at the tolerance) merge into one cluster, and the sweep searches only a cluster's first and last
point. These cases put max2 points at gaps just below, at and above dgap, duplicates, and windows
placed inside every gap and on both ends of it, with q2 at several sub-micro offsets so the windows'
"%f" rounding takes both widths. Each clip has its own key (one query per clip reads that clip's
exact frame count back as match_count), and all clips also share one key, where the groups batch
per wave and one clip has > 64 clusters. Bar: == the oracle's fp_search_fingerprint_info
(src/fp_handler.c:308-374), in the default (clip-major, clusters) form, over points
(TFP_WIDE_POINTS), with 128-query chunks only (TFP_WIDE_CH128; by default batches of queries under 256 frames take 256-query chunks),
with the (key, frame) pair sort instead of the packed keys-only sort (TFP_WIDE_UNPACKED), and with the
library sort instead of the bin sort on the speculative pass (TFP_WIDE_LIBSORT).
"""
import math
import os
import uuid as uuidlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHARED_KEY = 30


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


def _points(dgap, base, kind):
    """Ascending max2 points (micro-units) of one clip's group."""
    if kind == "many":  # > 64 clusters: every gap wider than any window
        return [base + i * (2 * dgap + 40) for i in range(100)]
    gaps = [max(dgap - 1, 0), dgap, dgap + 1, dgap + 2, dgap + 3, 0, 2 * dgap + 9, 1, dgap + 4, max(dgap - 2, 0), dgap]
    if kind == "b":
        gaps = gaps[::-1] + [3 * dgap + 11]
    pts = [base]
    for g in gaps:
        pts.append(pts[-1] + g)
    return pts


def _frames_for(pts, tol, k):
    """Query frames of trunc key k whose max2 windows sit at every gap's inner ends and middle."""
    t = tol * 1e6
    xs = set()
    for a, b in zip(pts[:-1], pts[1:]):
        for v in (a, b):
            for d in range(-4, 5):
                xs.add(v + t + d)   # L2 around v
                xs.add(v - t + d)   # U2 around v
        mid = (a + b) // 2
        for d in range(-3, 4):
            xs.add(mid + d)
    xs.add(pts[0] - t - 50)
    xs.add(pts[-1] + t + 50)
    q2 = []
    for x in sorted(xs):
        for frac in (0.0, 0.25, 0.5, 0.7):
            q2.append((x + frac) / 1e6)
    return np.full(len(q2), k + 0.5), np.asarray(q2)


@pytest.mark.parametrize("tol", [0.0, 0.000004, 0.001, 0.0105, 0.1, 0.45])
def test_sweep_clusters_gap_boundaries(oracle, tfp_lib, tol):
    dgap = max(0, math.floor(2 * tol * 1e6) - 3)
    kinds = ["a", "b", "a", "many", "b"]
    rng = np.random.default_rng(7)
    uuids = [str(uuidlib.UUID(bytes=rng.bytes(16), version=4)) for _ in kinds]
    m1, m2, clip = [], [], []
    groups = []
    for c, kind in enumerate(kinds):
        own = 10 + c
        base = 5_000_000 + c * 37
        pts = _points(dgap, base, kind)
        shared_base = 10_000_000 + c * (200 * dgap + 10_000_000)
        spts = _points(dgap, shared_base, kind)
        for k, p in ((own, pts), (SHARED_KEY, spts)):
            m1 += [k * 1_000_000] * len(p)
            m2 += p
            clip += [c] * len(p)
        groups.append((own, pts, spts))
    m1 = np.asarray(m1, np.int32)
    m2 = np.asarray(m2, np.int32)
    clip = np.asarray(clip, np.int32)
    queries = []
    for c, (own, pts, spts) in enumerate(groups):
        queries.append(_frames_for(pts, tol, own))
        queries.append(_frames_for(spts, tol, SHARED_KEY))
    q1 = np.concatenate([q[0] for q in queries])
    q2 = np.concatenate([q[1] for q in queries])
    qoff = np.concatenate([[0], np.cumsum([len(q[0]) for q in queries])])
    assert qoff[-1] < 2**31 and max(len(q[0]) for q in queries) < 65536
    frames = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                         ("q1", "<f8"), ("q2", "<f8")]))
    frames["q1"], frames["q2"] = q1, q2
    expect = []
    for i in range(len(queries)):
        s = slice(qoff[i], qoff[i + 1])
        found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[s], q2[s], 2, tol, -1, -1)
        expect.append((uuids[w], mc) if found else None)
    got = {}
    for form, env in (("clusters", {"TFP_WIDE_MIN_TOL": "0"}), ("points", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_POINTS": "1"}),
                      ("clusters-128", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_CH128": "1"}),
                      ("unpacked", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_UNPACKED": "1"}),
                      ("libsort", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_LIBSORT": "1"})):
        eng = _engine_with(tfp_lib, env)
        try:
            for c in range(len(kinds)):
                sel = clip == c
                eng.index_add(uuids[c], m1[sel], m2[sel])
            res, fcs = eng.search_batch(frames, qoff, tfp_lib.params(2, tol))
            got[form] = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
            assert list(fcs) == list(np.diff(qoff))
        finally:
            eng.close()
    assert got["clusters"] == expect, tol
    assert got["points"] == expect, tol
    assert got["clusters-128"] == expect, tol
    assert got["unpacked"] == expect, tol
    assert got["libsort"] == expect, tol
    # every query found its own clip with a partial count: windows in the gaps missed, others hit
    for i, e in enumerate(expect):
        assert e is not None and e[0] == uuids[i // 2]
        assert 0 < e[1] < qoff[i + 1] - qoff[i]


@pytest.mark.parametrize("tol", [0.001, 0.05, 0.3])
def test_sweep_many_keys_per_chunk(oracle, tfp_lib, tol):
    """Chunks that use more than 64 keys (the clip-major sweep takes them 64 per step), frames
    with and without max2 windows (a 3400 Hz ignore filter drops max2 conditions), 300 queries (two
    256-query chunks with 8-bit counts, or three 128-query chunks with TFP_WIDE_CH128), a last clip
    window only partly filled, and NULL max2 rows: every form == the oracle. Then the same batch with
    one query of 300 frames (over 8-bit counts: 128-query chunks)."""
    rng = np.random.default_rng(int(tol * 1e4) + 5)
    nclips, rows = 70, 260
    uuids = [str(uuidlib.UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips)]
    keys = rng.integers(-5, 120, nclips * rows)
    m1 = (keys * 1_000_000 + rng.integers(-350_000, 350_000, nclips * rows)).astype(np.int32)
    m2 = rng.integers(0, 40_000_000, nclips * rows).astype(np.int32)
    m2[rng.random(nclips * rows) < 0.02] = np.iinfo(np.int32).min  # NULL max2 (never matches a max2 window)
    clip = np.repeat(np.arange(nclips), rows).astype(np.int32)
    nq = 300
    q1s, q2s, qoff = [], [], [0]
    for i in range(nq):
        c = int(rng.integers(nclips))
        n = int(rng.integers(20, 120))
        src = rng.integers(c * rows, (c + 1) * rows, n)
        q1 = m1[src] / 1e6 + rng.normal(0, 0.02, n)
        q2 = np.where(m2[src] == np.iinfo(np.int32).min, 20.0, m2[src] / 1e6) + rng.normal(0, 0.02, n)
        q1s.append(q1)
        q2s.append(q2)
        qoff.append(qoff[-1] + n)
    q1 = np.concatenate(q1s)
    q2 = np.concatenate(q2s)
    qoff = np.asarray(qoff, np.int64)
    frames = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                         ("q1", "<f8"), ("q2", "<f8")]))
    frames["q1"], frames["q2"] = q1, q2
    low, high = -1, 3400  # 10 log10(3400) = 35.3: frames with q2 above it keep only their max1 box
    expect = []
    for i in range(nq):
        s = slice(qoff[i], qoff[i + 1])
        found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[s], q2[s], 2, tol, low, high)
        expect.append((uuids[w], mc) if found else None)
    assert sum(e is not None for e in expect) > nq // 2
    for form, env in (("clusters", {"TFP_WIDE_MIN_TOL": "0"}), ("points", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_POINTS": "1"}),
                      ("clusters-128", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_CH128": "1"}),
                      ("unpacked", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_UNPACKED": "1"}),
                      ("libsort", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_LIBSORT": "1"})):
        eng = _engine_with(tfp_lib, env)
        try:
            for c in range(nclips):
                sel = clip == c
                eng.index_add(uuids[c], m1[sel], m2[sel])
            res, fcs = eng.search_batch(frames, qoff, tfp_lib.params(2, tol, low, high))
            got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
            assert got == expect, (form, tol, [i for i in range(nq) if got[i] != expect[i]][:5])
            assert list(fcs) == list(np.diff(qoff))
        finally:
            eng.close()
    # query 0 repeated to 300 frames: the batch no longer fits 8-bit counts
    n0 = qoff[1] - qoff[0]
    rep = np.arange(300) % n0
    lq1 = np.concatenate([q1[rep], q1[qoff[1]:]])
    lq2 = np.concatenate([q2[rep], q2[qoff[1]:]])
    lqoff = np.concatenate([[0], qoff[1:] - n0 + 300]).astype(np.int64)
    found, w, mc, fc = oracle.search(m1, m2, clip, uuids, lq1[:300], lq2[:300], 2, tol, low, high)
    lexp = [(uuids[w], mc) if found else None] + expect[1:]
    lframes = np.zeros(len(lq1), frames.dtype)
    lframes["q1"], lframes["q2"] = lq1, lq2
    eng = _engine_with(tfp_lib, {"TFP_WIDE_MIN_TOL": "0"})
    try:
        for c in range(nclips):
            sel = clip == c
            eng.index_add(uuids[c], m1[sel], m2[sel])
        res, fcs = eng.search_batch(lframes, lqoff, tfp_lib.params(2, tol, low, high))
        got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
        assert got == lexp, (tol, [i for i in range(nq) if got[i] != lexp[i]][:5])
        assert fcs[0] == 300
    finally:
        eng.close()


@pytest.mark.parametrize("tol", [0.001, 0.45])
def test_sweep_8bit_count_field_edge(oracle, tfp_lib, tol):
    """The 256-query sweep chunks pack four 8-bit counts per lane word when every query has fewer
    than 256 frames (tfp_scan.hip: wide_prefix / wide_clips_kernel<4>): a query's count per clip
    and its prefix counts never exceed its frame count. This fills one chunk exactly (256 queries of
    255 frames, the field's maximum) with queries whose every frame hits one clip X (match_count 255,
    the four queries of a lane word all at 255 together), queries whose frames hit nothing (count 0
    beside them), and queries at 254 for another clip Y. Keys == the oracle (src/fp_handler.c:318-374).
    The same batch with one more non-hitting frame per query (256 frames: over the 8-bit field, so
    128-query chunks with 16-bit counts) gives identical results."""
    rng = np.random.default_rng(255)
    uuids = [str(uuidlib.UUID(bytes=rng.bytes(16), version=4)) for _ in range(4)]
    # every row in trunc key 20's max1 box ([20 - tol, 20 + tol] contains 20.000000); clip c's
    # max2 points around 30 + 10 c dB, far apart at either tolerance
    rows = 300
    m1 = np.full(4 * rows, 20_000_000, np.int32)
    m2 = np.concatenate([30_000_000 + 10_000_000 * c + rng.integers(-20, 20, rows) * 5 for c in range(4)]).astype(np.int32)
    clip = np.repeat(np.arange(4), rows).astype(np.int32)
    X, Y = 1, 2
    vx, vy, vnone = 30.0 + 10 * X, 30.0 + 10 * Y, -100.0

    def batch(nframes):
        q2 = []
        for q in range(256):
            kind = q % 4 if q < 128 else (q // 4) % 4  # lane words of one kind, and of mixed kinds
            if kind in (0, 2):
                v = np.full(255, vx)        # all 255 frames hit X
            elif kind == 1:
                v = np.full(255, vnone)     # no frame hits anything
            else:
                v = np.full(255, vy)        # 254 hit Y, one misses
                v[q % 255] = vnone
            q2.append(np.concatenate([v, np.full(nframes - 255, vnone)]))
        q2 = np.concatenate(q2)
        q1 = np.full(len(q2), 20.5)
        qoff = np.arange(257, dtype=np.int64) * nframes
        frames = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                             ("q1", "<f8"), ("q2", "<f8")]))
        frames["q1"], frames["q2"] = q1, q2
        return frames, q1, q2, qoff

    frames, q1, q2, qoff = batch(255)
    expect = []
    for i in range(256):
        s = slice(qoff[i], qoff[i + 1])
        found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[s], q2[s], 2, tol, -1, -1)
        expect.append((uuids[w], mc) if found else None)
    assert sum(e == (uuids[X], 255) for e in expect) == 128
    assert sum(e == (uuids[Y], 254) for e in expect) == 64 and sum(e is None for e in expect) == 64
    eng = tfp_lib.Engine(0)
    try:
        for c in range(4):
            sel = clip == c
            eng.index_add(uuids[c], m1[sel], m2[sel])
        res, fcs = eng.search_batch(frames, qoff, tfp_lib.params(2, tol))
        got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
        assert got == expect, [i for i in range(256) if got[i] != expect[i]][:8]
        assert list(fcs) == [255] * 256
        frames2, _, _, qoff2 = batch(256)
        res2, fcs2 = eng.search_batch(frames2, qoff2, tfp_lib.params(2, tol))
        got2 = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res2]
        assert got2 == expect
        assert list(fcs2) == [256] * 256
    finally:
        eng.close()


@pytest.mark.parametrize("tol", [0.001, 0.1])
def test_bin_sort_bin_sizes(oracle, tfp_lib, tol):
    """The sweep's bin sort (tfp_scan.hip wide_bin_hist .. wide_bin_sort, which also fills the
    directories) on bins of every size class: 600 queries (three 256-query chunks, the last partly filled) whose max2 values mix a wide
    spread (bins of a few frames: the in-register sort), a 4 dB cluster (bins of hundreds: the LDS
    sort), repeated values (equal keys), frames whose max2 condition an ignore filter drops (their
    segment is not sorted), NULL values and keys over the ignore filter (not kept: the chunk's tail); then the same queries with a
    0.02 dB cluster (a bin above the per-wave cap: the batch goes to the library sort). Keys == the
    oracle (src/fp_handler.c:318-374) and == the library sort (TFP_WIDE_LIBSORT)."""
    rng = np.random.default_rng(int(tol * 1e4) + 11)
    nclips, rows = 40, 300
    uuids = [str(uuidlib.UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips)]
    keys = rng.integers(20, 26, nclips * rows)
    m1 = (keys * 1_000_000 + rng.integers(0, 999_999, nclips * rows)).astype(np.int32)
    m2 = np.where(rng.random(nclips * rows) < 0.5, rng.normal(40e6, 2e6, nclips * rows),
                  rng.uniform(-60e6, 30e6, nclips * rows)).astype(np.int32)
    clip = np.repeat(np.arange(nclips), rows).astype(np.int32)
    nq = 600

    def batch(cluster_db):
        q1s, q2s, qoff = [], [], [0]
        for i in range(nq):
            c = int(rng.integers(nclips))
            n = int(rng.integers(150, 250))
            src = rng.integers(c * rows, (c + 1) * rows, n)
            q1 = m1[src] / 1e6 + rng.normal(0, 0.01, n)
            u = rng.random(n)
            q2 = np.where(u < 0.4, 40.0 + rng.uniform(-cluster_db / 2, cluster_db / 2, n), m2[src] / 1e6 + rng.normal(0, 0.01, n))
            q2 = np.where((u > 0.9) & (u < 0.95), 12.5, q2)             # repeated values
            q2 = np.where(u >= 0.97, 36.0, q2)                           # over the 3400 ignore: max1 box only
            q1 = np.where((u > 0.95) & (u < 0.955), -np.inf, q1)         # NULL value: key 0 (ast_json_real_get)
            q1 = np.where((u >= 0.955) & (u < 0.96), 50.0, q1)           # key over the ignore: not kept
            q1s.append(q1)
            q2s.append(q2)
            qoff.append(qoff[-1] + n)
        q1 = np.concatenate(q1s)
        q2 = np.concatenate(q2s)
        frames = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                             ("q1", "<f8"), ("q2", "<f8")]))
        frames["q1"], frames["q2"] = q1, q2
        return frames, q1, q2, np.asarray(qoff, np.int64)

    low, high = -1, 3400
    redo_seen = []
    for cluster_db in (4.0, 0.02):
        frames, q1, q2, qoff = batch(cluster_db)
        expect = []
        for i in range(nq):
            s = slice(qoff[i], qoff[i + 1])
            found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[s], q2[s], 2, tol, low, high)
            expect.append((uuids[w], mc) if found else None)
        assert sum(e is not None for e in expect) > nq // 2
        for form, env in (("bins", {"TFP_WIDE_MIN_TOL": "0"}), ("libsort", {"TFP_WIDE_MIN_TOL": "0", "TFP_WIDE_LIBSORT": "1"})):
            eng = _engine_with(tfp_lib, env)
            try:
                for c in range(nclips):
                    sel = clip == c
                    eng.index_add(uuids[c], m1[sel], m2[sel])
                st0 = eng.sweep_stats()
                res, fcs = eng.search_batch(frames, qoff, tfp_lib.params(2, tol, low, high))
                got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
                assert got == expect, (form, cluster_db, tol, [i for i in range(nq) if got[i] != expect[i]][:5])
                # the sort path that ran (tfp_sweep_stats): a silent fallback to the library sort fails here
                st = {k: v - st0[k] for k, v in eng.sweep_stats().items()}
                if form == "libsort":
                    assert (st["bins"], st["library"], st["redone"]) == (0, 1, 0), st
                elif cluster_db == 4.0:
                    assert (st["bins"], st["library"], st["redone"]) == (1, 0, 0), st
                else:  # the 0.02 dB cluster: a bin of distinct values above the per-wave cap redoes the batch
                    # with the library sort; where the cluster's bins stay under the cap (or hold one value:
                    # copied as a crowd) the bin sort stands
                    assert (st["bins"], st["library"], st["redone"]) in ((0, 1, 1), (1, 0, 0)), st
                    redo_seen.append(st["redone"])
            finally:
                eng.close()


def test_bin_sort_overflow_redone_with_library_sort(oracle, tfp_lib):
    """A window segment whose frames crowd into one bin with distinct values (990 frames of one key
    within 0.001 dB of 40 dB, 10 spread over 100 dB: the segment's bins are cut over its whole L2
    range) overflows the bin sort's per-wave cap: the speculative pass is redone with the library
    sort (tfp_sweep_stats: one redo, one library batch, no bin batch) and the keys == the oracle's
    (src/fp_handler.c:318-374)."""
    rng = np.random.default_rng(77)
    nclips, rows = 30, 200
    uuids = [str(uuidlib.UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips)]
    m1 = (20_000_000 + rng.integers(-900, 900, nclips * rows)).astype(np.int32)
    m2 = np.where(rng.random(nclips * rows) < 0.7, 40_000_000 + rng.integers(0, 1000, nclips * rows),
                  rng.integers(-50_000_000, 50_000_000, nclips * rows)).astype(np.int32)
    clip = np.repeat(np.arange(nclips), rows).astype(np.int32)
    nq, per = 10, 100
    q1 = np.full(nq * per, 20.3)
    q2 = 40.0 + rng.permutation(nq * per).astype(np.float64) * 1e-6  # 1,000 distinct values within 0.001 dB
    spread = rng.choice(nq * per, 10, replace=False)
    q2[spread] = rng.uniform(-50, 50, 10)
    qoff = np.arange(nq + 1, dtype=np.int64) * per
    frames = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                         ("q1", "<f8"), ("q2", "<f8")]))
    frames["q1"], frames["q2"] = q1, q2
    expect = []
    for i in range(nq):
        s = slice(qoff[i], qoff[i + 1])
        found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[s], q2[s], 2, 0.001, -1, -1)
        expect.append((uuids[w], mc) if found else None)
    assert sum(e is not None for e in expect) >= nq // 2
    eng = _engine_with(tfp_lib, {"TFP_WIDE_MIN_TOL": "0"})
    try:
        for c in range(nclips):
            sel = clip == c
            eng.index_add(uuids[c], m1[sel], m2[sel])
        st0 = eng.sweep_stats()
        res, _ = eng.search_batch(frames, qoff, tfp_lib.params(2, 0.001))
        got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
        assert got == expect
        st = {k: v - st0[k] for k, v in eng.sweep_stats().items()}
        assert (st["bins"], st["library"], st["redone"]) == (0, 1, 1), st
    finally:
        eng.close()


@pytest.mark.parametrize("tol", [0.001, 0.3])
def test_bin_sort_crowd_groups_and_sparse_directory_runs(oracle, tfp_lib, tol):
    """The bin sort's crowded groups and its directory runs of every length (tfp_scan.hip
    wide_bin_sort, dir_write). In every chunk one window segment (key 25) holds a crowd of one value
    (a quarter of the frames at exactly 40 dB: copied unsorted) after small bins of distinct values
    just below it in the same sort group (sorted together, then the crowd); another segment (key 24)
    mixes a dense cluster, tight clumps 20-30 dB apart and a thin spread, so its directories have
    runs of 1-8 buckets, of 9-256 (written by their own lanes) and of hundreds to thousands (by the
    whole wave), from every alignment. Keys == the oracle (src/fp_handler.c:318-374); the batch took
    the bin sort (no redo) and copied crowd bins (tfp_sweep_stats)."""
    rng = np.random.default_rng(int(tol * 1e3) + 5)
    nclips, rows, extra = 48, 250, 40
    uuids = [str(uuidlib.UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips)]

    def sparse_db(n):  # key 24's max2 mixture (dB)
        u = rng.random(n)
        return np.where(u < 0.4, 10.0 + rng.normal(0, 0.5, n),  # (wide enough that no bin passes 512 distinct values)
               np.where(u < 0.6, -40.0 + rng.uniform(-1.0, 1.0, n),
               np.where(u < 0.62, rng.uniform(-20.0, 0.0, n), 35.0 + rng.uniform(-1.5, 1.5, n))))

    m1s, m2s, clips = [], [], []
    for c in range(nclips):
        k = rng.integers(20, 24, rows)
        m1s.append(k * 1_000_000 + rng.integers(-800, 800, rows))  # (a frame's max1 box is its truncated max1 +- tol)
        m2s.append(np.where(rng.random(rows) < 0.3, rng.normal(40e6, 2e6, rows), rng.uniform(-60e6, 40e6, rows)))
        # rows of the crowd's key (max2 spread over 39-41 dB) and of the sparse key
        m1s.append(np.full(extra, 25_000_000) + rng.integers(-400, 400, extra))
        m2s.append(rng.uniform(39e6, 41e6, extra))
        m1s.append(np.full(extra, 24_000_000) + rng.integers(-400, 400, extra))
        m2s.append(sparse_db(extra) * 1e6)
        clips.append(np.full(rows + 2 * extra, c))
    m1 = np.concatenate(m1s).astype(np.int32)
    m2 = np.concatenate(m2s).astype(np.int32)
    clip = np.concatenate(clips).astype(np.int32)
    nq = 520  # three 256-query chunks, the last partly filled
    q1s, q2s, qoff = [], [], [0]
    for i in range(nq):
        c = int(rng.integers(nclips))
        n = int(rng.integers(120, 200))
        src = rng.choice(np.flatnonzero(clip == c)[:rows], n)
        q1 = m1[src] / 1e6 + rng.normal(0, 0.0003, n)
        q2 = m2[src] / 1e6 + rng.normal(0, 0.0003, n)
        u = rng.random(n)
        crowd, near, sparse = u < 0.25, (u >= 0.25) & (u < 0.28), (u >= 0.28) & (u < 0.40)
        q1 = np.where(crowd | near, 25.3, np.where(sparse, 24.4, q1))
        # the crowd at exactly 40 dB; its neighbours at least 2 mdB away (outside the crowd's bin)
        side = np.where(rng.random(n) < 0.5, -1.0, 1.0)
        q2 = np.where(crowd, 40.0, np.where(near, 40.0 + side * rng.uniform(0.002, 0.15, n), q2))
        q2 = np.where(sparse, sparse_db(n), q2)
        q1s.append(q1)
        q2s.append(q2)
        qoff.append(qoff[-1] + n)
    q1 = np.concatenate(q1s)
    q2 = np.concatenate(q2s)
    qoff = np.asarray(qoff, np.int64)
    frames = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                         ("q1", "<f8"), ("q2", "<f8")]))
    frames["q1"], frames["q2"] = q1, q2
    expect = []
    for i in range(nq):
        s = slice(qoff[i], qoff[i + 1])
        found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[s], q2[s], 2, tol, -1, -1)
        expect.append((uuids[w], mc) if found else None)
    assert sum(e is not None for e in expect) > nq // 2
    eng = _engine_with(tfp_lib, {"TFP_WIDE_MIN_TOL": "0"})
    try:
        for c in range(nclips):
            sel = clip == c
            eng.index_add(uuids[c], m1[sel], m2[sel])
        st0 = eng.sweep_stats()
        res, _ = eng.search_batch(frames, qoff, tfp_lib.params(2, tol))
        got = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
        assert got == expect, (tol, [i for i in range(nq) if got[i] != expect[i]][:5])
        st = {k: v - st0[k] for k, v in eng.sweep_stats().items()}
        assert (st["bins"], st["library"], st["redone"]) == (1, 0, 0) and st["crowd"] >= 2, st
    finally:
        eng.close()
