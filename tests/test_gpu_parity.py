"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle and the SQL goldens.

Bar: bit-exact micro-units (the stored max1/max2 "hash set") and identical search results
(uuid, match_count, frame_count) — integer work, no tolerance.
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

SEED_DB, SEED_Q = 0x7153A1, 0x7153B2


def _engine_with(tfp_lib, env):
    """A fresh engine created with test knobs in the environment (the engine reads them once)."""
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


def _pcm_cases():
    rng = np.random.default_rng(11)
    cases = {
        "empty": np.zeros(0, np.int16),
        "one": np.array([1234], np.int16),
        "hop-1": rng.integers(-30000, 30000, 255).astype(np.int16),
        "hop": rng.integers(-30000, 30000, 256).astype(np.int16),
        "hop+1": rng.integers(-30000, 30000, 257).astype(np.int16),
        "silence": np.zeros(3000, np.int16),
        "fullscale": np.where(np.arange(5000) % 2 == 0, 32767, -32768).astype(np.int16),
        "dc": np.full(4097, -32768, np.int16),
        "noise": rng.integers(-32768, 32767, 20000).astype(np.int16),
        "tiny": rng.integers(-2, 3, 9000).astype(np.int16),
    }
    return cases


def _assert_frames_equal(fr, micro, db):
    assert len(fr) == len(micro)
    bad = (fr["m1"] != micro[:, 0]) | (fr["m2"] != micro[:, 1])
    if bad.any():
        i = np.nonzero(bad)[0]
        print("mismatching frames:", len(i), "of", len(fr), "first:", i[:10])
        print("gpu q1,q2:", fr["q1"][i[:5]], fr["q2"][i[:5]])
        print("cpu q1,q2:", db[i[:5], 0], db[i[:5], 1])
    assert np.array_equal(fr["m1"], micro[:, 0]), np.nonzero(fr["m1"] != micro[:, 0])
    assert np.array_equal(fr["m2"], micro[:, 1]), np.nonzero(fr["m2"] != micro[:, 1])
    # q: the frame values are glibc's 10*log10|c| bit for bit (tfp_math.hpp LogFix); a NaN is a
    # NaN whatever its payload (x86 and gfx950 make different default NaNs)
    for k, col in (("q1", 0), ("q2", 1)):
        a, b = fr[k], db[:, col]
        same = (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))
        assert same.all(), np.nonzero(~same)


@pytest.mark.parametrize("name", list(_pcm_cases().keys()))
def test_fingerprint_edge_cases_bit_exact(engine, oracle, name):
    pcm = _pcm_cases()[name]
    fr = engine.fingerprint(pcm)
    _, db, micro = oracle.fingerprint(pcm)
    _assert_frames_equal(fr, micro, db)
    assert np.array_equal(fr["frame_idx"], np.arange(len(fr)))


def test_fingerprint_synthetic_clips_bit_exact(engine, oracle, tfp_lib):
    pcm = tfp_lib.synth_pcm(SEED_DB, range(24), 80000)  # C1 shape: 10 s at 8 kHz
    flat = pcm.reshape(-1)
    off = np.arange(25) * 80000
    fr = engine.fingerprint_batch(flat, off)
    micro, db = oracle.fingerprint_batch(flat, off, nthreads=8)
    _assert_frames_equal(fr, micro, db)
    assert len(fr) == 24 * 313


def _sparse_cases(nclips=256, n=4096, seed=21):
    """Spectra with exact zeros and tiny cancellation residues in both halves of the bins: sparse
    +-1..3 impulses (near the window's tails too), impulse pairs half a window apart, integer
    tones on exact bins, short periods dividing 512, and isolated full-scale spikes."""
    rng = np.random.default_rng(seed)
    clips = []
    t = np.arange(n)
    for c in range(nclips):
        kind = c % 5
        x = np.zeros(n, np.int32)
        if kind == 0:
            pos = rng.choice(n, size=int(rng.integers(1, 24)), replace=False)
            x[pos] = rng.choice([-3, -2, -1, 1, 2, 3], size=len(pos))
        elif kind == 1:
            for _ in range(int(rng.integers(1, 8))):
                p = int(rng.integers(0, n - 256))
                v = int(rng.choice([-2, -1, 1, 2]))
                x[p] = v
                x[p + 256] = v if rng.random() < 0.5 else -v
        elif kind == 2:
            k = int(rng.integers(1, 256))
            a = float(rng.choice([1.0, 2.0, 3.0, 30000.0]))
            x = np.rint(a * np.cos(2 * np.pi * k * t / 512 + float(rng.random()) * 2 * np.pi)).astype(np.int32)
        elif kind == 3:
            per = int(rng.choice([2, 4, 8, 16, 32, 64, 128, 256, 512]))
            base = rng.integers(-3, 4, per)
            x = base[t % per].astype(np.int32)
        else:
            x[int(rng.integers(0, n))] = int(rng.choice([-32768, 32767]))
        clips.append(np.clip(x, -32768, 32767).astype(np.int16))
    return clips


def test_fingerprint_sparse_and_cancelling_spectra_bit_exact(engine, oracle):
    """The throughput launch and the small launch on spectra full of exact zeros and rounding
    residues (the rare-bin test and both elements of every conjugate pair)."""
    clips = _sparse_cases()
    flat = np.concatenate(clips)
    off = np.concatenate([[0], np.cumsum([len(c) for c in clips])]).astype(np.int64)
    fr = engine.fingerprint_batch(flat, off)
    micro, db = oracle.fingerprint_batch(flat, off, nthreads=8)
    _assert_frames_equal(fr, micro, db)
    for c in clips[:10]:
        fr1 = engine.fingerprint(c)
        _, db1, micro1 = oracle.fingerprint(c)
        _assert_frames_equal(fr1, micro1, db1)


def test_fingerprint_ragged_batch_equals_single(engine, tfp_lib):
    rng = np.random.default_rng(2)
    lens = [0, 17, 256, 511, 4096, 4097, 12345, 0, 80000]
    clips = [tfp_lib.synth_pcm(SEED_Q, [i], n)[0] if n else np.zeros(0, np.int16) for i, n in enumerate(lens)]
    off = np.concatenate([[0], np.cumsum(lens)])
    batch = engine.fingerprint_batch(np.concatenate(clips), off)
    single = np.concatenate([engine.fingerprint(c) for c in clips])
    assert np.array_equal(batch, single)
    rng.shuffle(clips)


def test_fingerprint_other_sample_rates(engine, oracle, tfp_lib):
    pcm = tfp_lib.synth_pcm(5, [0], 30000)[0]
    for sr in (16000, 44100):
        fr = engine.fingerprint(pcm, sr)
        _, db, micro = oracle.fingerprint(pcm, sr)
        _assert_frames_equal(fr, micro, db)


# ---------------------------------------------------------------------------------- search

def _load_golden():
    with open(os.path.join(REPO, "tests", "golden", "match_cases.json")) as f:
        return json.load(f)


def _frames_from_q(q1, q2):
    fr = np.zeros(len(q1), np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                     ("q1", "<f8"), ("q2", "<f8")]))
    fr["q1"] = [-math.inf if v is None else v for v in q1]
    fr["q2"] = [-math.inf if v is None else v for v in q2]
    return fr


def test_search_golden_sqlite(engine, tfp_lib):
    """Every SQLite-produced golden case, through tfp_index_add + tfp_search."""
    g = _load_golden()
    n = 0
    for s in g["scenarios"]:
        engine.index_clear()
        clip = np.asarray(s["clip"], np.int64)
        m1 = np.asarray(s["m1"], np.int64)
        m2 = np.asarray(s["m2"], np.int64)
        for c, u in enumerate(s["uuids"]):
            sel = clip == c
            engine.index_add(u, m1[sel].astype(np.int32), m2[sel].astype(np.int32))
        for q in s["queries"]:
            p = tfp_lib.params(q["coefs"], q["tol"], q["low"], q["high"])
            r, fc = engine.search(_frames_from_q(q["q1"], q["q2"]), p)
            got = None if r is None else {"audio_uuid": r["audio_uuid"], "match_count": r["match_count"],
                                          "frame_count": r["frame_count"]}
            assert got == q["expect"], (s["name"], q["coefs"], q["tol"], q["low"], q["high"])
            assert fc == q["frame_count"]
            n += 1
    engine.index_clear()
    assert n > 900


def _build_db(engine, oracle, tfp_lib, nclips, seconds, seed=SEED_DB):
    n = 8000 * seconds
    pcm = tfp_lib.synth_pcm(seed, range(nclips), n)
    off = np.arange(nclips + 1) * n
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), off, nthreads=8, want_db=False)
    nf = (n + 255) // 256
    rng = np.random.default_rng(seed)
    uuids = [str(__import__("uuid").UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips)]
    engine.index_clear()
    for c in range(nclips):
        engine.index_add(uuids[c], micro[c * nf:(c + 1) * nf, 0], micro[c * nf:(c + 1) * nf, 1])
    clip = np.repeat(np.arange(nclips), nf)
    return uuids, micro, clip


def _queries(tfp_lib, nq, db_clips, seconds_db, seconds_q, seed=SEED_Q):
    rng = np.random.default_rng(seed)
    specs_seed, clips, offs = [], [], []
    n = 8000 * seconds_q
    out = np.zeros((nq, n), np.int16)
    for i in range(nq):
        if i % 4 != 3:
            c = int(rng.integers(db_clips))
            o = 256 * int(rng.integers(0, (8000 * seconds_db - n) // 256))
            out[i] = tfp_lib.synth_pcm(SEED_DB, [c], n, offsets=[o])[0]
        else:
            out[i] = tfp_lib.synth_pcm(seed, [i], n)[0]
    return out


@pytest.mark.parametrize("coefs,tol,low,high", [
    (1, 0.001, -1, -1), (1, -1.0, -1, -1), (1, 0.01, -1, -1), (1, 0.1, 100, 3400), (1, 0.45, -1, -1),
    (2, 0.001, -1, -1), (2, 0.1, -1, -1), (2, 0.45, 100, 3400), (2, 1.0, -1, -1),
])
def test_search_pcm_vs_oracle(engine, oracle, tfp_lib, coefs, tol, low, high):
    uuids, micro, clip = _build_db(engine, oracle, tfp_lib, 120, 12)
    qpcm = _queries(tfp_lib, 24, 120, 12, 5)
    off = np.arange(25) * qpcm.shape[1]
    res, fcs = engine.search_pcm_batch(qpcm.reshape(-1), off, tfp_lib.params(coefs, tol, low, high))
    for i in range(24):
        _, qdb, _ = oracle.fingerprint(qpcm[i])
        found, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], clip, uuids, qdb[:, 0], qdb[:, 1],
                                         coefs, tol, low, high)
        exp = {"audio_uuid": uuids[w], "match_count": mc} if found else None
        got = None if res[i] is None else {"audio_uuid": res[i]["audio_uuid"], "match_count": res[i]["match_count"]}
        assert got == exp, (i, coefs, tol)
        assert fcs[i] == fc == 157


@pytest.mark.parametrize("path", ["sweep", "cells"])
@pytest.mark.parametrize("tol,low,high", [(0.001, -1, -1), (0.01, -1, -1), (0.1, 50, 60), (0.45, -1, -1)])
def test_general_paths_vs_oracle(oracle, tfp_lib, path, tol, low, high):
    """coefs=2 through the general path both ways (csrc/tfp_scan.hip): the sweep by groups (the
    default) and the clip-set cells (forced with TFP_WIDE_MIN_TOL, read at engine creation).
    150 queries = three 64-query chunks of the sweep, the last partial; the 50/60 Hz filter leaves
    frames whose max2 condition is dropped (they hit every clip of their key,
    src/fp_handler.c:324-337). == the oracle."""
    eng = _engine_with(tfp_lib, {"TFP_WIDE_MIN_TOL": "0" if path == "sweep" else "1e9"})
    try:
        uuids, micro, clip = _build_db(eng, oracle, tfp_lib, 120, 12)
        qpcm = _queries(tfp_lib, 150, 120, 12, 5)
        off = np.arange(151) * qpcm.shape[1]
        res, fcs = eng.search_pcm_batch(qpcm.reshape(-1), off, tfp_lib.params(2, tol, low, high))
        nfound = 0
        for i in range(150):
            _, qdb, _ = oracle.fingerprint(qpcm[i])
            found, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], clip, uuids, qdb[:, 0], qdb[:, 1],
                                             2, tol, low, high)
            exp = {"audio_uuid": uuids[w], "match_count": mc} if found else None
            got = None if res[i] is None else {"audio_uuid": res[i]["audio_uuid"], "match_count": res[i]["match_count"]}
            assert got == exp, (i, tol)
            assert fcs[i] == fc
            nfound += found
        assert nfound > 0
    finally:
        eng.close()


@pytest.mark.parametrize("path", ["sweep", "cells"])
def test_search_scan_fallback_many_frames_one_key(oracle, tfp_lib, path):
    """> 2048 frames with the same key exceed fp16-exact counts: the general path must take over
    (both of its forms: the sweep by groups, the clip-set cells)."""
    engine = _engine_with(tfp_lib, {"TFP_WIDE_MIN_TOL": "0" if path == "sweep" else "1e9"})
    try:
        _fallback_case(engine, oracle, tfp_lib)
    finally:
        engine.close()


def _fallback_case(engine, oracle, tfp_lib):
    uuids, micro, clip = _build_db(engine, oracle, tfp_lib, 40, 6)
    q = np.zeros(2100 * 256, np.int16)  # silence: every frame has the same trunc key
    res, fcs = engine.search_pcm_batch(q, [0, len(q)], tfp_lib.params(1, 0.45))
    _, qdb, _ = oracle.fingerprint(q)
    found, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], clip, uuids, qdb[:, 0], qdb[:, 1], 1, 0.45, -1, -1)
    got = None if res[0] is None else (res[0]["audio_uuid"], res[0]["match_count"])
    assert got == ((uuids[w], mc) if found else None)
    assert fcs[0] == 2100


def test_index_remove_and_readd(engine, oracle, tfp_lib):
    uuids, micro, clip = _build_db(engine, oracle, tfp_lib, 30, 6)
    qpcm = _queries(tfp_lib, 8, 30, 6, 3)
    off = np.arange(9) * qpcm.shape[1]
    p = tfp_lib.params(1, 0.1)
    res, _ = engine.search_pcm_batch(qpcm.reshape(-1), off, p)
    winners = {r["audio_uuid"] for r in res if r}
    assert winners
    for u in winners:
        engine.index_remove(u)
    keep = np.array([u not in winners for u in uuids])
    res2, _ = engine.search_pcm_batch(qpcm.reshape(-1), off, p)
    sel = keep[clip]
    for i in range(8):
        _, qdb, _ = oracle.fingerprint(qpcm[i])
        found, w, mc, _ = oracle.search(micro[sel, 0], micro[sel, 1], clip[sel],
                                        uuids, qdb[:, 0], qdb[:, 1], 1, 0.1, -1, -1)
        got = None if res2[i] is None else (res2[i]["audio_uuid"], res2[i]["match_count"])
        assert got == ((uuids[w], mc) if found else None)
    with pytest.raises(tfp_lib.TfpError):
        engine.index_remove(next(iter(winners)))
    with pytest.raises(tfp_lib.TfpError):
        engine.index_add(uuids[0] if uuids[0] not in winners else uuids[1], [1], [1])


def test_search_bad_coefs_is_notfound(engine, tfp_lib):
    fr = _frames_from_q([24.3], [1.0])
    for c in (0, 3, -1):
        r, fc = engine.search(fr, tfp_lib.params(c, 0.001))
        assert r is None and fc == 1


def test_fp_handler_mirror_end_to_end(tmp_path, oracle, tfp_lib):
    """The reference's create/search flow (app_tiresias enrolment + dialplan search)."""
    from tiresias_amd.fp_handler import FpHandler, write_wav_mono16
    fp = FpHandler(0)
    assert fp.fp_init()
    pcm = tfp_lib.synth_pcm(SEED_DB, range(12), 8000 * 8)
    files = []
    for i in range(12):
        f = str(tmp_path / f"clip{i}.wav")
        write_wav_mono16(f, pcm[i])
        files.append(f)
        assert fp.fp_craete_audio_list_info("ctx%d" % (i % 2), f)
    assert fp.fp_craete_audio_list_info("ctx0", files[0])  # already enrolled -> true
    assert len(fp.fp_get_audio_lists_all()) == 12
    q = str(tmp_path / "q.wav")
    write_wav_mono16(q, pcm[5][256 * 40: 256 * 40 + 24000])
    res = fp.fp_search_fingerprint_info("ctx1", q, 1, 0.45, -1, -1)
    # expected through the oracle chain
    rows = [oracle.fingerprint(pcm[i])[2] for i in range(12)]
    uu = {r["name"]: r["uuid"] for r in fp.fp_get_audio_lists_all()}
    uuids = [uu["clip%d.wav" % i] for i in range(12)]
    micro = np.concatenate(rows)
    clip = np.repeat(np.arange(12), len(rows[0]))
    _, qdb, _ = oracle.fingerprint(pcm[5][256 * 40: 256 * 40 + 24000])
    found, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], clip, uuids, qdb[:, 0], qdb[:, 1], 1, 0.45, -1, -1)
    if found:
        assert res["uuid"] == uuids[w] and res["match_count"] == mc and res["frame_count"] == fc == 94
        assert res["name"] == "clip%d.wav" % w and res["context"] == "ctx%d" % (w % 2)
        assert fp.fp_delete_audio_list_info(res["uuid"])
    else:
        assert res is None
    assert fp.fp_search_fingerprint_info("ctx1", q, 3, 0.45, -1, -1) is None
    assert fp.fp_search_fingerprint_info("ctx1", str(tmp_path / "missing.wav"), 1, 0.45, -1, -1) is None
    assert fp.fp_term()


@pytest.mark.parametrize("knob", [("TFP_GENERIC", "1"), ("TFP_RARE_THR_LOG2", "100")])
def test_fingerprint_kernel_variants_bit_exact(engine, oracle, tfp_lib, knob):
    """The 8 kHz kernel's other paths against the oracle: the generic kernel (TFP_GENERIC=1), and
    the real split's spec-order slow path taken by every non-zero bin (TFP_RARE_THR_LOG2=100;
    in production only bins with 0 < |S|^2 < 2^-98 take it)."""
    pcm = tfp_lib.synth_pcm(SEED_DB, range(6), 80000)
    flat = np.concatenate([pcm.reshape(-1)] + list(_pcm_cases().values()))
    lens = [80000] * 6 + [len(v) for v in _pcm_cases().values()]
    off = np.concatenate([[0], np.cumsum(lens)])
    micro, db = oracle.fingerprint_batch(flat, off, nthreads=8)
    eng = _engine_with(tfp_lib, {knob[0]: knob[1]})  # knobs are read once, at engine creation
    try:
        fr = eng.fingerprint_batch(flat, off)
    finally:
        eng.close()
    _assert_frames_equal(fr, micro, db)


@pytest.mark.parametrize("tol,low,high", [(0.001, -1, -1), (0.1, 100, 3400), (0.45, -1, -1), (-1.0, 300, -1)])
def test_search_small_batches_equal_general(engine, oracle, tfp_lib, tol, low, high):
    """Batches of <= 8 queries take the small-batch kernels (tfp_kernels.hpp, kSmallQ); a batch of
    24 takes the vote GEMM. Both must give the same (uuid, match_count, frame_count)."""
    _build_db(engine, oracle, tfp_lib, 120, 12)
    qpcm = _queries(tfp_lib, 24, 120, 12, 5)
    n = qpcm.shape[1]
    p = tfp_lib.params(1, tol, low, high)
    big, fb = engine.search_pcm_batch(qpcm.reshape(-1), np.arange(25) * n, p)
    small, fs = [], []
    for lo, hi in ((0, 1), (1, 4), (4, 12), (12, 13), (13, 21), (21, 24)):
        r, f = engine.search_pcm_batch(qpcm[lo:hi].reshape(-1), np.arange(hi - lo + 1) * n, p)
        small += r
        fs += list(f)
    key = lambda r: None if r is None else (r["audio_uuid"], r["match_count"])  # noqa: E731
    assert [key(r) for r in small] == [key(r) for r in big]
    assert list(fs) == list(fb)
    if low < 0 and high < 0:
        assert any(r is not None for r in big)


def test_search_small_out_of_range_key_falls_back(engine, tfp_lib):
    """A query key outside the vote range (|k| > 511, impossible for real fingerprints) sends a
    small batch to the general scan path, as key_hist does for large batches."""
    engine.index_clear()
    engine.index_add("00000000-0000-4000-8000-000000000001", np.array([1000000000, 24000000], np.int32),
                     np.array([0, 0], np.int32))
    engine.index_add("00000000-0000-4000-8000-000000000002", np.array([24000100], np.int32), np.array([0], np.int32))
    r, fc = engine.search(_frames_from_q([1000.0005, 24.2], [0.0, 0.0]), tfp_lib.params(1, 0.001))
    assert r is not None and r["audio_uuid"].endswith("001") and r["match_count"] == 2 and fc == 2
    engine.index_clear()


def test_speculative_sweep_redone_for_out_of_range_key(engine, oracle, tfp_lib):
    """coefs = 2 batches take the sweep without a host wait for its sort's counts (the sweep runs on
    the speculation that every frame's key lies in the clip-set cache and every max2 window fits the
    one-sort key); the counts come back with the results. A batch with a key outside the cache
    (|k| > 511) must then be redone on the row scan: its results == the oracle's, and == a batch
    without that query."""
    engine.index_clear()
    rng = np.random.default_rng(4)
    m1s, m2s, clip, uu = [], [], [], []
    for c in range(40):
        n = 30
        m1 = (rng.integers(22, 26, n) * 1000000 + rng.integers(-300000, 300000, n)).astype(np.int32)
        m2 = rng.integers(-3000000, 3000000, n).astype(np.int32)
        if c == 7:
            m1[:3] = 1000000000 + np.arange(3)  # rows at 1000 dB
        u = "00000000-0000-4000-8000-%012d" % c
        engine.index_add(u, m1, m2)
        m1s.append(m1), m2s.append(m2), clip.append(np.full(n, c, np.int32)), uu.append(u)
    m1, m2, cl = np.concatenate(m1s), np.concatenate(m2s), np.concatenate(clip)
    qs = []
    for i in range(6):
        q1 = rng.uniform(21.5, 26.5, 50)
        q2 = rng.uniform(-3.2, 3.2, 50)
        if i == 2:
            q1[:2] = 1000.0005  # key 1000: outside the cache, only the row scan can serve it
            q2[:2] = m2s[7][0] / 1e6
        qs.append((q1, q2))
    fr = _frames_from_q(np.concatenate([q[0] for q in qs]), np.concatenate([q[1] for q in qs]))
    qoff = np.arange(7) * 50
    for tol in (0.3, 0.05):
        p = tfp_lib.params(2, tol)
        res, fcs = engine.search_batch(fr, qoff, p)
        for i, (q1, q2) in enumerate(qs):
            found, w, mc, fc = oracle.search(m1, m2, cl, uu, q1, q2, 2, tol, -1, -1)
            got = None if res[i] is None else (res[i]["audio_uuid"], res[i]["match_count"])
            assert got == ((uu[w], mc) if found else None), (tol, i)
        keep = [0, 1, 3, 4, 5]
        fr2 = _frames_from_q(np.concatenate([qs[i][0] for i in keep]), np.concatenate([qs[i][1] for i in keep]))
        res2, _ = engine.search_batch(fr2, np.arange(6) * 50, p)
        assert [res[i] for i in keep] == list(res2)
    engine.index_clear()


def _many_key_index(engine, nclips, spread, seed):
    """Rows whose max1 sit within +-0.002 of integers in [-spread, spread] (half inside the
    tol=0.001 boxes), so queries with keys over that range use up to 2*spread+1 vote keys."""
    rng = np.random.default_rng(seed)
    uuids = sorted(str(__import__("uuid").UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips))
    rng.shuffle(uuids)
    m1s, m2s, clip = [], [], []
    engine.index_clear()
    for c in range(nclips):
        n = int(rng.integers(5, 60))
        k = rng.integers(-spread, spread + 1, n)
        m1 = (k * 1000000 + rng.integers(-2000, 2001, n)).astype(np.int32)
        m2 = rng.integers(-5000000, 5000000, n).astype(np.int32)
        engine.index_add(uuids[c], m1, m2)
        m1s.append(m1), m2s.append(m2), clip.append(np.full(n, c, np.int32))
    return uuids, np.concatenate(m1s), np.concatenate(m2s), np.concatenate(clip)


@pytest.mark.parametrize("spread", [1, 4, 40, 300])
@pytest.mark.parametrize("class_max", ["-1", "10"])
def test_vote_paths_vs_oracle(engine, oracle, tfp_lib, spread, class_max):
    """The coefs=1 vote: the pattern-class path (few used keys, Ku <= 10), the GEMM with A in
    registers (Kp <= 128) and the streamed GEMM (larger Kp). TFP_VOTE_CLASS_MAX=-1 forces the
    GEMM for every batch. Same (uuid, match_count) as the oracle's per-query search."""
    eng = _engine_with(tfp_lib, {"TFP_VOTE_CLASS_MAX": class_max})  # read once, at engine creation
    uuids, m1, m2, clip = _many_key_index(eng, 700, spread, 17 + spread)
    rng = np.random.default_rng(spread)
    nq, lens = 40, rng.integers(1, 120, 40)
    qoff = np.concatenate([[0], np.cumsum(lens)])
    k = rng.integers(-spread, spread + 1, qoff[-1])
    q1 = k + rng.choice([0.2, 0.7, -0.3], qoff[-1]) * np.sign(k + 0.5)  # trunc(q1) == k
    q2 = np.zeros(qoff[-1])
    try:
        res, fcs = eng.search_batch(_frames_from_q(q1, q2), qoff, tfp_lib.params(1, 0.001))
    finally:
        eng.close()
    nfound = 0
    for i in range(nq):
        a, b = qoff[i], qoff[i + 1]
        found, w, mc, fc = oracle.search(m1, m2, clip, uuids, q1[a:b], q2[a:b], 1, 0.001, -1, -1)
        exp = (uuids[w], mc) if found else None
        got = None if res[i] is None else (res[i]["audio_uuid"], res[i]["match_count"])
        assert got == exp, (i, spread, class_max)
        assert fcs[i] == fc == b - a
        nfound += found
    assert nfound > nq // 2
    engine.index_clear()


# ---- fp32-sample path (tfp_fingerprint_f32_batch / tfp_search_f32_batch) ------------------
def _f32_cases(tfp_lib):
    """aubio hop values that are not int16 steps: stereo / 3-channel means of synthetic clips (as
    tfp_wav_decode_f32 computes them), 24-bit-like fine values, and edge lengths."""
    import oracle_py
    rng = np.random.default_rng(21)
    a = tfp_lib.synth_pcm(SEED_DB, [1, 2, 3], 30000)
    cases = {
        "stereo": oracle_py.wav_mono_f32(a[:2].T, 16),
        "3ch": oracle_py.wav_mono_f32(a.T, 16),
        "24bit": oracle_py.wav_mono_f32(rng.integers(-(1 << 23), 1 << 23, (20000, 2)), 24),
        "float": (rng.standard_normal(7000) * 0.2).astype(np.float32),
        "tiny": (rng.standard_normal(3000) * 1e-7).astype(np.float32),
    }
    for n in (0, 1, 255, 256, 257):
        cases["len%d" % n] = (rng.standard_normal(n) * 0.5).astype(np.float32)
    return cases


@pytest.mark.parametrize("sr", [8000, 16000])
def test_fingerprint_f32_bit_exact(engine, oracle, tfp_lib, sr):
    cases = _f32_cases(tfp_lib)
    xs = list(cases.values())
    off = np.concatenate([[0], np.cumsum([len(x) for x in xs])]).astype(np.int64)
    fr = engine.fingerprint_f32_batch(np.concatenate(xs), off, sr)
    want = [oracle.fingerprint_f32(x, sr) for x in xs]
    micro = np.concatenate([w[2] for w in want]) if len(fr) else np.zeros((0, 2), np.int32)
    db = np.concatenate([w[1] for w in want]) if len(fr) else np.zeros((0, 2))
    _assert_frames_equal(fr, micro, db)
    single = engine.fingerprint_f32_batch(cases["stereo"], [0, len(cases["stereo"])], sr)
    assert np.array_equal(single["m1"], fr["m1"][:len(single)])


def test_fingerprint_f32_nonfinite_and_huge_bit_exact(engine, oracle, tfp_lib):
    """fp32 samples that overflow the FFT (|x| near FLT_MAX) or are inf / NaN (a float WAV may hold
    them): aubio's dense filterbank turns a non-finite bin into NaN in every band (0 * inf), and
    fvec_log10 passes NaN / inf through; the kernel redoes such frames densely. Stored rows and
    NULLs equal the dense oracle's."""
    rng = np.random.default_rng(21)
    t = np.arange(8000 * 2, dtype=np.float64)
    base = (0.3 * np.sin(2 * np.pi * 700 * t / 8000)).astype(np.float32)
    cases = []
    x = (base * np.float32(3e38)).astype(np.float32)  # FFT sums overflow to inf, inf - inf = NaN
    cases.append(x)
    x = (base * np.float32(1e37)).astype(np.float32)  # |X| finite, band sums may overflow
    cases.append(x)
    x = base.copy(); x[5000] = np.nan; cases.append(x)
    x = base.copy(); x[9000] = np.inf; cases.append(x)
    x = base.copy(); x[1234] = -np.inf; x[1235] = np.inf; cases.append(x)
    x = base.copy(); x[rng.integers(0, len(x), 20)] = np.float32(3.0e38); cases.append(x)
    cases.append(base.copy())  # a finite clip in the same launch
    off = np.concatenate([[0], np.cumsum([len(c) for c in cases])]).astype(np.int64)
    fr = engine.fingerprint_f32_batch(np.concatenate(cases), off)
    want = [oracle.fingerprint_f32(c) for c in cases]
    micro = np.concatenate([w[2] for w in want])
    db = np.concatenate([w[1] for w in want])
    assert (micro == oracle.NULL_MICRO).any()  # the cases do reach the NULL rule
    _assert_frames_equal(fr, micro, db)


def test_f32_path_equals_int16_path(engine, tfp_lib):
    """x = s / 32768 through the fp32 kernel gives the int16 path's frames (aubio's value is the
    same real number; the window scaling by 2^-15 is exact)."""
    pcm = tfp_lib.synth_pcm(SEED_Q, [4, 5], 24000).reshape(-1)
    off = np.array([0, 24000, 48000], np.int64)
    a = engine.fingerprint_batch(pcm, off)
    b = engine.fingerprint_f32_batch(pcm.astype(np.float32) / np.float32(32768), off)
    assert np.array_equal(a["m1"], b["m1"]) and np.array_equal(a["m2"], b["m2"])
    assert np.array_equal(a["q1"], b["q1"]) and np.array_equal(a["q2"], b["q2"])


def test_search_f32_equals_frame_search(engine, oracle, tfp_lib):
    """search_f32_batch == tfp_search_batch on the fp32 path's own frames (whose search is the
    SQL-golden-pinned path), for stereo-mean queries of enrolled clips."""
    _build_db(engine, oracle, tfp_lib, 60, 12)
    import oracle_py
    q = tfp_lib.synth_pcm(SEED_DB, [7, 9, 11, 13], 40000, offsets=[2560, 0, 5120, 256])
    xs = [oracle_py.wav_mono_f32(np.stack([q[i], q[(i + 1) % 4]], 1), 16) for i in range(4)]
    xs.append(oracle_py.wav_mono_f32(np.stack([q[0], q[0]], 1), 16))  # identical channels: == int16 path
    off = np.concatenate([[0], np.cumsum([len(x) for x in xs])]).astype(np.int64)
    for p in (tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.45), tfp_lib.params(2, 0.5)):
        got, fc = engine.search_f32_batch(np.concatenate(xs), off, p)
        fr = engine.fingerprint_f32_batch(np.concatenate(xs), off)
        qoff = np.concatenate([[0], np.cumsum([(len(x) + 255) // 256 for x in xs])]).astype(np.int64)
        want, fw = engine.search_batch(fr, qoff, p)
        assert got == want and list(fc) == list(fw)
    r16, _ = engine.search_pcm_batch(q[0], [0, 40000], tfp_lib.params(1, 0.001))
    r32, _ = engine.search_f32_batch(xs[4], [0, 40000], tfp_lib.params(1, 0.001))
    assert r32 == r16


def test_small_path_epoch_wrap(engine, oracle, tfp_lib):
    """The small path stamps clips with a per-call epoch byte and clears only the rows stamped
    since the last clear when the epoch wraps (every 255 calls): 600 calls (two wraps) over
    queries with different used-key counts give the first calls' results, and so does a call
    after the index (hence the stamp row stride) changes."""
    _build_db(engine, oracle, tfp_lib, 80, 12)
    qpcm = _queries(tfp_lib, 12, 80, 12, 5)
    n = qpcm.shape[1]
    ps = [tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.45), tfp_lib.params(1, 2.0)]
    want = {}
    for i in range(12):
        for j, p in enumerate(ps):
            r, _ = engine.search_pcm_batch(qpcm[i], [0, n], p)
            want[i, j] = r[0]
    for call in range(600):
        i, j = call % 12, (call // 12) % 3
        r, _ = engine.search_pcm_batch(qpcm[i], [0, n], ps[j])
        assert r[0] == want[i, j], (call, i, j)
    engine.index_add("ffffffff-0000-4000-8000-000000000000", np.array([1, 2], np.int32), np.array([3, 4], np.int32))
    for i in range(12):
        r, _ = engine.search_pcm_batch(qpcm[i], [0, n], ps[1])
        big, _ = engine.search_pcm_batch(np.tile(qpcm[i], 9), np.arange(10) * n, ps[1])  # general path
        assert r[0] == big[0]
