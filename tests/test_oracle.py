"""The CPU oracle pinned against the reference's own SQL (golden fixtures) and against an
independent float64 DSP restatement."""
import json
import math
import os

import numpy as np
import pytest

from conftest import REPO

GOLDEN = os.path.join(REPO, "tests", "golden", "match_cases.json")


def load_golden():
    with open(GOLDEN) as f:
        return json.load(f)


def _q(vals):
    return [math.inf if v is None else v for v in vals]


def test_oracle_search_matches_sqlite_golden(oracle):
    g = load_golden()
    n = 0
    for s in g["scenarios"]:
        for q in s["queries"]:
            found, w, mc, fc = oracle.search(s["m1"], s["m2"], s["clip"], s["uuids"], _q(q["q1"]), _q(q["q2"]),
                                             q["coefs"], q["tol"], q["low"], q["high"])
            got = {"audio_uuid": s["uuids"][w], "match_count": mc, "frame_count": fc} if found else None
            assert got == q["expect"], (s["name"], q["coefs"], q["tol"], q["low"], q["high"])
            n += 1
    assert n > 900


def test_golden_regenerates_identically(tmp_path):
    """The committed fixtures are exactly what the reference SQL produces under SQLite now."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import make_golden
    import numpy as np_
    rng = np_.random.default_rng(make_golden.SEED)
    first = make_golden.make_scenario(rng, "rand_00", int(rng.integers(1, 30)), 60, 0.2, 40, prefix_share=True)
    committed = load_golden()["scenarios"][0]
    assert first["uuids"] == committed["uuids"]
    for a, b in zip(first["queries"], committed["queries"]):
        assert a["expect"] == b["expect"]


def test_sql_tiebreak_is_greatest_uuid():
    g = load_golden()
    tie = [s for s in g["scenarios"] if s["name"] == "tie_2000"][0]
    assert tie["queries"][0]["expect"]["audio_uuid"] == max(tie["uuids"])
    assert tie["queries"][0]["expect"]["match_count"] == 1


def test_fmt6_matches_printf(oracle):
    for x in [0.0, -0.0, 1e-7, -4e-7, 5e-7, 0.0078125, -0.0078125, 23.999, 24.001, 1.5e-6, 2.5e-6, 458.6, -458.6]:
        s = "%f" % x
        neg = s.startswith("-")
        ip, fp = s.lstrip("-").split(".")
        v = int(ip) * 1000000 + int(fp)
        assert oracle.fmt6(x) == (-v if neg else v), x


def test_mel_filterbank_shape(oracle):
    t = oracle.table_arrays(8000)
    mel = t["mel"]
    assert int((mel != 0).sum()) == 490
    assert (mel[34:] == 0).all() and (mel[:34] != 0).any(axis=1).all()
    assert np.all(mel >= 0)


def test_oracle_dsp_vs_float64(oracle):
    import dsp_f64
    rng = np.random.default_rng(3)
    t = np.arange(8000 * 4)
    pcm = (6000 * np.sin(2 * np.pi * 440 * t / 8000) + 2500 * np.sin(2 * np.pi * 1234.5 * t / 8000)
           + rng.normal(0, 800, len(t))).astype(np.int16)
    coef, db, micro = oracle.fingerprint(pcm)
    ref = dsp_f64.fingerprint_f64(pcm, oracle.table_arrays())
    # float32 pipeline vs float64: c0 ~ -50, relative agreement ~1e-5
    np.testing.assert_allclose(coef[:, 0], ref[:, 0], rtol=3e-5, atol=2e-3)
    np.testing.assert_allclose(coef[:, 1], ref[:, 1], rtol=3e-5, atol=2e-3)
    assert coef.shape == (125, 2)


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 512, 1000])
def test_oracle_frame_count_and_null_rule(oracle, n):
    pcm = np.zeros(n, np.int16)
    coef, db, micro = oracle.fingerprint(pcm)
    assert len(micro) == (n + 255) // 256
    # silence: every band clamps to 2e-42 -> c0 = constant, c1 = rounding residue of the DCT
    if n:
        assert np.all(micro[:, 0] == micro[0, 0])
        assert np.all(np.isfinite(db))


def test_oracle_batch_equals_single(oracle):
    rng = np.random.default_rng(5)
    lens = [0, 100, 256, 3000, 4097]
    clips = [rng.integers(-20000, 20000, n).astype(np.int16) for n in lens]
    pcm = np.concatenate(clips)
    off = np.concatenate([[0], np.cumsum(lens)])
    micro, db = oracle.fingerprint_batch(pcm, off, nthreads=3)
    single = np.concatenate([oracle.fingerprint(c)[2] for c in clips])
    assert np.array_equal(micro, single)


@pytest.mark.parametrize("method,mode", [("scan", 0), ("boxes", 0), ("boxes", 1), ("boxes", 2)])
def test_sorted_index_search_matches_sqlite_golden(oracle, method, mode):
    """The sorted-index batch searches (large tables) give the SQLite-pinned results too: every
    golden scenario, every query, ties by uuid rank; the per-box form in both of its forms."""
    g = load_golden()
    n = 0
    for s in g["scenarios"]:
        if not s["uuids"]:
            continue
        order = sorted(range(len(s["uuids"])), key=lambda c: s["uuids"][c])
        rank = np.empty(len(order), np.int32)
        rank[order] = np.arange(len(order))
        idx = oracle.SortedIndex(s["m1"], s["m2"], s["clip"], rank)
        assert np.all(np.diff(idx.m1.astype(np.int64)) >= 0)
        groups = {}
        for q in s["queries"]:  # one batch per parameter set
            groups.setdefault((q["coefs"], q["tol"], q["low"], q["high"]), []).append(q)
        for (coefs, tol, low, high), qs in groups.items():
            q1 = np.concatenate([_q(q["q1"]) for q in qs]) if qs else np.zeros(0)
            q2 = np.concatenate([_q(q["q2"]) for q in qs])
            qoff = np.concatenate([[0], np.cumsum([len(q["q1"]) for q in qs])])
            w, mc = idx.search_batch(q1, q2, qoff, coefs, tol if tol is not None else float("nan"), low, high, nthreads=3,
                                     method=method, mode=mode)
            for i, q in enumerate(qs):
                got = {"audio_uuid": s["uuids"][w[i]], "match_count": int(mc[i]), "frame_count": len(q["q1"])} \
                    if w[i] >= 0 else None
                assert got == q["expect"], (s["name"], coefs, tol, low, high)
                n += 1
    assert n > 900


@pytest.mark.parametrize("method,mode", [("scan", 0), ("boxes", 0), ("boxes", 1), ("boxes", 2)])
def test_sorted_index_search_equals_linear_scan(oracle, method, mode):
    """Random tables with NULL rows, coefs 1 and 2, ignore filters: sorted searches == row scan."""
    rng = np.random.default_rng(17)
    nclips, nrows = 300, 40000
    m1 = rng.integers(-5_000_000, 5_000_000, nrows).astype(np.int32)
    m1[rng.random(nrows) < 0.05] = oracle.NULL_MICRO
    m2 = rng.integers(-3_000_000, 3_000_000, nrows).astype(np.int32)
    m2[rng.random(nrows) < 0.05] = oracle.NULL_MICRO
    clip = rng.integers(0, nclips, nrows).astype(np.int32)
    uuids = ["%08x-0000-4000-8000-%012x" % (int(rng.integers(1 << 30)), c) for c in range(nclips)]
    order = sorted(range(nclips), key=lambda c: uuids[c])
    rank = np.empty(nclips, np.int32)
    rank[order] = np.arange(nclips)
    idx = oracle.SortedIndex(m1, m2, clip, rank)
    nq = 24
    lens = rng.integers(0, 40, nq)
    qoff = np.concatenate([[0], np.cumsum(lens)])
    q1 = rng.uniform(-5.5, 5.5, qoff[-1])
    q2 = rng.uniform(-3.5, 3.5, qoff[-1])
    q1[rng.random(len(q1)) < 0.05] = np.inf
    for coefs, tol, low, high in [(1, 0.001, -1, -1), (1, 0.4, -1, -1), (2, 0.3, -1, -1), (2, 0.05, 1, 3),
                                  (1, -1.0, 1, -1), (3, 0.1, -1, -1)]:
        w, mc = idx.search_batch(q1, q2, qoff, coefs, tol, low, high, nthreads=4, method=method, mode=mode)
        for i in range(nq):
            a, b = qoff[i], qoff[i + 1]
            found, ww, mm, _ = oracle.search(m1, m2, clip, uuids, q1[a:b], q2[a:b], coefs, tol, low, high)
            assert (w[i] >= 0) == found and (not found or (w[i], mc[i]) == (ww, mm)), (i, coefs, tol)


@pytest.mark.parametrize("variant", [1, 2])
def test_fft_order_variants_are_valid_dfts(oracle, variant):
    """The sensitivity study's other FFT orders (scripts/fft_sensitivity.py) are correct DFTs: the
    same float64 agreement as the canonical order, and stored values within a few micro-units."""
    import dsp_f64
    rng = np.random.default_rng(3)
    t = np.arange(8000 * 4)
    pcm = (6000 * np.sin(2 * np.pi * 440 * t / 8000) + 2500 * np.sin(2 * np.pi * 1234.5 * t / 8000)
           + rng.normal(0, 800, len(t))).astype(np.int16)
    base, db0 = oracle.fingerprint_batch(pcm, np.array([0, len(pcm)]))
    mic, db = oracle.fingerprint_batch(pcm, np.array([0, len(pcm)]), fft_variant=variant)
    ref = dsp_f64.fingerprint_f64(pcm, oracle.table_arrays())
    np.testing.assert_allclose(10 ** (db / 10), np.abs(ref), rtol=3e-5, atol=2e-3)
    assert np.abs(mic.astype(np.int64) - base.astype(np.int64)).max() <= 5
    assert (mic != base).any()  # a different rounding pattern, not the same code path
