"""Concurrent callers on one engine. The reference's fp_search_fingerprint_info is called from many
channel threads at once, plus the CLI and the load thread (SURVEY §8b threading row); the C-ABI
serialises every call per engine, so results under concurrency must equal the serial ones.
ctypes releases the GIL during each foreign call, so these threads really overlap in the C-ABI."""
import threading

import numpy as np
import pytest

from test_gpu_parity import _build_db, _queries

pytestmark = pytest.mark.gpu


def _key(r):
    return None if r is None else (r["audio_uuid"], r["match_count"])


def test_concurrent_searches_equal_serial(engine, oracle, tfp_lib):
    _build_db(engine, oracle, tfp_lib, 120, 12)
    qpcm = _queries(tfp_lib, 24, 120, 12, 5)
    n = qpcm.shape[1]
    params = [tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.1), tfp_lib.params(2, 0.5), tfp_lib.params(1, 0.001, 100, 3400)]
    # serial answers: single queries (small path) per parameter set, and the fingerprints
    want = {}
    for pi, p in enumerate(params):
        for q in range(24):
            r, f = engine.search_pcm_batch(qpcm[q], [0, n], p)
            want[pi, q] = (_key(r[0]), f[0])
    fp_want = engine.fingerprint_batch(qpcm[:6].reshape(-1), np.arange(7) * n)

    errors = []

    def worker(t):
        rng = np.random.default_rng(100 + t)
        try:
            for it in range(12):
                pi = int(rng.integers(len(params)))
                kind = int(rng.integers(4))
                if kind == 0:  # one query (batch-1 path)
                    q = int(rng.integers(24))
                    r, f = engine.search_pcm_batch(qpcm[q], [0, n], params[pi])
                    got = [(_key(r[0]), f[0])]
                    exp = [want[pi, q]]
                elif kind == 1:  # a few queries (small batch)
                    q0 = int(rng.integers(0, 21))
                    r, f = engine.search_pcm_batch(qpcm[q0:q0 + 3].reshape(-1), np.arange(4) * n, params[pi])
                    got = [(_key(a), b) for a, b in zip(r, f)]
                    exp = [want[pi, q] for q in range(q0, q0 + 3)]
                elif kind == 2:  # the whole set (vote GEMM / class path)
                    r, f = engine.search_pcm_batch(qpcm.reshape(-1), np.arange(25) * n, params[pi])
                    got = [(_key(a), b) for a, b in zip(r, f)]
                    exp = [want[pi, q] for q in range(24)]
                else:  # fingerprints in between searches
                    fr = engine.fingerprint_batch(qpcm[:6].reshape(-1), np.arange(7) * n)
                    got = [bool(np.array_equal(fr["m1"], fp_want["m1"]) and np.array_equal(fr["m2"], fp_want["m2"]))]
                    exp = [True]
                if got != exp:
                    errors.append((t, it, kind, pi, got[:3], exp[:3]))
        except Exception as ex:  # pragma: no cover - reported below
            errors.append((t, repr(ex)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a caller thread did not finish"
    assert not errors, errors[:5]
    assert any(v[0] is not None for v in want.values())


def test_group_concurrent_searches_during_enrolment(oracle, tfp_lib):
    """The shim's device group (tfp_group_*) under the module's real mix: channel threads
    searching while the load / CLI thread enrols and deletes (src/app_tiresias.c:413,
    src/cli_handler.c). The enrolled-and-deleted clips hold only NULL rows (a file whose every
    coefficient printed as inf: src/fp_handler.c:649-652), which no box ever matches, so every
    search must equal its serial answer whatever the interleaving, while each enrolment and
    deletion forces an index merge on a shard between the searches."""
    g = tfp_lib.Group([0, 0, 0])
    class _Rows:  # _build_db's rows and uuids, added to the group below instead of an engine
        def index_clear(self):
            pass

        def index_add(self, *a):
            pass

    uuids, micro, _ = _build_db(_Rows(), oracle, tfp_lib, 120, 12)
    nf = len(micro) // 120
    for c in range(120):
        g.index_add(uuids[c], micro[c * nf:(c + 1) * nf, 0], micro[c * nf:(c + 1) * nf, 1])
    g.index_commit()
    qpcm = _queries(tfp_lib, 24, 120, 12, 5)
    n = qpcm.shape[1]
    params = [tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.1), tfp_lib.params(2, 0.5)]
    want = {}
    for pi, p in enumerate(params):
        r, f = g.search_pcm_batch(qpcm.reshape(-1), np.arange(25) * n, p)
        for q in range(24):
            want[pi, q] = (_key(r[q]), f[q])
    assert any(v[0] is not None for v in want.values())
    null_rows = np.full(nf, tfp_lib.NULL_MICRO, np.int32)
    errors, stop = [], threading.Event()

    def searcher(t):
        rng = np.random.default_rng(200 + t)
        try:
            for it in range(10):
                pi = int(rng.integers(len(params)))
                q0 = int(rng.integers(0, 22))
                k = 1 if it % 2 else 3
                r, f = g.search_pcm_batch(qpcm[q0:q0 + k].reshape(-1), np.arange(k + 1) * n, params[pi])
                got = [(_key(a), b) for a, b in zip(r, f)]
                exp = [want[pi, q] for q in range(q0, q0 + k)]
                if got != exp:
                    errors.append((t, it, pi, q0, got, exp))
        except Exception as ex:  # pragma: no cover - reported below
            errors.append((t, repr(ex)))

    def enroller():
        i = 0
        try:
            while not stop.is_set() and i < 200:
                u = "%08x-0000-4000-8000-%012x" % (0xE0000000 + i, i)
                g.index_add(u, null_rows, null_rows)
                if i % 3 == 2:
                    g.index_remove(u)
                i += 1
        except Exception as ex:  # pragma: no cover
            errors.append(("enrol", repr(ex)))

    threads = [threading.Thread(target=searcher, args=(t,)) for t in range(6)]
    en = threading.Thread(target=enroller)
    en.start()
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=200)
    stop.set()
    en.join(timeout=100)
    assert not any(th.is_alive() for th in threads + [en]), "a caller thread did not finish"
    assert not errors, errors[:5]
    # the NULL-row clips are enrolled (and counted) but never match
    nrows, nclips = g.index_stats()
    assert nclips > 120
    for pi, p in enumerate(params):
        r, f = g.search_pcm_batch(qpcm.reshape(-1), np.arange(25) * n, p)
        assert [(_key(r[q]), f[q]) for q in range(24)] == [want[pi, q] for q in range(24)]
    g.close()


def _stats(fn, h):
    import ctypes as C
    a, b = C.c_int64(), C.c_int64()
    assert fn(h, C.byref(a), C.byref(b)) == 0
    return a.value, b.value


@pytest.mark.parametrize("kind", ["engine", "group"])
def test_failing_caller_in_coalesced_batch_is_isolated(oracle, tfp_lib, kind, monkeypatch):
    """32 channel threads search at once on one shared handle (application_handler.c:180 over
    fp_handler.c:1161-1169) while one of them submits a query that fails on the device (test knob
    TFP_TEST_FAIL_QUERY_SAMPLES: a forced allocation failure for a query of that length). Concurrent
    calls are coalesced into shared batches (tfp_coalesce.hpp); a batch holding the failing query
    fails as a whole and is re-run request by request, so the 31 others get their serial results and
    only the failing caller sees an error, with its own message read on its own thread."""
    from tiresias_amd._lib import TfpError, lib
    bad_len = 8000 * 2 + 77
    monkeypatch.setenv("TFP_TEST_FAIL_QUERY_SAMPLES", str(bad_len))
    h = tfp_lib.Engine(0) if kind == "engine" else tfp_lib.Group([0, 0])
    try:
        n = 8000 * 12
        pcm = tfp_lib.synth_pcm(7, range(60), n)
        micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(61) * n, nthreads=8, want_db=False)
        nf = (n + 255) // 256
        for c in range(60):
            h.index_add("%032x" % (c + 1), micro[c * nf:(c + 1) * nf, 0], micro[c * nf:(c + 1) * nf, 1])
        # 31 three-second excerpts of enrolled clips (the 31 good callers' queries)
        qpcm = np.stack([tfp_lib.synth_pcm(7, [2 * c], 8000 * 3, offsets=[256 * (7 * c + 3)])[0] for c in range(31)])
        nq = qpcm.shape[1]
        p = tfp_lib.params(1, 0.001)
        want = [_key(h.search_pcm_batch(qpcm[t], [0, nq], p)[0][0]) for t in range(31)]
        assert sum(w is not None for w in want) >= 8
        bad = tfp_lib.synth_pcm(99, [0], bad_len)[0]
        with pytest.raises(TfpError) as ei:  # alone, first: the knob is live
            h.search_pcm_batch(bad, [0, bad_len], p)
        assert "TFP_TEST_FAIL_QUERY_SAMPLES" in str(ei.value)
        statfn = lib().tfp_search_coalesce_stats if kind == "engine" else lib().tfp_group_search_coalesce_stats
        c0, b0 = _stats(statfn, h.handle)
        iters = 25
        bar = threading.Barrier(32)
        errors, bad_seen = [], []

        def worker(t):
            try:
                for it in range(iters):
                    bar.wait(timeout=60)
                    if t == 31:
                        try:
                            h.search_pcm_batch(bad, [0, bad_len], p)
                            errors.append((t, it, "no error"))
                        except TfpError as ex:
                            bad_seen.append(str(ex))
                    else:
                        r, f = h.search_pcm_batch(qpcm[t], [0, nq], p)
                        if _key(r[0]) != want[t] or f[0] != tfp_lib.frame_count(nq):
                            errors.append((t, it, _key(r[0]), want[t]))
            except Exception as ex:  # pragma: no cover - reported below
                errors.append((t, repr(ex)))
                bar.abort()

        threads = [threading.Thread(target=worker, args=(t,)) for t in range(32)]
        for th in threads:
            th.start()
        for th in threads:
            th.join(timeout=200)
        assert not any(th.is_alive() for th in threads), "a caller thread did not finish"
        assert not errors, errors[:5]
        assert len(bad_seen) == iters
        # the failing caller's own message (its query alone: "query 0 of 1"), never a neighbour's
        assert all("TFP_TEST_FAIL_QUERY_SAMPLES" in m and "query 0 of 1" in m for m in bad_seen), bad_seen[:3]
        c1, b1 = _stats(statfn, h.handle)
        assert c1 - c0 == 32 * iters and b1 - b0 < c1 - c0  # calls were coalesced (some batches held the bad query)
    finally:
        h.close()


def test_operational_switches_without_test_knobs(tfp_lib, monkeypatch):
    """TFP_COALESCE=0 (include/tiresias_fp.h) is an operational switch: it takes effect without
    TFP_TEST_KNOBS (which only gates the test-form knobs), so a deployment that follows the header
    gets what it documents. A search through the engine then never enters the coalescer."""
    from tiresias_amd._lib import lib
    monkeypatch.setenv("TFP_TEST_KNOBS", "0")
    n = 8000 * 4
    pcm = tfp_lib.synth_pcm(11, range(3), n)
    p = tfp_lib.params(1, 0.45)
    for setting, expect_calls in (("0", 0), ("1", 1)):
        monkeypatch.setenv("TFP_COALESCE", setting)
        eng = tfp_lib.Engine(0)
        try:
            fr = eng.fingerprint_batch(pcm.reshape(-1), np.arange(4) * n)
            nf = (n + 255) // 256
            for c in range(3):
                eng.index_add("%032x" % (c + 1), fr["m1"][c * nf:(c + 1) * nf], fr["m2"][c * nf:(c + 1) * nf])
            eng.search_pcm_batch(pcm[1], [0, n], p)
            calls, _ = _stats(lib().tfp_search_coalesce_stats, eng.handle)
            assert calls == expect_calls, (setting, calls)
        finally:
            eng.close()
