"""Device-resident paths (inputs already in HBM): plan + tfp_fingerprint_device,
tfp_index_add_device, tfp_search_device, tfp_synth_pcm_device — equal to the host paths."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_synth_device_equals_host(engine, tfp_lib, torch_cuda):
    torch = torch_cuda
    n = 50000
    d = torch.empty((6, n), dtype=torch.int16, device="cuda")
    engine.synth_device(0x7153A1, range(100, 106), n, d.data_ptr(), offsets=[0, 256, 512, 0, 7, 99999])
    host = tfp_lib.synth_pcm(0x7153A1, range(100, 106), n, offsets=[0, 256, 512, 0, 7, 99999])
    assert np.array_equal(d.cpu().numpy(), host)


def test_device_fingerprint_and_search_equal_host(engine, tfp_lib, torch_cuda):
    torch = torch_cuda
    nclips, n = 64, 8000 * 10
    pcm = torch.empty((nclips, n), dtype=torch.int16, device="cuda")
    engine.synth_device(0x7153A1, range(nclips), n, pcm.data_ptr())
    off = np.arange(nclips + 1, dtype=np.int64) * n
    plan = engine.plan(off)
    micro = torch.empty((plan.nframes, 2), dtype=torch.int32, device="cuda")
    db = torch.empty((plan.nframes, 2), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    engine.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), db.data_ptr(), stream)
    torch.cuda.synchronize()
    host = engine.fingerprint_batch(pcm.cpu().numpy().reshape(-1), off)
    assert np.array_equal(micro.cpu().numpy()[:, 0], host["m1"])
    assert np.array_equal(micro.cpu().numpy()[:, 1], host["m2"])
    assert np.array_equal(db.cpu().numpy()[:, 0], host["q1"])

    # enrol from the device buffer, search device-resident queries
    nf = plan.nframes // nclips
    uuids = ["%08x-0000-4000-8000-%012x" % (i * 7919 % 65536, i) for i in range(nclips)]
    engine.index_clear()
    engine.index_add_device(uuids, np.arange(nclips + 1) * nf, micro.data_ptr(), stream)
    nq, qn = 32, 8000 * 5
    qpcm = torch.empty((nq, qn), dtype=torch.int16, device="cuda")
    engine.synth_device(0x7153A1, [i % nclips for i in range(nq)], qn, qpcm.data_ptr(),
                        offsets=[256 * (i % 50) for i in range(nq)])
    qplan = engine.plan(np.arange(nq + 1, dtype=np.int64) * qn)
    keys = torch.zeros(nq, dtype=torch.int64, device="cuda")
    p = tfp_lib.params(1, 0.05)
    engine.search_device(qplan, qpcm.data_ptr(), p, keys.data_ptr(), stream)
    torch.cuda.synchronize()
    res, _ = engine.search_pcm_batch(qpcm.cpu().numpy().reshape(-1), np.arange(nq + 1) * qn, p)
    k = keys.cpu().numpy().view(np.uint64)
    for i in range(nq):
        if res[i] is None:
            assert k[i] == 0
        else:
            assert int(k[i] >> np.uint64(32)) == res[i]["match_count"]
            assert engine.uuid_of_key(int(k[i] & np.uint64(0xffffffff))) == res[i]["audio_uuid"]
    engine.index_clear()


def test_search_q_device_equals_search_device(engine, tfp_lib, torch_cuda):
    """tfp_search_q_device on frame values fingerprinted in two halves (as two ranks of the
    query-sharded configs[3] step would, concatenated) == tfp_search_device on the whole batch."""
    torch = torch_cuda
    nclips, n = 48, 8000 * 10
    pcm = torch.empty((nclips, n), dtype=torch.int16, device="cuda")
    engine.synth_device(0x7153A1, range(nclips), n, pcm.data_ptr())
    plan = engine.plan(np.arange(nclips + 1, dtype=np.int64) * n)
    micro = torch.empty((plan.nframes, 2), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    engine.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, stream)
    nf = plan.nframes // nclips
    engine.index_clear()
    engine.index_add_device(["%08x-0000-4000-8000-%012x" % (i * 31, i) for i in range(nclips)],
                            np.arange(nclips + 1) * nf, micro.data_ptr(), stream)
    nq, qn = 40, 8000 * 5
    nfq = (qn + 255) // 256
    qpcm = torch.empty((nq, qn), dtype=torch.int16, device="cuda")
    engine.synth_device(0x7153A1, [i % nclips for i in range(nq)], qn, qpcm.data_ptr(),
                        offsets=[256 * (i % 40) for i in range(nq)])
    half = engine.plan(np.arange(nq // 2 + 1, dtype=np.int64) * qn)
    q = torch.empty((nq * nfq, 2), dtype=torch.float64, device="cuda")
    qm = torch.empty((nq * nfq, 2), dtype=torch.int32, device="cuda")
    for h in range(2):
        rows = slice(h * (nq // 2) * nfq, (h + 1) * (nq // 2) * nfq)
        engine.fingerprint_device(half, qpcm[h * (nq // 2):].data_ptr(), qm[rows].data_ptr(), q[rows].data_ptr(), stream)
    for p in (tfp_lib.params(1, 0.001), tfp_lib.params(1, 0.3), tfp_lib.params(2, 0.5)):
        k1 = torch.zeros(nq, dtype=torch.int64, device="cuda")
        k2 = torch.zeros(nq, dtype=torch.int64, device="cuda")
        engine.search_q_device(q.data_ptr(), np.arange(nq + 1) * nfq, p, k1.data_ptr(), stream)
        engine.search_device(engine.plan(np.arange(nq + 1, dtype=np.int64) * qn), qpcm.data_ptr(), p, k2.data_ptr(), stream)
        torch.cuda.synchronize()
        assert torch.equal(k1, k2)
    assert int((k2 != 0).sum()) > 0


def test_tiebreak_override_covers_every_live_clip(engine, tfp_lib):
    """A clip added after tfp_index_set_tiebreak has no global key: the next search fails with
    TFP_E_ARG instead of giving it a local rank that may collide; duplicate keys fail too."""
    rng = np.random.default_rng(2)
    engine.index_clear()
    for c in range(4):
        engine.index_add("u%d" % c, rng.integers(0, 9, 20) * 1000000, rng.integers(0, 9, 20) * 1000000)
    engine.set_tiebreak(np.array([10, 40, 20, 30], np.int32))
    engine.index_commit()
    engine.index_add("u4", np.zeros(5, np.int32), np.zeros(5, np.int32))
    with pytest.raises(tfp_lib.TfpError):
        engine.index_commit()
    engine.set_tiebreak(np.array([10, 40, 20, 30, 40], np.int32))  # duplicate 40
    with pytest.raises(tfp_lib.TfpError):
        engine.index_commit()
    engine.set_tiebreak(np.array([10, 40, 20, 30, 50], np.int32))
    engine.index_commit()
    assert engine.uuid_of_key(50) == "u4"
    engine.set_tiebreak(np.zeros(0, np.int32))  # cleared: uuid ranks again
    engine.index_commit()
    assert engine.uuid_of_key(4) == "u4"
    engine.index_clear()


def test_remove_readd_cycles_compact_staging(engine, oracle, tfp_lib):
    """Delete / re-enrol cycles (tfp_index_remove + tfp_index_add) keep the search exact while the
    staging rows of removed clips are compacted away."""
    rng = np.random.default_rng(8)
    engine.index_clear()
    nclips, nrows = 40, 3000
    rows = {}
    for c in range(nclips):
        rows[c] = ((rng.integers(-3, 4, nrows) * 1000000 + rng.integers(-900, 901, nrows)).astype(np.int32),
                   rng.integers(-5000000, 5000000, nrows).astype(np.int32))
        engine.index_add("clip-%03d" % c, *rows[c])
    for cycle in range(30):  # ~30 x 20 x 3000 rows removed: several compactions
        for c in rng.choice(nclips, 20, replace=False):
            engine.index_remove("clip-%03d" % c)
            rows[c] = ((rng.integers(-3, 4, nrows) * 1000000 + rng.integers(-900, 901, nrows)).astype(np.int32),
                       rng.integers(-5000000, 5000000, nrows).astype(np.int32))
            engine.index_add("clip-%03d" % c, *rows[c])
        if cycle % 10 == 9:
            uuids = ["clip-%03d" % c for c in range(nclips)]
            m1 = np.concatenate([rows[c][0] for c in range(nclips)])
            m2 = np.concatenate([rows[c][1] for c in range(nclips)])
            clip = np.repeat(np.arange(nclips), nrows)
            q1 = rng.integers(-3, 4, 50) + 0.4
            fr = np.zeros(50, np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                        ("q1", "<f8"), ("q2", "<f8")]))
            fr["q1"] = q1
            res, _ = engine.search_batch(fr, [0, 50], tfp_lib.params(1, 0.001))
            found, w, mc, _ = oracle.search(m1, m2, clip, uuids, q1, np.zeros(50), 1, 0.001)
            assert (res[0]["audio_uuid"], res[0]["match_count"]) == (uuids[w], mc)
            for c in (0, 17, 39):
                a, b = engine.index_rows("clip-%03d" % c)
                assert np.array_equal(a, rows[c][0]) and np.array_equal(b, rows[c][1])
    assert engine.index_stats() == (nclips * nrows, nclips)
    engine.index_clear()


def test_scan_path_on_caller_stream_then_host_search(engine, tfp_lib, torch_cuda):
    """tfp_search_q_device with coefs=2 (scan path) on a torch stream, immediately followed by a
    host search on the engine's own stream: the shared scratch must not be overwritten while the
    first search still runs (each result equals the same search run alone)."""
    torch = torch_cuda
    nclips, n = 32, 8000 * 10
    pcm = tfp_lib.synth_pcm(0x7153A1, range(nclips), n)
    fr = engine.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n)
    nf = fr.shape[0] // nclips
    engine.index_clear()
    engine.index_add_batch(["s%03d" % c for c in range(nclips)], np.arange(nclips + 1) * nf, fr["m1"], fr["m2"])
    nq, qn = 16, 8000 * 3
    q = np.stack([pcm[i % nclips, 256 * i: 256 * i + qn] for i in range(nq)])
    qfr = engine.fingerprint_batch(q.reshape(-1), np.arange(nq + 1) * qn)
    nfq = qfr.shape[0] // nq
    d_q = torch.from_numpy(np.stack([qfr["q1"], qfr["q2"]], 1).copy()).cuda()
    p2 = tfp_lib.params(2, 0.5)
    alone = torch.zeros(nq, dtype=torch.int64, device="cuda")
    side = torch.cuda.Stream()
    engine.search_q_device(d_q.data_ptr(), np.arange(nq + 1) * nfq, p2, alone.data_ptr(), side.cuda_stream)
    torch.cuda.synchronize()
    ref_host, _ = engine.search_batch(qfr, np.arange(nq + 1) * nfq, tfp_lib.params(1, 0.3))
    for _ in range(5):
        keys = torch.zeros(nq, dtype=torch.int64, device="cuda")
        engine.search_q_device(d_q.data_ptr(), np.arange(nq + 1) * nfq, p2, keys.data_ptr(), side.cuda_stream)
        host, _ = engine.search_batch(qfr, np.arange(nq + 1) * nfq, tfp_lib.params(1, 0.3))
        torch.cuda.synchronize()
        assert torch.equal(keys, alone)
        assert host == ref_host
    engine.index_clear()


def test_host_alloc_buffers_read_in_place(engine, tfp_lib):
    """tfp_host_alloc buffers, which the small path's kernel reads where they lie (no staging copy),
    give the same results as ordinary memory: queries at the buffer's start and at two misaligned
    sample offsets (checked loads), a single query, and a small fingerprint call."""
    import ctypes
    from tiresias_amd._lib import lib
    L = lib()
    nclips, n_db, qn = 24, 8000 * 10, 8000 * 3
    db = tfp_lib.synth_pcm(0x7153A1, range(nclips), n_db)
    fr = engine.fingerprint_batch(db.reshape(-1), np.arange(nclips + 1) * n_db)
    nf = (n_db + 255) // 256
    engine.index_clear()
    engine.index_add_batch(["%08x-0000-4000-8000-%012x" % (i * 7919 % 65536, i) for i in range(nclips)],
                           np.arange(nclips + 1) * nf, fr["m1"], fr["m2"])
    q = tfp_lib.synth_pcm(0x7153A1, [3, 7, 11], qn, offsets=[256 * 5, 999, 0]).reshape(-1)
    off = np.arange(4, dtype=np.int64) * qn
    p = tfp_lib.params(1, 0.001)
    ref, _ = engine.search_pcm_batch(q, off, p)
    assert sum(r is not None for r in ref) == 3
    ptr = ctypes.c_void_p()
    total = 3 * qn + 8
    assert L.tfp_host_alloc(2 * total, ctypes.byref(ptr)) == 0 and ptr.value
    try:
        buf = np.ctypeslib.as_array((ctypes.c_int16 * total).from_address(ptr.value))
        for start in (0, 1, 7):
            buf[start:start + 3 * qn] = q
            got, _ = engine.search_pcm_batch(buf[start:start + 3 * qn], off, p)
            assert got == ref, start
            one, _ = engine.search_pcm_batch(buf[start:start + qn], [0, qn], p)
            assert one[0] == ref[0], start
        buf[:3 * qn] = q
        fa = engine.fingerprint_batch(buf[:3 * qn], off)
        fb = engine.fingerprint_batch(q, off)
        assert np.array_equal(fa["m1"], fb["m1"]) and np.array_equal(fa["m2"], fb["m2"])
    finally:
        L.tfp_host_free(ptr)
    bad = ctypes.c_void_p()
    assert L.tfp_host_alloc(0, ctypes.byref(bad)) != 0
    L.tfp_host_free(None)
    engine.index_clear()


def test_device_fingerprint_of_a_clip_past_the_buffer_range(engine, oracle, torch_cuda):
    """A clip of >= 2^30 - 2^16 samples (kDirectMaxSamples, 37 h at 8 kHz) would overflow the 8 kHz
    kernel's 32-bit buffer range and offsets; the plan sends it to the generic kernel (64-bit sample
    offsets). Its first frames, frames in the middle and its zero-padded end equal the oracle's
    fingerprints of the same samples (frame f depends only on hops f - 1 and f, so a slice that starts
    one hop before frame f reproduces it from its second frame on)."""
    torch = torch_cuda
    n = (1 << 30) - (1 << 16) + 12345
    pcm = torch.empty(n, dtype=torch.int16, device="cuda")
    engine.synth_device(0x7153C3, [5], n, pcm.data_ptr())
    plan = engine.plan(np.array([0, n], dtype=np.int64))
    micro = torch.empty((plan.nframes, 2), dtype=torch.int32, device="cuda")
    engine.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    nf = plan.nframes
    assert nf == (n + 255) // 256
    for f0 in (0, nf // 2 + 3, nf - 40):
        s0 = max(0, 256 * (f0 - 1))
        s1 = min(n, 256 * (f0 + 40))
        x = pcm[s0:s1].cpu().numpy()
        _, _, want = oracle.fingerprint(x)
        skip = 0 if f0 == 0 else 1
        got = micro[f0:f0 + len(want) - skip].cpu().numpy()
        assert np.array_equal(got, want[skip:skip + len(got)]), f0
    del pcm, micro
    torch.cuda.empty_cache()
