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
