"""configs[3] at its own workload: the 100k-clip DB sharded 8 ways.

Eight fresh processes (mp.spawn, gloo), each with its own Engine on this box's one GPU, play the
eight ranks of bench.py's configs[3] step: each enrols its round-robin 12,500-clip shard of the
100,000 x 30 s DB exactly as bench.enroll does, sets the global uuid-rank tie keys, runs
QueryShardedSearch on bench.c3_queries' 4,096 x 5 s batch (fingerprint 1/8 of the queries,
all_gather of the frame values, search of the local clips, all_reduce(MAX) of the keys) and the
batch-1 key combine. The parent checks every key against the unsharded engine over all 100,000
clips and against the oracle's sorted-index search over the same 93.8 M rows (count(*) DESC,
ties to the greatest audio_uuid: src/fp_handler.c:367-374; clip-aligned shards: :353)."""
import json
import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

DB_CLIPS, NQ, WORLD = 100_000, 4096, 8
PARAMS = [(1, 0.001, -1, -1), (2, 0.001, -1, -1)]
N_COEFS2 = 256  # queries checked at coefs = 2 (the oracle's per-frame box scans)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, PKG)
    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist
    import bench
    import tiresias_amd as T
    from tiresias_amd import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sh = torch.cuda.current_stream().cuda_stream
    eng = T.Engine(0)
    mine = sharding.shard_clips(DB_CLIPS, world, rank).tolist()
    bench.enroll(eng, torch, dev, sh, mine)
    if rank == 0:
        print("[c4] rank 0 enrolled %d clips" % len(mine), flush=True)
    grank = sharding.global_tiebreak([bench.uuid_of(g) for g in range(DB_CLIPS)])
    eng.set_tiebreak(grank[mine])
    eng.index_commit()
    qn = 8000 * 5
    qpcm = bench.c3_queries(eng, torch, dev, sh, NQ, DB_CLIPS)
    out = {"rank": rank, "rows": eng.index_stats()[0], "batch": []}
    qs = sharding.QueryShardedSearch(eng, torch, dev, dist, NQ, qn)
    for coefs, tol, lo, hi in PARAMS:
        keys = torch.zeros(NQ, dtype=torch.int64, device=dev)
        qs(qpcm.data_ptr(), T.params(coefs, tol, lo, hi), keys, sh)
        torch.cuda.synchronize()
        out["batch"].append([int(v) for v in keys.cpu().numpy().view(np.uint64)])
    # batch-1: the local small-path winner -> global key -> 8-byte all_reduce(MAX)
    host = qpcm[:8].cpu().numpy()
    clip_of = {bench.uuid_of(g): g for g in mine}
    out["single"] = []
    for i in range(8):
        res, _ = eng.search_pcm_batch(host[i], [0, qn], T.params(1, 0.001))
        r = res[0]
        k = torch.tensor([sharding.make_key(r["match_count"], int(grank[clip_of[r["audio_uuid"]]])) if r else 0],
                         dtype=torch.int64)
        sharding.combine(k, dist)
        out["single"].append(int(k.item()))
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump(out, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(1200)
def test_configs3_sharded_8_ranks_equals_unsharded_and_oracle(tmp_path, oracle, tfp_lib):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    print("[c4] 8 ranks done", flush=True)
    outs = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(WORLD)]
    for o in outs[1:]:  # every rank holds the same reduced keys
        assert o["batch"] == outs[0]["batch"] and o["single"] == outs[0]["single"]
    assert sum(o["rows"] for o in outs) == DB_CLIPS * 938

    # the unsharded engine over all 100,000 clips, and the oracle over the same rows
    sys.path.insert(0, REPO)
    import bench
    from test_gpu_configs import _enroll_db
    dev = torch.device("cuda", 0)
    sh = torch.cuda.current_stream().cuda_stream
    eng = tfp_lib.Engine(0)
    rows, _ = _enroll_db(eng, torch, dev, sh, list(range(DB_CLIPS)))
    qn = 8000 * 5
    qpcm = bench.c3_queries(eng, torch, dev, sh, NQ, DB_CLIPS)
    plan = eng.plan(np.arange(NQ + 1, dtype=np.int64) * qn)
    uuids = [bench.uuid_of(g) for g in range(DB_CLIPS)]
    order = np.argsort(np.asarray(uuids))
    rank = np.empty(DB_CLIPS, np.int32)
    rank[order] = np.arange(DB_CLIPS, dtype=np.int32)
    print("[c4] unsharded engine enrolled", flush=True)
    idx = oracle.SortedIndex(rows[:, 0], rows[:, 1], np.repeat(np.arange(DB_CLIPS, dtype=np.int32), 938), rank)
    print("[c4] oracle index sorted", flush=True)
    del rows
    host = qpcm.cpu().numpy()
    nfq = (qn + 255) // 256
    qoff = np.arange(NQ + 1, dtype=np.int64) * nfq
    _, qdb = oracle.fingerprint_batch(host.reshape(-1), np.arange(NQ + 1) * qn, nthreads=16)
    for j, (coefs, tol, lo, hi) in enumerate(PARAMS):
        keys = torch.zeros(NQ, dtype=torch.int64, device=dev)
        eng.search_device(plan, qpcm.data_ptr(), tfp_lib.params(coefs, tol, lo, hi), keys.data_ptr(), sh)
        torch.cuda.synchronize()
        unsharded = keys.cpu().numpy().view(np.uint64)
        sharded = np.array(outs[0]["batch"][j], np.uint64)
        nchk = NQ if coefs == 1 else N_COEFS2
        w, mc = idx.search_batch(qdb[:nchk * nfq, 0], qdb[:nchk * nfq, 1], qoff[:nchk + 1], coefs, tol, lo, hi,
                                 nthreads=16)
        exp = np.where(w >= 0, (mc.astype(np.uint64) << np.uint64(32)) | rank[np.maximum(w, 0)].astype(np.uint64), 0)
        exp = exp.astype(np.uint64)
        # each against the oracle first (a mismatch names the side and the queries), then each other
        bad_u = np.nonzero(unsharded[:nchk] != exp)[0]
        bad_s = np.nonzero(sharded[:nchk] != exp)[0]
        assert bad_u.size == 0, ("unsharded", coefs, bad_u.size, bad_u[:8], unsharded[bad_u[:4]], exp[bad_u[:4]])
        assert bad_s.size == 0, ("sharded", coefs, bad_s.size, bad_s[:8], sharded[bad_s[:4]], exp[bad_s[:4]])
        assert np.array_equal(sharded, unsharded), (coefs, np.nonzero(sharded != unsharded)[0][:8])
        if coefs == 1:
            assert (w >= 0).sum() >= 1000
    assert outs[0]["single"] == [int(v) for v in np.array(outs[0]["batch"][0][:8], np.uint64)]
    eng.close()
