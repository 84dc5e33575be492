"""The multi-GPU protocol (tiresias_amd.sharding) on the HIP engine itself:
2 and 3 ranks, each a fresh process with its own Engine on this box's GPU over a round-robin clip
shard, joined by gloo. Each rank: tfp_index_set_tiebreak with the global uuid ranks,
QueryShardedSearch (fingerprint 1/N of the queries, all_gather of the frame values,
tfp_search_q_device on the local clips, all_reduce(MAX) of the keys) and the batch-1 key
combine. Every key must equal the unsharded engine's and the oracle's (count(*) DESC, ties to the
greatest audio_uuid: src/fp_handler.c:367-374).

World 1 runs the same step over RCCL (backend "nccl"), the backend bench.py's N-GPU runs use: its
all_gather_into_tensor of the frame values and an explicit int64 all_reduce(MAX) of the keys
(identities at one rank, but the RCCL calls, dtypes and tensor shapes of the N-GPU path)."""
import json
import os
import socket

import numpy as np
import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

SEED_DB, SEED_Q = 0x7153A1, 0x7153B2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, backend="gloo"):
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle_py
    import tiresias_amd as T
    from tiresias_amd import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world)
    stream = torch.cuda.current_stream().cuda_stream
    nclips, n_db, qn = 60, 8000 * 10, 8000 * 3
    nf_db = (n_db + 255) // 256
    nfq = (qn + 255) // 256
    rng = np.random.default_rng(9)
    uuids = [str(__import__("uuid").UUID(bytes=rng.bytes(16), version=4)) for _ in range(nclips)]
    # ties on purpose: clips 40..59 repeat the audio of clips 0..19 under other uuids
    src = [c if c < 40 else c - 40 for c in range(nclips)]
    pcm = T.synth_pcm(SEED_DB, src, n_db)
    grank = sharding.global_tiebreak(uuids)
    eng = T.Engine(0)
    mine = sharding.shard_clips(nclips, world, rank)
    fr = eng.fingerprint_batch(pcm[mine].reshape(-1), np.arange(len(mine) + 1) * n_db)
    eng.index_add_batch([uuids[c] for c in mine], np.arange(len(mine) + 1) * nf_db, fr["m1"], fr["m2"])
    eng.set_tiebreak(grank[mine])
    nq = 12 * max(world, 2)
    qsrc = [(SEED_DB, src[int(rng.integers(nclips))], 256 * int(rng.integers(0, 100)) + int(rng.integers(0, 3)) * 17)
            if i % 4 != 3 else (SEED_Q, i, 0) for i in range(nq)]
    qpcm = np.stack([T.synth_pcm(sd, [c], qn, offsets=[o])[0] for sd, c, o in qsrc])
    d_q = torch.from_numpy(qpcm).to(dev)
    out = {"batch": [], "single": []}
    for p in (T.params(1, 0.001), T.params(1, 0.3), T.params(2, 0.5), T.params(1, 0.2, 100, 3400)):
        keys = torch.zeros(nq, dtype=torch.int64, device=dev)
        qs = sharding.QueryShardedSearch(eng, torch, dev, dist, nq, qn)
        qs(d_q.data_ptr(), p, keys, stream)
        if backend == "nccl":  # sharding.combine skips a 1-rank group: run the RCCL reduction anyway
            dist.all_reduce(keys, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize()
        out["batch"].append([int(v) for v in keys.cpu().numpy().view(np.uint64)])
    # batch-1: local small-path result -> global key -> 8-byte all_reduce(MAX)
    for i in range(6):
        res, _ = eng.search_pcm_batch(qpcm[i], [0, qn], T.params(1, 0.001))
        r = res[0]
        k = torch.tensor([sharding.make_key(r["match_count"], grank[uuids.index(r["audio_uuid"])]) if r else 0],
                         dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        sharding.combine(k, dist)
        out["single"].append(int(k.item()))
    if rank == 0:
        # the unsharded engine on every clip, and the oracle, on the same queries
        full = T.Engine(0)
        frall = full.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n_db)
        full.index_add_batch(uuids, np.arange(nclips + 1) * nf_db, frall["m1"], frall["m2"])
        clip = np.repeat(np.arange(nclips), nf_db)
        exp_batch, exp_engine = [], []
        for p in (T.params(1, 0.001), T.params(1, 0.3), T.params(2, 0.5), T.params(1, 0.2, 100, 3400)):
            keys = torch.zeros(nq, dtype=torch.int64, device=dev)
            full.search_device(full.plan(np.arange(nq + 1, dtype=np.int64) * qn), d_q.data_ptr(), p, keys.data_ptr(),
                               stream)
            torch.cuda.synchronize()
            exp_engine.append([int(v) for v in keys.cpu().numpy().view(np.uint64)])
            ek = []
            for i in range(nq):
                _, qdb, _ = oracle_py.fingerprint(qpcm[i])
                found, w, mc, _ = oracle_py.search(frall["m1"], frall["m2"], clip, uuids, qdb[:, 0], qdb[:, 1], p.coefs,
                                                   p.tolerance, p.freq_ignore_low, p.freq_ignore_high)
                ek.append(sharding.make_key(mc, grank[w]) if found else 0)
            exp_batch.append(ek)
        out["expect_oracle"] = exp_batch
        out["expect_engine"] = [[int(v) for v in e] for e in exp_engine]
        out["found"] = int(sum(k != 0 for k in exp_batch[0]))
        full.close()
        with open(out_path, "w") as f:
            json.dump(out, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(1, "nccl"), (2, "gloo"), (3, "gloo")])
def test_sharded_hip_engine_equals_unsharded(tmp_path, world, backend):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.json")
    mp.spawn(_worker, args=(world, _free_port(), out, backend), nprocs=world, join=True)
    r = json.load(open(out))
    assert r["batch"] == r["expect_oracle"] == r["expect_engine"]
    assert r["single"] == r["expect_oracle"][0][:6]
    assert r["found"] > 4
