"""The multi-GPU protocol (tiresias_amd.sharding) on CPU with gloo, world_size 2: clip-sharded
search + one all_reduce(MAX) of per-query keys == the unsharded search, on the SQLite goldens."""
import json
import math
import os
import socket

import numpy as np
import pytest

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle_py
    from tiresias_amd import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with open(os.path.join(REPO, "tests", "golden", "match_cases.json")) as f:
        g = json.load(f)
    results = []
    for s in g["scenarios"]:
        uuids = s["uuids"]
        if not uuids:
            continue
        tb = sharding.global_tiebreak(uuids)
        mine = set(sharding.shard_clips(len(uuids), world, rank).tolist())
        clip = np.asarray(s["clip"])
        sel = np.array([c in mine for c in clip], bool)
        keys = []
        for q in s["queries"]:
            q1 = [math.inf if v is None else v for v in q["q1"]]
            q2 = [math.inf if v is None else v for v in q["q2"]]
            found, w, mc, _ = oracle_py.search(np.asarray(s["m1"])[sel], np.asarray(s["m2"])[sel], clip[sel], uuids,
                                               q1, q2, q["coefs"], q["tol"], q["low"], q["high"])
            keys.append(sharding.make_key(mc, tb[w]) if found else 0)
        t = torch.tensor(keys, dtype=torch.int64)
        sharding.combine(t, dist)
        inv = {int(r): u for u, r in zip(uuids, tb)}
        for q, k in zip(s["queries"], t.tolist()):
            f, mc, r = sharding.decode_key(k)
            got = {"audio_uuid": inv[r], "match_count": mc} if f else None
            exp = None if q["expect"] is None else {"audio_uuid": q["expect"]["audio_uuid"],
                                                    "match_count": q["expect"]["match_count"]}
            results.append(got == exp)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(results, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_search_equals_unsharded(tmp_path, oracle, world):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.json")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    res = json.load(open(out))
    assert len(res) > 900 and all(res)


def test_key_order_matches_sql_sort():
    from tiresias_amd import sharding
    uu = ["b", "a", "c"]
    tb = sharding.global_tiebreak(uu)
    ks = [sharding.make_key(5, tb[0]), sharding.make_key(5, tb[2]), sharding.make_key(4, tb[1])]
    assert max(ks) == ks[1]  # same count -> greatest uuid "c"
    assert sharding.make_key(0, 7) == 0 and sharding.decode_key(ks[1]) == (True, 5, 2)


def _qshard_worker(rank, world, port, out_path):
    """configs[3] protocol with the query batch fingerprinted once across ranks: rank r
    fingerprints its share (oracle), all_gather_rows of the q values (gloo), search of its clip
    shard (oracle), all_reduce(MAX) of the keys; rank 0 checks against the unsharded search."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle_py
    from tiresias_amd import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(3)
    nclips, n_db, nq, qn = 12, 8000 * 4, 4 * world, 8000
    from tiresias_amd import synth_pcm
    db = synth_pcm(0x7153A1, range(nclips), n_db)
    uuids = ["%08x-0000-4000-8000-%012x" % (int(rng.integers(1 << 30)), c) for c in range(nclips)]
    micro, _ = oracle_py.fingerprint_batch(db.reshape(-1), np.arange(nclips + 1) * n_db, want_db=False)
    nf_db = (n_db + 255) // 256
    clip = np.repeat(np.arange(nclips), nf_db).astype(np.int32)
    q = np.stack([db[i % nclips, 256 * (i % 5): 256 * (i % 5) + qn] if i % 4 != 3 else
                  (rng.standard_normal(qn) * 3000).astype(np.int16) for i in range(nq)])
    b, e = sharding.query_share(nq, world, rank)
    nfq = (qn + 255) // 256
    mine = np.concatenate([oracle_py.fingerprint(q[i])[1] for i in range(b, e)])
    qall = torch.empty((world, (e - b) * nfq, 2), dtype=torch.float64)
    sharding.all_gather_rows(qall, torch.from_numpy(mine), dist)
    qv = qall.reshape(-1, 2).numpy()
    tb = sharding.global_tiebreak(uuids)
    sel = np.isin(clip, sharding.shard_clips(nclips, world, rank))
    keys = []
    for i in range(nq):
        f = qv[i * nfq:(i + 1) * nfq]
        found, w, mc, _ = oracle_py.search(micro[sel, 0], micro[sel, 1], clip[sel], uuids, f[:, 0], f[:, 1], 1, 0.45)
        keys.append(sharding.make_key(mc, tb[w]) if found else 0)
    t = torch.tensor(keys, dtype=torch.int64)
    sharding.combine(t, dist)
    if rank == 0:
        ok = []
        for i in range(nq):
            f = oracle_py.fingerprint(q[i])[1]
            found, w, mc, _ = oracle_py.search(micro[:, 0], micro[:, 1], clip, uuids, f[:, 0], f[:, 1], 1, 0.45)
            ok.append(int(t[i]) == (sharding.make_key(mc, tb[w]) if found else 0))
        with open(out_path, "w") as fh:
            json.dump({"ok": ok, "found": int((t != 0).sum())}, fh)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_query_sharded_search_equals_unsharded(tmp_path, oracle, world):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.json")
    mp.spawn(_qshard_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    res = json.load(open(out))
    assert all(res["ok"]) and res["found"] > 0
