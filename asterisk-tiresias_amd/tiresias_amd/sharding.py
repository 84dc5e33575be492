"""Clip-sharded search across GPUs: the multi-GPU protocol.

The enrolled DB is split by clip — never inside a clip, because the per-frame
`GROUP BY audio_uuid` dedup of fp_handler.c:353 is not additive across a split clip. Every
rank searches the same queries against its own clips and reduces each query to one 64-bit key

    key = match_count << 32 | global_uuid_rank      (0 = no hit on this rank)

ordered exactly like the reference's final sort (count(*) DESC, ties -> greatest audio_uuid,
fp_handler.c:367). One all_reduce(MAX) of the keys over RCCL (backend "nccl") gives every
rank the global winner.

A query batch is fingerprinted once, not once per rank: each rank fingerprints an equal share
of the queries, one all_gather of the frame values (q1, q2: 16 B per frame) gives every rank
the whole batch, and each searches its clips (`QueryShardedSearch`). The frame values are the
same bits whichever GPU computes them, so the result is the unsharded search's.
"""
from __future__ import annotations

import numpy as np


def shard_clips(nclips: int, world: int, rank: int) -> np.ndarray:
    """Round-robin clip ids owned by `rank`."""
    return np.arange(rank, nclips, world, dtype=np.int64)


def global_tiebreak(uuids) -> np.ndarray:
    """Rank of every uuid in the lexicographic order of all uuids (the SQLite tie-break)."""
    order = np.argsort(np.asarray(uuids))
    rank = np.empty(len(order), np.int32)
    rank[order] = np.arange(len(order), dtype=np.int32)
    return rank


def make_key(match_count: int, tiebreak: int) -> int:
    return 0 if match_count <= 0 else (int(match_count) << 32) | int(tiebreak)


def decode_key(key: int):
    """-> (found, match_count, tiebreak)"""
    key = int(key) & (2**64 - 1)
    return key != 0, key >> 32, key & 0xFFFFFFFF


def combine(keys, dist=None, group=None):
    """In-place all_reduce(MAX) of an int64 key tensor (no-op without a process group)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group)
    return keys


def query_share(nq: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [begin, end) of the queries this rank fingerprints (equal shares: nq % world == 0)."""
    if nq % world:
        raise ValueError("query batch of %d does not split evenly over %d ranks" % (nq, world))
    per = nq // world
    return rank * per, (rank + 1) * per


def all_gather_rows(out, mine, dist, group=None):
    """out[world, ...] <- every rank's `mine` (RCCL all_gather_into_tensor; gloo via a list)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, mine, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), mine, group=group)
    return out


class QueryShardedSearch:
    """configs[3] step on rank r of N: fingerprint queries [r·nq/N, (r+1)·nq/N) of equal-length
    queries (tfp_fingerprint_device -> their q values), all_gather the q values, search the whole
    batch against this rank's clips (tfp_search_q_device), all_reduce(MAX) the keys."""

    def __init__(self, eng, torch, dev, dist, nq: int, samples_per_query: int, sample_rate: int = 8000):
        import numpy as _np
        self.eng, self.dist = eng, dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.b, self.e = query_share(nq, self.world, self.rank)
        per = self.e - self.b
        self.nfq = (samples_per_query + 255) // 256
        self.plan = eng.plan(_np.arange(per + 1, dtype=_np.int64) * samples_per_query, sample_rate)
        self.qall = torch.empty((self.world, per * self.nfq, 2), dtype=torch.float64, device=dev)
        self.qmine = torch.empty((per * self.nfq, 2), dtype=torch.float64, device=dev)
        self.micro = torch.empty((per * self.nfq, 2), dtype=torch.int32, device=dev)
        self.qoff = _np.arange(nq + 1, dtype=_np.int64) * self.nfq
        self.qn = samples_per_query

    def __call__(self, d_pcm_all: int, p, keys, stream: int):
        """d_pcm_all: device int16 [nq, samples_per_query] (this rank reads its share only);
        keys: int64 device tensor [nq], the global winners on return (stream-ordered)."""
        d_mine = d_pcm_all + 2 * self.b * self.qn
        self.eng.fingerprint_device(self.plan, d_mine, self.micro.data_ptr(), self.qmine.data_ptr(), stream)
        all_gather_rows(self.qall, self.qmine, self.dist)
        self.eng.search_q_device(self.qall.data_ptr(), self.qoff, p, keys.data_ptr(), stream)
        return combine(keys, self.dist)
