"""Clip-sharded search across GPUs: the multi-GPU protocol.

The enrolled DB is split by clip — never inside a clip, because the per-frame
`GROUP BY audio_uuid` dedup of fp_handler.c:353 is not additive across a split clip. Every
rank searches the same queries against its own clips and reduces each query to one 64-bit key

    key = match_count << 32 | global_uuid_rank      (0 = no hit on this rank)

ordered exactly like the reference's final sort (count(*) DESC, ties -> greatest audio_uuid,
fp_handler.c:367). One all_reduce(MAX) of the keys over RCCL (backend "nccl") gives every
rank the global winner; nothing else crosses ranks.
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
