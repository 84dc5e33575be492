"""Diagnostic (not a test): batch-1 search latency through a device group vs one engine, on this
box's one GPU (every shard on device 0), over a 20k-clip DB split across the shards."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import tiresias_amd as T  # noqa: E402

SEED_DB = 0x7153A1
nclips, n = 20000, 8000 * 30
nf = (n + 255) // 256
e0 = T.Engine(0)
uu, m1s, m2s = [], [], []
for b in range(0, nclips, 1000):
    pcm = T.synth_pcm(SEED_DB, range(b, b + 1000), n)
    fr = e0.fingerprint_batch(pcm.reshape(-1), np.arange(1001) * n)
    m1s.append(fr["m1"]); m2s.append(fr["m2"])
    uu += ["%08x-0000-4000-8000-%012x" % (c, c) for c in range(b, b + 1000)]
m1, m2 = np.concatenate(m1s), np.concatenate(m2s)
fo = np.arange(nclips + 1) * nf
qn = 8000 * 5
qs = [np.ascontiguousarray(T.synth_pcm(SEED_DB, [c], qn, offsets=[256 * 100])[0]) for c in range(0, 400, 10)]
p = T.params(1, 0.001)
for shards in (0, 1, 2, 3):
    t = e0 if shards == 0 else T.Group([0] * shards)
    t.index_clear()
    t.index_add_batch(uu, fo, m1, m2)
    t.index_commit()
    for q in qs[:5]:
        t.search_pcm_batch(q, [0, qn], p)
    ts = []
    for r in range(10):
        for q in qs:
            t0 = time.perf_counter()
            t.search_pcm_batch(q, [0, qn], p)
            ts.append((time.perf_counter() - t0) * 1e3)
    print("%s: batch-1 p50 %.4f ms p99 %.4f ms" % ("engine" if shards == 0 else "group x%d" % shards,
                                                  np.percentile(ts, 50), np.percentile(ts, 99)), flush=True)
    if shards:
        t.close()
