"""Batch-1 search latency probe: a DB of --db-clips synthetic 30 s clips, then --n single 5 s
queries from host PCM (tfp_search_pcm_batch, as bench.py's latency leg). Prints p50/p99 ms.
Run under `rocprofv3 --hip-trace --kernel-trace --stats` to see where the time goes."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "asterisk-tiresias_amd"))
import tiresias_amd as T  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--db-clips", type=int, default=20000)
ap.add_argument("--n", type=int, default=200)
a = ap.parse_args()
import torch  # noqa: E402  (device buffers for the DB build only)
eng = T.Engine(0)
dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
sh = stream.cuda_stream
n_db, qn = 240000, 40000
nf_db = (n_db + 255) // 256
chunk = 1024
buf = torch.empty((chunk, n_db), dtype=torch.int16, device=dev)
micro = torch.empty((chunk * nf_db, 2), dtype=torch.int32, device=dev)
for s in range(0, a.db_clips, chunk):
    ids = list(range(s, min(a.db_clips, s + chunk)))
    k = len(ids)
    plan = eng.plan(np.arange(k + 1, dtype=np.int64) * n_db)
    eng.synth_device(0x7153A1, ids, n_db, buf.data_ptr(), stream=sh)
    eng.fingerprint_device(plan, buf.data_ptr(), micro.data_ptr(), 0, sh)
    eng.index_add_device(["%08x-0000-4000-8000-%012x" % (g, g) for g in ids], np.arange(k + 1, dtype=np.int64) * nf_db,
                         micro.data_ptr(), sh)
eng.index_commit()
torch.cuda.synchronize(dev)
rng = np.random.default_rng(5)
qs = [T.synth_pcm(0x7153A1, [int(rng.integers(a.db_clips))], qn, offsets=[256 * int(rng.integers(0, 700))])[0] for _ in range(32)]
p = T.params(1, 0.001)
for q in qs[:4]:
    eng.search_pcm_batch(q, [0, qn], p)
for mode in ("0", "1"):  # TFP_SMALL_SYNC: 0 = spin on the published result, 1 = stream sync
    os.environ["TFP_SMALL_SYNC"] = mode
    lat = []
    for i in range(a.n):
        q = qs[i % len(qs)]
        t0 = time.perf_counter()
        res, fc = eng.search_pcm_batch(q, [0, qn], p)
        lat.append((time.perf_counter() - t0) * 1e3)
    print("TFP_SMALL_SYNC=%s batch-1 latency p50 %.3f ms p99 %.3f ms (n=%d, db %d clips)"
          % (mode, np.percentile(lat, 50), np.percentile(lat, 99), a.n, a.db_clips))
