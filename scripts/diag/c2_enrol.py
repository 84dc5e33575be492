"""Diagnostic (not a test): the bench's coefs2_cache after_enrol leg alone, for a kernel trace. The
100k-clip DB, both tolerances' caches warm, then N rounds of (tfp_index_add of one 30 s clip, one
batch-1 coefs = 2 search from host PCM) at tol 0.001 / 0.45 in turn, each round timed on the host;
the clips are removed at the end. Args: rounds [tol ...] (default 8, 0.001 0.45)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import tiresias_amd as T  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
tols = [float(x) for x in sys.argv[2:]] or [0.001, 0.45]
dev = torch.device("cuda", 0)
sh = torch.cuda.current_stream().cuda_stream
eng = T.Engine(0)
bench.enroll(eng, torch, dev, sh, list(range(100_000)))
eng.index_commit()
qn = 8000 * 5
hq = [T.synth_pcm(bench.SEED_DB, [i], qn)[0] for i in range(4)]
ps = [T.params(2, t) for t in tols]
for i in range(2 * len(ps)):
    eng.search_pcm_batch(hq[i % len(hq)], [0, qn], ps[i % len(ps)])
n_db = 8000 * 30
nf_db = (n_db + bench.HOP - 1) // bench.HOP
pcm = np.random.default_rng(0x7153C4).integers(-32768, 32768, (rounds, n_db)).astype(np.int16)
fr = eng.fingerprint_batch(pcm.reshape(-1), np.arange(rounds + 1) * n_db)
uuids = ["fffffffe-ffff-4fff-bfff-%012x" % i for i in range(rounds)]
for i, u in enumerate(uuids):
    t0 = time.perf_counter()
    eng.index_add(u, fr["m1"][i * nf_db:(i + 1) * nf_db], fr["m2"][i * nf_db:(i + 1) * nf_db])
    t1 = time.perf_counter()
    eng.search_pcm_batch(hq[i % len(hq)], [0, qn], ps[i % len(ps)])
    t2 = time.perf_counter()
    print("round %d tol %g: add %.3f ms, search %.3f ms, total %.3f ms" %
          (i, tols[i % len(tols)], (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t2 - t0) * 1e3), flush=True)
print("cache", eng.index_cache_stats(), flush=True)
for u in uuids:
    eng.index_remove(u)
eng.index_commit()
eng.close()
