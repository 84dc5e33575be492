"""Diagnostic (not a test): the bench's coefs2_cache alternation leg alone (batch-1 coefs = 2 from host
PCM on the 100k-clip DB, tolerances given in turn), p50 / p99 over N calls after 4 untimed ones.
The library is TFP_LIB_PATH's (A/B builds) or the in-tree one. Args: N tol... (default 200 0.001 0.45)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import tiresias_amd as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
tols = [float(x) for x in sys.argv[2:]] or [0.001, 0.45]
dev = torch.device("cuda", 0)
sh = torch.cuda.current_stream().cuda_stream
eng = T.Engine(0)
bench.enroll(eng, torch, dev, sh, list(range(100_000)))
eng.index_commit()
qn = 8000 * 5
hq = [T.synth_pcm(bench.SEED_DB, [i], qn)[0] for i in range(4)]
ps = [T.params(2, t) for t in tols]
for i in range(4):
    eng.search_pcm_batch(hq[i % len(hq)], [0, qn], ps[i % len(ps)])
lat = [[] for _ in ps]
for i in range(n):
    t0 = time.perf_counter()
    eng.search_pcm_batch(hq[i % len(hq)], [0, qn], ps[i % len(ps)])
    lat[i % len(ps)].append((time.perf_counter() - t0) * 1e3)
tag = os.environ.get("TAG", "")
for t, x in zip(tols, lat):
    print("%s batch-1 coefs 2 tol %g: p50 %.3f p99 %.3f ms" % (tag, t, np.percentile(x, 50), np.percentile(x, 99)), flush=True)
eng.close()
