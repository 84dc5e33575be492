"""Diagnostic (not a test): the first batch-1 coefs = 2 search at tolerances not used before on the
100k-clip DB (each call builds that tolerance's clip-set cache from the clip order inside the call;
the first call also sorts the order), host-timed, for a kernel trace of the cache builds.
Args: tol ... (default 0.001 0.01 0.1 0.45 0.002 0.3)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import tiresias_amd as T  # noqa: E402

tols = [float(x) for x in sys.argv[1:]] or [0.001, 0.01, 0.1, 0.45, 0.002, 0.3]
dev = torch.device("cuda", 0)
sh = torch.cuda.current_stream().cuda_stream
eng = T.Engine(0)
bench.enroll(eng, torch, dev, sh, list(range(100_000)))
eng.index_commit()
qn = 8000 * 5
hq = T.synth_pcm(bench.SEED_DB, [3], qn)[0]
eng.search_pcm_batch(hq, [0, qn], T.params(1, 0.001))  # (coefs = 1 warm-up: ranges, bitsets)
for t in tols:
    t0 = time.perf_counter()
    eng.search_pcm_batch(hq, [0, qn], T.params(2, t))
    t1 = time.perf_counter()
    eng.search_pcm_batch(hq, [0, qn], T.params(2, t))
    t2 = time.perf_counter()
    print("tol %g: first search %.3f ms (cache built), second %.3f ms" % (t, (t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)
print("cache", eng.index_cache_stats(), flush=True)
eng.close()
