"""Diagnostic (not a test): configs[2]'s 100k-clip DB and bench.c3_queries' batch, several search
settings timed in one process (one enrolment), each setting's calls back to back (a tolerance change
rebuilds the coefs=2 clip-set cache, which is not what these timings are for). Args: reps setting... where a setting is coefs:tol (e.g. 1:0.001 2:0.45). The library is
TFP_LIB_PATH's (A/B builds) or the in-tree one."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import tiresias_amd as T  # noqa: E402

reps = int(sys.argv[1])
settings = [(int(s.split(":")[0]), float(s.split(":")[1])) for s in sys.argv[2:]]
tag = os.environ.get("TAG", "")
dev = torch.device("cuda", 0)
sh = torch.cuda.current_stream().cuda_stream
eng = T.Engine(0)
bench.enroll(eng, torch, dev, sh, list(range(100_000)))
eng.index_commit()
nq, qn = 4096, 8000 * 5
qpcm = bench.c3_queries(eng, torch, dev, sh, nq, 100_000)
plan = eng.plan(np.arange(nq + 1, dtype=np.int64) * qn)
keys = torch.zeros(nq, dtype=torch.int64, device=dev)
ps = [T.params(c, t) for c, t in settings]
ts = [[] for _ in ps]
found = [0] * len(ps)
t_end = time.perf_counter() + 0.25  # clock warm-up
while time.perf_counter() < t_end:
    eng.search_device(plan, qpcm.data_ptr(), ps[0], keys.data_ptr(), sh)
    torch.cuda.synchronize()
for i, p in enumerate(ps):
    for _ in range(2):
        eng.search_device(plan, qpcm.data_ptr(), p, keys.data_ptr(), sh)
    torch.cuda.synchronize()
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.search_device(plan, qpcm.data_ptr(), p, keys.data_ptr(), sh)
        torch.cuda.synchronize()
        ts[i].append((time.perf_counter() - t0) * 1e3)
        found[i] = int((keys.cpu().numpy() != 0).sum())
for (c, t), x, f in zip(settings, ts, found):
    print("%s coefs %d tol %g: median %.3f ms, min %.3f, found %d" % (tag, c, t, float(np.median(x)), float(np.min(x)), f),
          flush=True)
