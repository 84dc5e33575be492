"""Diagnostic (not a test): configs[2]'s 100k-clip DB and bench.c3_queries' batch, one search setting
timed K times (for rocprofv3 kernel traces of the general path). Args: coefs tol [reps]."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import tiresias_amd as T  # noqa: E402

coefs, tol = int(sys.argv[1]), float(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
sh = torch.cuda.current_stream().cuda_stream
eng = T.Engine(0)
bench.enroll(eng, torch, dev, sh, list(range(100_000)))
eng.index_commit()
nq, qn = 4096, 8000 * 5
qpcm = bench.c3_queries(eng, torch, dev, sh, nq, 100_000)
plan = eng.plan(np.arange(nq + 1, dtype=np.int64) * qn)
keys = torch.zeros(nq, dtype=torch.int64, device=dev)
p = T.params(coefs, tol)
for _ in range(2):
    eng.search_device(plan, qpcm.data_ptr(), p, keys.data_ptr(), sh)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    eng.search_device(plan, qpcm.data_ptr(), p, keys.data_ptr(), sh)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print("coefs %d tol %g: median %.3f ms, found %d" % (coefs, tol, float(np.median(ts)),
                                                     int((keys.cpu().numpy() != 0).sum())), flush=True)
