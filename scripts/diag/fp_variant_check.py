"""Diagnostic (not a test): one 1,024-clip x 2 s fingerprint launch (16-frame tiles) of the library
TFP_LIB_PATH points at, against the oracle: prints the count of differing rows and the first few
(got vs expected micro-units)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import oracle_py  # noqa: E402
import tiresias_amd as T  # noqa: E402

nclips, n = 1024, 8000 * 2
dev = torch.device("cuda", 0)
s = torch.cuda.Stream()
eng = T.Engine(0)
pcm = torch.empty((nclips, n), dtype=torch.int16, device=dev)
eng.synth_device(0x7153A1, range(nclips), n, pcm.data_ptr(), stream=s.cuda_stream)
off = np.arange(nclips + 1, dtype=np.int64) * n
plan = eng.plan(off)
micro = torch.zeros((plan.nframes, 2), dtype=torch.int32, device=dev)
eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, s.cuda_stream)
s.synchronize()
got = micro.cpu().numpy()
exp, _ = oracle_py.fingerprint_batch(pcm.cpu().numpy().reshape(-1), off, nthreads=16, want_db=False)
bad = np.nonzero((got != exp).any(axis=1))[0]
print("%s: %d of %d rows differ" % (os.path.basename(os.path.dirname(T.LIB_PATH)), len(bad), len(got)))
for i in bad[:6]:
    print("  row %d (clip %d frame %d): got %s exp %s" % (i, i // plan.nframes * nclips, i % (plan.nframes // nclips),
                                                         got[i].tolist(), exp[i].tolist()))
