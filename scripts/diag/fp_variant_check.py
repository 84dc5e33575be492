"""Diagnostic (not a test): one 1,024-clip x 2 s fingerprint launch (16-frame tiles) of the library
TFP_LIB_PATH points at, against the oracle: prints the count of differing rows and the first few
(got vs expected micro-units). Then 400 clips of random lengths (odd and even, 1 to 9,000 samples)
back to back in one buffer, so clips start on odd samples too."""
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

# ragged: random lengths back to back (odd starts, odd lengths, clips shorter than a tile)
rng = np.random.default_rng(7)
lens = rng.integers(1, 9000, 400)
lens[:8] = [1, 2, 255, 256, 257, 511, 512, 513]
off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
host = rng.integers(-32768, 32768, int(off[-1])).astype(np.int16)
d_pcm = torch.from_numpy(host).to(dev)
plan = eng.plan(off)
micro = torch.zeros((max(plan.nframes, 1), 2), dtype=torch.int32, device=dev)
eng.fingerprint_device(plan, d_pcm.data_ptr(), micro.data_ptr(), 0, s.cuda_stream)
s.synchronize()
got = micro.cpu().numpy()[:plan.nframes]
exp, _ = oracle_py.fingerprint_batch(host, off, nthreads=16, want_db=False)
bad = np.nonzero((got != exp).any(axis=1))[0]
print("%s ragged: %d of %d rows differ" % (os.path.basename(os.path.dirname(T.LIB_PATH)), len(bad), len(got)))
