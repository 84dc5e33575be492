"""Diagnostic (not a test): configs[1]'s fingerprint launch (1,024 x 30 s clips in HBM), timed with
HIP events over K launches after a clock warm-up; prints the median ms. Environment knobs of the
engine (TFP_FP_BLOCKS_PER_CU, TFP_LIB_PATH) select the variant; FP_CLIPS / FP_SECONDS another batch
shape (4096 / 5: configs[2]'s query batch). Args: [reps]."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import tiresias_amd as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
s = torch.cuda.Stream()  # a real stream: the null stream's handle (0) would send the launches to the engine's own
eng = T.Engine(0)
nclips, n = int(os.environ.get("FP_CLIPS", 1024)), 8000 * int(os.environ.get("FP_SECONDS", 30))
tag = "C2" if (nclips, n) == (1024, 240000) else "%dx%ds" % (nclips, n // 8000)
pcm = torch.empty((nclips, n), dtype=torch.int16, device=dev)
eng.synth_device(0x7153A1, range(nclips), n, pcm.data_ptr(), stream=s.cuda_stream)
plan = eng.plan(np.arange(nclips + 1, dtype=np.int64) * n)
micro = torch.empty((plan.nframes, 2), dtype=torch.int32, device=dev)
for _ in range(300):  # clock warm-up
    eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, s.cuda_stream)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, s.cuda_stream)
    b.record(s)
    b.synchronize()
    ts.append(a.elapsed_time(b))
print("fp " + tag + " [%s %s]: median %.4f ms (min %.4f)" % (os.environ.get("TFP_FP_BLOCKS_PER_CU", "default"), os.path.basename(os.path.dirname(T.LIB_PATH)), float(np.median(ts)),
                                                float(np.min(ts))), flush=True)
