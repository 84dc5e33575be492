"""Diagnostic (not a test): the fingerprint launch on configs[1]'s batch (1,024 x 30 s clips) and on
configs[2]'s query batch shape (4,096 x 5 s), in one process, alternating, each timed with HIP events
on its stream after a clock warm-up; prints per shape the median ms and ns per frame. With
ENROL=1 the 100k-clip enrolment of c3_sweep.py runs first (the context the C3 batch is timed in).
With GAP_MS > 0 the host sleeps that long between launches (idle time between searches).
Args: [reps]."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "asterisk-tiresias_amd")]
import torch  # noqa: E402
import tiresias_amd as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
gap = float(os.environ.get("GAP_MS", "0")) / 1e3
dev = torch.device("cuda", 0)
s = torch.cuda.Stream()
eng = T.Engine(0)
if os.environ.get("ENROL") == "1":
    import bench
    bench.enroll(eng, torch, dev, s.cuda_stream, list(range(100_000)))
    eng.index_commit()
shapes = {}
for tag, nclips, n in (("C2", 1024, 240000), ("C3q", 4096, 40000)):
    pcm = torch.empty((nclips, n), dtype=torch.int16, device=dev)
    eng.synth_device(0x7153A1 if tag == "C2" else 0x7153B2, range(nclips), n, pcm.data_ptr(), stream=s.cuda_stream)
    plan = eng.plan(np.arange(nclips + 1, dtype=np.int64) * n)
    micro = torch.empty((plan.nframes, 2), dtype=torch.int32, device=dev)
    shapes[tag] = (pcm, plan, micro)
t_end = time.perf_counter() + 0.5  # clock warm-up
while time.perf_counter() < t_end:
    for tag, (pcm, plan, micro) in shapes.items():
        eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, s.cuda_stream)
    torch.cuda.synchronize()
ts = {k: [] for k in shapes}
for _ in range(reps):
    for tag, (pcm, plan, micro) in shapes.items():
        if gap:
            time.sleep(gap)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, s.cuda_stream)
        b.record(s)
        b.synchronize()
        ts[tag].append(a.elapsed_time(b))
for tag, (pcm, plan, micro) in shapes.items():
    m = float(np.median(ts[tag]))
    print("%s enrol=%s gap=%g: %d frames, median %.4f ms (min %.4f), %.4f ns/frame" %
          (tag, os.environ.get("ENROL", "0"), gap * 1e3, plan.nframes, m, float(np.min(ts[tag])), m * 1e6 / plan.nframes),
          flush=True)
