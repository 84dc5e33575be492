"""Where a small fingerprint launch's time goes (build with EXTRA=-DTFP8_TIMING=1): one 5 s query
(157 frames, 40 four-frame tiles) through tfp_fingerprint_batch, then each wave's s_memtime stamps
at the kernel's 8 points, as medians over waves of the deltas from the wave's entry stamp."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "asterisk-tiresias_amd"))
import tiresias_amd as T  # noqa: E402
from tiresias_amd._lib import lib  # noqa: E402

eng = T.Engine(0)
q = T.synth_pcm(0x7153B2, [3], 40000)[0]
for _ in range(50):
    eng.fingerprint_batch(q, [0, len(q)])
buf = (C.c_ulonglong * (64 * 8))()
assert lib().tfp_debug_fp_timing(buf) == 0
t = np.array(buf, dtype=np.uint64).reshape(64, 8).astype(np.int64)[:40]
d = t - t[:, :1]
names = ["entry", "tile+pcm issued", "tables staged", "pcm in LDS", "fft done", "split done", "mel+logs done", "tail done"]
for i, n in enumerate(names):
    print("%-16s median %8.0f  min %8.0f  max %8.0f" % (n, np.median(d[:, i]), d[:, i].min(), d[:, i].max()))
print("per-step medians:", [int(np.median(d[:, i + 1] - d[:, i])) for i in range(7)])
