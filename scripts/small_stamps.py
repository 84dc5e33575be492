"""Phase stamps of the batch-1 fingerprint launch (build with EXTRA=-DTFP_STAMPS): a 2,000-clip
index, one 5 s query searched a few times; the kernel prints s_memtime deltas from block 0."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "asterisk-tiresias_amd"))
import tiresias_amd as T  # noqa: E402

eng = T.Engine(0)
n = 8000 * 30
for c in range(0, 2000, 500):
    pcm = T.synth_pcm(1234, range(c, c + 500), n)
    micro = eng.fingerprint_batch(pcm.reshape(-1), np.arange(501) * n)
    nf = (n + 255) // 256
    eng.index_add_batch([f"00000000-0000-4000-8000-{i:012d}" for i in range(c, c + 500)], np.arange(501) * nf,
                        micro["m1"], micro["m2"])
q = T.synth_pcm(1234, [7], 8000 * 5)[0]
for _ in range(4):
    r, fc = eng.search_pcm_batch(q, [0, len(q)], T.params(1, 0.001))
print("result", r[0] and r[0]["match_count"], fc, flush=True)
eng.close()
