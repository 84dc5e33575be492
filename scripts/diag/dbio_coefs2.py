"""Diagnostic (not a test): the test_dbio coefs=2 tol 0.5 case, piece by piece."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "asterisk-tiresias_amd"), os.path.join(REPO, "oracle")]
import oracle_py as oracle  # noqa: E402
import tiresias_amd._lib as L  # noqa: E402
if os.environ.get("TFP_LIB"):
    L.LIB_PATH = os.environ["TFP_LIB"]
    for k in [k for k in L._SIGS if k.startswith("tfp_group") or k == "tfp_index_build_stats"]:
        del L._SIGS[k]
import tiresias_amd as T  # noqa: E402
print("lib", L.LIB_PATH)

nclips, n = 12, 8000 * 4
pcm = T.synth_pcm(0x5EED, range(nclips), n)
micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n, nthreads=4, want_db=False)
nf = (n + 255) // 256
uu = ["%08x-0000-4000-8000-%012d" % (c * 7919, c) for c in range(nclips)]
e = T.Engine(0)
e.index_add_batch(uu, np.arange(nclips + 1) * nf, micro[:, 0], micro[:, 1])
q = pcm[3][4096:4096 + 16000]
_, qdb, _ = oracle.fingerprint(q)
fr = e.fingerprint(q)
print("engine q == oracle q:", np.array_equal(fr["q1"].view(np.uint64), qdb[:, 0].view(np.uint64)),
      np.array_equal(fr["q2"].view(np.uint64), qdb[:, 1].view(np.uint64)))
clip = np.repeat(np.arange(nclips), nf)
for coefs, tol in ((1, 0.001), (2, 0.5), (2, 0.001), (1, 0.5)):
    p = T.params(coefs, tol)
    found, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], clip, uu, qdb[:, 0], qdb[:, 1], coefs, tol, -1, -1)
    frames = np.zeros(len(qdb), T.FRAME_DTYPE)
    frames["q1"], frames["q2"] = qdb[:, 0], qdb[:, 1]
    r1, _ = e.search_batch(frames, [0, len(frames)], p)
    r2, _ = e.search_pcm_batch(q, [0, len(q)], p)
    r3, _ = e.search_batch(np.concatenate([frames] * 3), [0, len(frames), 2 * len(frames), 3 * len(frames)], p) \
        if hasattr(L, "LIB_PATH") else (None,)
    print(coefs, tol, "oracle", (uu[w], mc) if found else None, "frames", r1[0] and (r1[0]["audio_uuid"], r1[0]["match_count"]),
          "pcm", r2[0] and (r2[0]["audio_uuid"], r2[0]["match_count"]),
          "x3", [r and (r["audio_uuid"], r["match_count"]) for r in r3])
