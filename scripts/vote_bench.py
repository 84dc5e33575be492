"""Vote-path timing at configs[2] scale with a controllable number of used keys (the bench's
synthetic audio uses only 3): 100k clips x 938 rows with max1 uniform over [-S-0.5, S+0.5], so
each tol=0.001 box holds 0.2 % of its key's rows, and 4096 queries x 157 frames with keys in
[-S, S]. Times tfp_search_batch (host
frames in, results out) per path: TFP_VOTE_CLASS_MAX=-1 (GEMM) and the default (pattern classes
when Ku <= 10). Run under rocprofv3 --kernel-trace for per-kernel times.
Usage: python scripts/vote_bench.py [SPREAD ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "asterisk-tiresias_amd"))
from tiresias_amd.engine import Engine, params  # noqa: E402


def main():
    spreads = [int(a) for a in sys.argv[1:]] or [1, 5, 40, 300]
    rng = np.random.default_rng(1)
    nclips, rows, nq, qf = 100000, 938, 4096, 157
    with Engine(0) as eng:
        for spread in spreads:
            eng.index_clear()
            uu = [f"{i:08x}-0000-4000-8000-000000000000" for i in range(nclips)]
            k = rng.integers(-spread, spread + 1, nclips * rows)
            m1 = (k * 1000000 + rng.integers(-500000, 500000, nclips * rows)).astype(np.int32)
            m2 = np.zeros(nclips * rows, np.int32)
            eng.index_add_batch(uu, np.arange(nclips + 1, dtype=np.int64) * rows, m1, m2)
            eng.index_commit()
            fr = np.zeros(nq * qf, np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                                             ("q1", "<f8"), ("q2", "<f8")]))
            kq = rng.integers(-spread, spread + 1, nq * qf)
            fr["q1"] = kq + 0.25 * np.where(kq >= 0, 1, -1)
            qoff = np.arange(nq + 1, dtype=np.int64) * qf
            p = params(1, 0.001)
            for cm in ("-1", "10"):
                os.environ["TFP_VOTE_CLASS_MAX"] = cm
                for _ in range(3):
                    eng.search_batch(fr, qoff, p)
                ts = []
                for _ in range(10):
                    t0 = time.perf_counter()
                    res, _ = eng.search_batch(fr, qoff, p)
                    ts.append(time.perf_counter() - t0)
                found = sum(r is not None for r in res)
                print(f"spread {spread} class_max {cm}: median {np.median(ts) * 1e3:.3f} ms, found {found}", flush=True)
            del os.environ["TFP_VOTE_CLASS_MAX"]


if __name__ == "__main__":
    main()
