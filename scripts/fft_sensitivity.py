"""How unpinned is the DSP? The canonical pipeline against other valid fp32 operation
orders of the parts a real libaubio build may compute differently (oracle
tfo_fingerprint_batch_variant): the FFT (1 = radix-2 256-point complex FFT + the canonical real split,
2 = radix-2 512-point complex FFT of the real input), the filterbank's and the DCT's summation
order (4 / 8: a vectorised-sgemv row dot, 8 interleaved partial sums combined as a tree, in place of
aubio's sequential fmat_vecmul, src/fp_handler.c:642 -> aubio_mfcc_do), and their combinations; on
configs[1]'s data (1,024 x 30 s synthetic clips, 960,512 frames) and on configs[2]-style searches.

Usage: python scripts/fft_sensitivity.py [--clips 1024] [--out profiles/r03/fft_sensitivity.json]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "asterisk-tiresias_amd"))
import oracle_py  # noqa: E402
import tiresias_amd as T  # noqa: E402

NULL = oracle_py.NULL_MICRO


VARIANTS = {1: "FFT: radix-2 256-point complex FFT + canonical real split",
            2: "FFT: radix-2 512-point complex FFT of the real input",
            4: "filterbank: sgemv-style blocked sum (8 partial sums, tree)",
            8: "DCT: sgemv-style blocked sum (8 partial sums, tree)",
            12: "filterbank + DCT blocked",
            13: "FFT 1 + filterbank + DCT blocked",
            14: "FFT 2 + filterbank + DCT blocked"}


def box_member(m, tol_micro=1000):
    """Would a stored max1 of m micro-units fall in its own integer key's box at tol 0.001?"""
    r = np.round(m / 1e6) * 1e6
    return (m != NULL) & (np.abs(m - r) <= tol_micro)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--db-clips", type=int, default=2000)
    ap.add_argument("--queries", type=int, default=256)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "fft_sensitivity.json"))
    a = ap.parse_args()
    n = 8000 * 30
    t0 = time.time()
    pcm = T.synth_pcm(0x7153A1, range(a.clips), n)
    off = np.arange(a.clips + 1, dtype=np.int64) * n
    base, dbase = oracle_py.fingerprint_batch(pcm.reshape(-1), off, nthreads=a.threads)
    res = {"workload": f"configs[1] data: {a.clips} x 30 s synthetic clips ({len(base)} frames)", "variants": {}}
    for v, name in VARIANTS.items():
        mic, db = oracle_py.fingerprint_batch(pcm.reshape(-1), off, nthreads=a.threads, fft_variant=v)
        d1 = base[:, 0] != mic[:, 0]
        d2 = base[:, 1] != mic[:, 1]
        nullflip = (base == NULL) != (mic == NULL)
        both = (base != NULL) & (mic != NULL)
        delta = np.abs(base.astype(np.int64) - mic.astype(np.int64))[both.all(1)]
        k0 = np.trunc(np.where(np.isfinite(dbase[:, 0]), dbase[:, 0], 0.0))
        k1 = np.trunc(np.where(np.isfinite(db[:, 0]), db[:, 0], 0.0))
        res["variants"][name] = {"variant": v,
            "frames_m1_differs": float(d1.mean()), "frames_m2_differs": float(d2.mean()),
            "frames_any_differs": float((d1 | d2).mean()),
            "null_status_differs": float(nullflip.any(1).mean()),
            "trunc_key_differs": float((k0 != k1).mean()),
            "m1_box_membership_flips_tol_0.001": float((box_member(base[:, 0]) != box_member(mic[:, 0])).mean()),
            "max_abs_delta_micro": [int(delta[:, 0].max()) if len(delta) else 0,
                                    int(delta[:, 1].max()) if len(delta) else 0],
            "p99_abs_delta_micro": [float(np.percentile(delta[:, 0], 99)), float(np.percentile(delta[:, 1], 99))],
        }
        print(name, json.dumps(res["variants"][name]), flush=True)
    # search level: a DB and queries fingerprinted with each variant, the same SQL semantics
    nd, nq, qn = a.db_clips, a.queries, 8000 * 5
    dpcm = pcm[:nd] if nd <= a.clips else T.synth_pcm(0x7153A1, range(nd), n)
    doff = np.arange(nd + 1, dtype=np.int64) * n
    rng = np.random.default_rng(5)
    qs = [T.synth_pcm(0x7153A1, [int(rng.integers(nd))], qn, offsets=[256 * int(rng.integers(0, 700))])[0]
          if i % 4 != 3 else T.synth_pcm(0x7153B2, [i], qn)[0] for i in range(nq)]
    qpcm = np.concatenate(qs)
    qoff = np.arange(nq + 1, dtype=np.int64) * qn
    rank = np.arange(nd, dtype=np.int32)
    out = {}
    for v in (0, *VARIANTS):
        dm, _ = oracle_py.fingerprint_batch(dpcm.reshape(-1), doff, nthreads=a.threads, want_db=False, fft_variant=v)
        _, qdb = oracle_py.fingerprint_batch(qpcm, qoff, nthreads=a.threads, fft_variant=v)
        idx = oracle_py.SortedIndex(dm[:, 0], dm[:, 1], np.repeat(np.arange(nd, dtype=np.int32), len(dm) // nd), rank)
        nfq = len(qdb) // nq
        for coefs, tol in ((1, 0.001), (1, 0.1), (2, 0.01)):
            w, mc = idx.search_batch(qdb[:, 0], qdb[:, 1], np.arange(nq + 1) * nfq, coefs, tol, nthreads=a.threads)
            out.setdefault((coefs, tol), {})[v] = (w, mc)
    res["search"] = {"workload": f"{nq} x 5 s queries (75 % excerpts) vs {nd} x 30 s clips, DB and queries "
                                 f"fingerprinted with each variant (variant numbers as in 'variants')"}
    for (coefs, tol), r in out.items():
        w0, m0 = r[0]
        res["search"][f"coefs={coefs} tol={tol}"] = {
            "found_canonical": int((w0 >= 0).sum()),
            **{f"result_differs_variant{v}": float(((r[v][0] != w0) | (r[v][1] != m0)).mean()) for v in VARIANTS},
            **{f"winner_differs_variant{v}": float((r[v][0] != w0).mean()) for v in VARIANTS}}
    res["seconds"] = time.time() - t0
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res["search"], indent=1))


if __name__ == "__main__":
    main()
