"""Per-search summary of the coefs=2 general path at C3 (scripts/diag/c3_sweep.py under rocprofv3):
the kernel-trace stats of the search's kernels, and HBM bytes per kernel per search from the
FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE x2 per MI355X_MICROARCH.md's gfx950 correction for
16-B/lane reads: an upper estimate for the kernels whose reads are narrower).

usage: python scripts/tools/wide_summary.py TRACE_DIR TRACE_SEARCHES PMC_FETCH_DIR PMC_WRITE_DIR PMC_SEARCHES
(searches = c3_sweep's 2 warm-up calls + its reps)."""
import collections
import csv
import glob
import json
import os
import re
import sys

trace, nt, fdir, wdir, npm = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5])
SEARCH = re.compile(r"wide_|prep_boxes|radix|onesweep|DeviceRadix|scan|key_ranges|cell|fingerprint8k_kernel<1>|"
                    r"fingerprint8k_kernel<4>|finish_db|scan_")


def short(n):
    n = n.replace("tfp::(anonymous namespace)::", "").replace("tfp::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)


stats = {}
for path in glob.glob(os.path.join(trace, "**", "*kernel_trace.csv"), recursive=True):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, v in per.items():
        if k.startswith("wide_") or k.startswith("prep_boxes"):
            stats[k] = {"calls_per_search": len(v) / nt, "ms_per_search": sum(v) / 1e6 / nt, "avg_us": sum(v) / len(v) / 1e3}


def bytes_of(d, counter):
    out = collections.defaultdict(float)
    for path in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                out[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024.0
    return {k: v / npm for k, v in out.items()}


fb, wb = bytes_of(fdir, "FETCH_SIZE"), bytes_of(wdir, "WRITE_SIZE")
for k in sorted(set(fb) | set(wb)):
    s = stats.setdefault(k, {})
    s["fetch_bytes_raw"] = fb.get(k, 0.0)
    s["hbm_bytes"] = 2 * fb.get(k, 0.0) + wb.get(k, 0.0)
    if s.get("ms_per_search"):
        s["hbm_GBps"] = s["hbm_bytes"] / (s["ms_per_search"] * 1e-3) / 1e9
tot_ms = sum(s.get("ms_per_search", 0.0) for s in stats.values())
tot_b = sum(s.get("hbm_bytes", 0.0) for s in stats.values())
print(json.dumps({"workload": "configs[2] DB (100k x 30 s clips, 93.8 M rows), the 4,096-query C3 batch, coefs=2 tol 0.001",
                  "kernels": stats, "wide_kernels_ms_per_search": tot_ms, "wide_kernels_hbm_bytes_per_search": tot_b,
                  "alg_bytes_one_index_pass": 1135889152}, indent=1))
