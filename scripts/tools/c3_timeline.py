"""Kernel timeline of the configs[2] match batches in a rocprofv3 kernel trace: every kernel from
each large query-fingerprint launch to the next vote_gemm, with start offsets and durations (us).
Usage: python scripts/tools/c3_timeline.py TRACE.csv [MIN_FP_US]"""
import csv
import sys

trace = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
for i, r in enumerate(rows):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "fingerprint8k_kernel<4>" not in r["Kernel_Name"] or d < min_us:
        continue
    j = i
    while j < len(rows) and "vote_gemm" not in rows[j]["Kernel_Name"]:
        j += 1
    if j == len(rows):
        continue
    t0 = int(rows[max(0, i - 2)]["Start_Timestamp"])
    for r2 in rows[max(0, i - 2): j + 3]:
        s, e = int(r2["Start_Timestamp"]), int(r2["End_Timestamp"])
        print("%9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, r2["Kernel_Name"][:72]))
    print()
