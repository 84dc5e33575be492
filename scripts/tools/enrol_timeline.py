"""Kernel timeline of scripts/diag/c2_enrol.py under rocprofv3 --kernel-trace: every dispatch after
the added clips' fingerprint launch (fingerprint8k_kernel<4>), as start (us from the first), gap
to the previous dispatch's end, duration and kernel name. usage: enrol_timeline.py trace.csv [n]
(n: dispatches to print, default all)."""
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("tfp::", "")
    return re.sub(r"\(.*", "", n)[-60:]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
lim = int(sys.argv[2]) if len(sys.argv) > 2 else None
fp4 = [i for i, r in enumerate(rows) if "fingerprint8k_kernel<4>" in r["Kernel_Name"]]
seg = rows[fp4[-1] + 1:][:lim]
t0 = int(seg[0]["Start_Timestamp"])
prev = None
print("%9s %8s %8s  %s" % ("start_us", "gap_us", "dur_us", "kernel"))
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%9.1f %8.1f %8.1f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3 if prev else 0.0, (e - s) / 1e3, short(r["Kernel_Name"])))
    prev = e
