"""Per-dispatch durations of the C2 fingerprint launches from a rocprofv3 kernel trace.

The bench's first fingerprint_kernel dispatches are the configs[1] batch: `warmup` untimed then
`steps` timed launches, all with the C2 grid (later dispatches are DB-build / query batches).
Usage: python scripts/tools/c2_dispatches.py TRACE.csv WARMUP STEPS OUT.csv"""
import csv
import re
import sys

trace, warm, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
rows = [r for r in csv.DictReader(open(trace)) if re.search(r"fingerprint(8k)?_kernel", r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[: warm + steps]
with open(out, "w") as f:
    f.write("dispatch,duration_ms,timed\n")
    for i, r in enumerate(rows):
        f.write("%d,%.6f,%d\n" % (i, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, int(i >= warm)))
timed = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[warm:]]
print("timed C2 dispatches: %d, mean %.4f ms" % (len(timed), sum(timed) / max(1, len(timed))))
