"""Per-step durations of the C2 fingerprint launches from a rocprofv3 kernel trace.

The bench's first fingerprint dispatches are the configs[1] batch: `warmup` untimed then `steps`
timed launches, all with the C2 grid (later dispatches are DB-build / query batches). At 8 kHz a
step is fingerprint8k_kernel followed by finish_db_kernel (dB and "%f" of the stored
coefficients); bench.py's HIP events bracket both, so a step's time here is from the fingerprint
kernel's start to the finish kernel's end (kernel and finish durations are also listed).
Usage: python scripts/tools/c2_dispatches.py TRACE.csv WARMUP STEPS OUT.csv"""
import csv
import re
import sys

trace, warm, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
allk = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
steps_rows = []
for i, r in enumerate(allk):
    if not re.search(r"fingerprint(8k)?_kernel", r["Kernel_Name"]):
        continue
    fin = allk[i + 1] if i + 1 < len(allk) and "finish_db_kernel" in allk[i + 1]["Kernel_Name"] else None
    steps_rows.append((r, fin))
    if len(steps_rows) == warm + steps:
        break


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6


with open(out, "w") as f:
    f.write("dispatch,step_ms,fingerprint_kernel_ms,finish_kernel_ms,timed\n")
    for i, (r, fin) in enumerate(steps_rows):
        end = int((fin or r)["End_Timestamp"])
        step = (end - int(r["Start_Timestamp"])) / 1e6
        f.write("%d,%.6f,%.6f,%.6f,%d\n" % (i, step, dur(r), dur(fin) if fin else 0.0, int(i >= warm)))
timed = steps_rows[warm:]
n = max(1, len(timed))
mean_step = sum((int((fin or r)["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r, fin in timed) / n
mean_k = sum(dur(r) for r, _ in timed) / n
print("timed C2 steps: %d, mean %.4f ms (fingerprint kernel %.4f ms)" % (len(timed), mean_step, mean_k))
