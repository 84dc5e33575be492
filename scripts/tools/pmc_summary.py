"""Per-launch / per-frame summary of rocprofv3 --pmc passes of the C2 fingerprint launch.

Usage: python scripts/tools/pmc_summary.py DIR [DIR ...]  (each DIR a gpurun_out/<tag>/pN with
run_counter_collection.csv). Picks the fingerprint kernel dispatches of the largest grid (the C2
launch), averages each counter over them (summed over the counter's instances per dispatch), and
prints per-launch totals, per-frame instruction counts and the SQ cycle split.
FRAMES (default 960512, the C2 launch) and LAST (only the last LAST such dispatches of each pass,
e.g. the C3 query launches after a DB enrolment of the same grid) from the environment."""
import collections
import csv
import glob
import json
import os
import re
import sys

FRAMES = int(os.environ.get("FRAMES", "960512"))
LAST = int(os.environ.get("LAST", "0"))
vals = collections.defaultdict(list)
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(path)) if re.search(r"fingerprint(8k)?_kernel", r["Kernel_Name"])]
        grid = max(int(r["Grid_Size"]) for r in rows)
        keep = sorted({int(r["Dispatch_Id"]) for r in rows if int(r["Grid_Size"]) == grid})
        keep = set(keep[-LAST:] if LAST else keep)
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in rows:
            if int(r["Dispatch_Id"]) in keep:
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for c, dd in per.items():
            vals[c].append(sum(dd.values()) / len(dd))
m = {c: sum(v) / len(v) for c, v in vals.items()}
out = {"per_launch": m, "per_frame": {}}
for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH"):
    if c in m:
        out["per_frame"][c] = m[c] / FRAMES
if "SQ_WAVE_CYCLES" in m:
    wc = m["SQ_WAVE_CYCLES"]
    out["wave_cycle_split"] = {k: m[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS")
                               if k in m}
if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
    out["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
if "GRBM_GUI_ACTIVE" in m and "SQ_BUSY_CYCLES" in m:
    out["grbm_gui_active"] = m["GRBM_GUI_ACTIVE"]
print(json.dumps(out, indent=1))
