"""Per-kernel averages of rocprofv3 --pmc passes (any kernels): for each kernel name, each counter's
value per dispatch (summed over its instances), averaged over the dispatches, plus per-wave
instruction counts and the SQ cycle split when the counters are there.

usage: python scripts/tools/pmc_kernels.py DIR [DIR ...]   (each DIR holds run_counter_collection.csv)"""
import collections
import csv
import glob
import json
import os
import re
import sys

per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")).replace("tfp::", "")
            per[k][r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
out = {}
for k, cs in per.items():
    m = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    o = {"per_dispatch": m}
    if m.get("SQ_WAVES"):
        o["per_wave"] = {c: m[c] / m["SQ_WAVES"] for c in m if c.startswith("SQ_INSTS")}
    if m.get("SQ_WAVE_CYCLES"):
        o["wave_cycle_split"] = {c: m[c] / m["SQ_WAVE_CYCLES"] for c in m
                                 if c.startswith("SQ_ACTIVE") or c.startswith("SQ_WAIT")}
    out[k] = o
json.dump(out, sys.stdout, indent=1)
