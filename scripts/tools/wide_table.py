"""Per-kernel table of the coefs=2 C3 batch from a rocprofv3 kernel trace of scripts/diag/c3_sweep.py:
each batch runs from its query fingerprint launch (fingerprint8k_kernel<4>) to wide_part_max; the last
N batches are averaged kernel by kernel (position in the batch, name, mean duration), with the batch's
span (first start to last end) and the kernels' sum.

usage: python scripts/tools/wide_table.py TRACE.csv N OUT.json [NOTE]"""
import csv
import json
import sys

trace, nlast, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
note = sys.argv[4] if len(sys.argv) > 4 else ""
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
batches, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if "fingerprint8k_kernel<4>" in name:
        cur = []
    if cur is None:
        continue
    cur.append((name.replace("tfp::(anonymous namespace)::", "").replace("tfp::", "").split("(")[0],
                int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if "wide_part_max" in name:
        batches.append(cur)
        cur = None
batches = batches[-nlast:]
shape = [k[0] for k in batches[0]]
assert all([k[0] for k in b] == shape for b in batches), "batches differ in their kernels"
table = []
for i, name in enumerate(shape):
    ds = [(b[i][2] - b[i][1]) / 1e3 for b in batches]
    table.append({"kernel": name, "mean_us": round(sum(ds) / len(ds), 2)})
spans = [(b[-1][2] - b[0][1]) / 1e3 for b in batches]
res = {"trace": trace, "batches": len(batches), "note": note,
       "span_us_mean": round(sum(spans) / len(spans), 1),
       "kernels_sum_us": round(sum(t["mean_us"] for t in table), 1), "kernels": table}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))
for t in table:
    print(f"{t['mean_us']:9.1f}  {t['kernel']}")
