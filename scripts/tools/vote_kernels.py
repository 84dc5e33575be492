"""Per-spread vote kernel times from a rocprofv3 kernel trace of scripts/vote_bench.py: spreads
are separated by the index rebuild (index_gather_kernel); within one, the first half of the
searches forces the GEMM (TFP_VOTE_CLASS_MAX=-1), the second half is the default.
Usage: python scripts/tools/vote_kernels.py TRACE.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
groups, cur = [], None
for r in rows:
    n = r["Kernel_Name"]
    if "index_gather_kernel" in n:
        cur = []
        groups.append(cur)
    elif cur is not None:
        cur.append(r)
names = ["key_mask", "vote_compact", "build_A", "zero_bt", "build_B", "class_max", "vote_gemm", "class_vote"]  # zero_bt / class_max: traces before r02z (folded into build_A / vote_gemm_regs)
for gi, g in enumerate(groups):
    seq = [r for r in g if any(k in r["Kernel_Name"] for k in names)]
    nsearch = sum("key_mask" in r["Kernel_Name"] for r in seq)
    half = nsearch // 2
    for label, lo, hi in (("gemm forced", 0, half), ("default", half, nsearch)):
        acc, cnt, i = collections.defaultdict(float), 0, -1
        for r in seq:
            if "key_mask" in r["Kernel_Name"]:
                i += 1
            if lo <= i < hi:
                k = next(k for k in names if k in r["Kernel_Name"])
                acc[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = hi - lo
        print(f"group {gi} {label:11s}: " + ", ".join(f"{k} {acc[k] / n:.1f}" for k in names) + f"  (us, {n} searches)")
