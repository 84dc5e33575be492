# A/B of compile flags for the batch-1 search path (rebuilt on the box): the small-path parity
# subset, the latency probe (both completion-wait modes), then the probe under a kernel trace with
# each kernel's median duration.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for fl in "$@"; do
  i=$((i+1))
  make -s -C asterisk-tiresias_amd clean && make -s -j16 -C asterisk-tiresias_amd EXTRA="$fl" > /dev/null 2>&1 || exit 3
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "small or golden" > gpurun_out/abl_$i.log 2>&1; rc=$?; echo "[$fl] pytest rc=$rc $(tail -1 gpurun_out/abl_$i.log)"; case $rc in 0) ;; *) exit $rc;; esac
  timeout -k 10 300 python scripts/lat_probe.py --db-clips 100000 --n 1000 > gpurun_out/abl_$i.txt 2>&1; rc=$?; grep latency gpurun_out/abl_$i.txt; case $rc in 0) ;; *) exit $rc;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abl_$i -o run -- python3 scripts/lat_probe.py --db-clips 100000 --n 300 > gpurun_out/abl_${i}_prof.out 2>&1; rc=$?; case $rc in 0) ;; *) exit $rc;; esac
  python3 - gpurun_out/abl_$i/run_kernel_trace.csv "$fl" <<'PY'
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows[-1500:]:
    d[r["Kernel_Name"].split("(")[0][-28:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"[{sys.argv[2]}]", {k: round(sorted(v)[len(v) // 2], 1) for k, v in d.items() if len(v) > 50})
PY
done
