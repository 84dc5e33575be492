# A/B of compile flags for the vote GEMM (rebuilt on the box): vote-path parity subset, then
# scripts/vote_bench.py under a kernel trace; prints each vote_gemm kernel's durations.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for fl in "$@"; do
  i=$((i+1))
  make -s -C asterisk-tiresias_amd clean && make -s -j16 -C asterisk-tiresias_amd EXTRA="$fl" > /dev/null 2>&1 || exit 3
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "vote" > gpurun_out/abv_$i.log 2>&1; rc=$?; echo "[$fl] pytest rc=$rc $(tail -1 gpurun_out/abv_$i.log)"; case $rc in 0|1) ;; *) exit $rc;; esac
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abv_$i -o run -- python3 scripts/vote_bench.py ${SPREADS:-1 40} > gpurun_out/abv_$i.out 2>&1; rc=$?; case $rc in 0) ;; *) exit $rc;; esac
  python3 - gpurun_out/abv_$i/run_kernel_trace.csv "$fl" <<'PY'
import collections, csv, sys
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "vote_gemm" in r["Kernel_Name"]:
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if t > 8:
            d[r["Kernel_Name"].split("(")[0][-24:]].append(t)
print(f"[{sys.argv[2]}]", {k: [round(x, 1) for x in sorted(v)[len(v) // 4::max(1, len(v) // 4)]] for k, v in d.items()})
PY
done
