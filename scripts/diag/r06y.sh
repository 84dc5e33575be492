# Round 6: the directory's runs: up to 8 buckets dword by dword, 9-256 by their own lane in 16-byte
# stores, longer by the whole wave: per-phase wave clocks (abv/clk), C3 A/B against the committed
# tree (abv/pre), and both under a kernel trace (the bin sort's duration).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06y
TFP_LIB_PATH=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/clk/libtiresias_fp.so TFP_TEST_KNOBS=1 TFP_DEBUG_BINS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.001 1 > gpurun_out/${R}_bins.log 2>&1 || { tail -20 gpurun_out/${R}_bins.log; exit 3; }
grep -E "bin sort waves|cycles" gpurun_out/${R}_bins.log | tail -6
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in pre new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
for v in pre new; do
  L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
  export TFP_LIB_PATH=$L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace_$v -o t -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_trace_$v.log 2>&1 || { tail gpurun_out/${R}_trace_$v.log; exit 5; }
done
unset TFP_LIB_PATH
python3 - <<'PY'
import csv, glob
for v in ("pre", "new"):
    f = glob.glob(f"gpurun_out/r06y_trace_{v}/**/t_kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "wide_" in r["Name"]:
            print(v, r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
