# coefs=2 general path over clusters at C3: kernel traces at tol 0.001 and 0.45 (the cluster form)
# and the point form at 0.45 (TFP_WIDE_POINTS) for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for t in 0.001 0.45; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03w_trace_$t -o c3 -- python3 scripts/diag/c3_sweep.py 2 $t 5 > gpurun_out/r03w_trace_$t.log 2>&1; rc=$?; echo "trace $t rc=$rc"; tail -1 gpurun_out/r03w_trace_$t.log; [ $rc = 0 ] || exit $rc
done
TFP_WIDE_POINTS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.45 5 > gpurun_out/r03w_points_0.45.log 2>&1; rc=$?; echo "points rc=$rc"; tail -1 gpurun_out/r03w_points_0.45.log; exit $rc
