# coefs=2 frame order by per-segment LDS sorts instead of hipCUB's merge sort: the sweep and
# parity tests, C3 timings of both orders (TFP_WIDE_RADIX A/B), and a kernel trace of the new one.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sweep_clusters.py tests/test_gpu_parity.py > gpurun_out/r03ap_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ap_pytest.log; [ $rc = 0 ] || exit $rc
for tol in 0.001 0.01 0.1 0.45; do
  timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $tol 10 > gpurun_out/r03ap_c3_seg_$tol.log 2>&1; rc=$?; echo "seg $tol rc=$rc: $(tail -1 gpurun_out/r03ap_c3_seg_$tol.log)"; [ $rc = 0 ] || exit $rc
  TFP_WIDE_RADIX=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $tol 10 > gpurun_out/r03ap_c3_radix_$tol.log 2>&1; rc=$?; echo "radix $tol rc=$rc: $(tail -1 gpurun_out/r03ap_c3_radix_$tol.log)"; [ $rc = 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ap_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/r03ap_trace.log 2>&1; echo "trace rc=$?"
