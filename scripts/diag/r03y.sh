# General-path parity tests, then C3 kernel traces at tol 0.001 and 0.45 (TAG names the outputs),
# and the key-major form (TFP_WIDE_GROUPS) timed beside it at both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sweep_clusters.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "clusters or general or golden or pcm_vs_oracle or fallback or configs2 or index" > gpurun_out/${TAG:-r03y}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG:-r03y}_pytest.log; [ $rc = 0 ] || exit $rc
for t in 0.001 0.45; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG:-r03y}_trace_$t -o c3 -- python3 scripts/diag/c3_sweep.py 2 $t 5 > gpurun_out/${TAG:-r03y}_trace_$t.log 2>&1; rc=$?; echo "trace $t rc=$rc"; grep median gpurun_out/${TAG:-r03y}_trace_$t.log; [ $rc = 0 ] || exit $rc
done
TFP_WIDE_GROUPS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.45 5 > gpurun_out/${TAG:-r03y}_groups_0.45.log 2>&1; rc=$?; echo "groups form rc=$rc"; grep median gpurun_out/${TAG:-r03y}_groups_0.45.log; [ $rc = 0 ] || exit $rc
TFP_WIDE_GROUPS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${TAG:-r03y}_groups_0.001.log 2>&1; rc=$?; echo "groups form rc=$rc"; grep median gpurun_out/${TAG:-r03y}_groups_0.001.log; exit $rc
