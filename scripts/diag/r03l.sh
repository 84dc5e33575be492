# coefs=2 general-path change: parity (configs sweeps, parity, dbio, index) then C3 timings + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r03l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_dbio.py tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc = 0 ] || exit $rc
for tol in 0.001 0.01 0.45; do timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 || exit $?; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${T}_wide_trace.log 2>&1; echo "trace rc=$?"
