# Add-only host fast path of the index update (no pass over every clip) and one host wait per
# merge: the index tests, then the enrol-then-search bench leg (engine timings) and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_index.py tests/test_gpu_group.py tests/test_gpu_fp_handler.py tests/test_shim.py > gpurun_out/r03an_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03an_pytest.log; [ $rc = 0 ] || exit $rc
TFP_DEBUG_INDEX=1 timeout -k 10 400 python3 bench.py --no-cpu --no-strong --no-sweeps --steps 3 --warmup 1 --stream-ticks 5 > gpurun_out/r03an_bench.json 2> gpurun_out/r03an_bench.err; rc=$?; echo "bench rc=$rc"; grep -E "enrol|index merge" gpurun_out/r03an_bench.err | tail -12; [ $rc = 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03an_trace -o b -- python3 bench.py --no-cpu --no-strong --no-sweeps --steps 3 --warmup 1 --stream-ticks 5 > /dev/null 2> gpurun_out/r03an_trace.err; echo "trace rc=$?"
