set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_group.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03k_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03k_pytest.log; [ $rc = 0 ] || exit $rc
TFP_DEBUG_INDEX=1 timeout -k 10 400 python bench.py --no-cpu --no-strong > gpurun_out/r03k_bench.json 2> gpurun_out/r03k_bench.err; rc=$?; echo "bench rc=$rc"; grep -E "enrol|index merge" gpurun_out/r03k_bench.err | tail -30; exit $rc
