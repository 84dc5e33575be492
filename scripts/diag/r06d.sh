# Round 6: the clip-order clip-set caches (LRU, carried through merges): their GPU tests, the sweep and
# index suites on the new tree, the earlier failing concurrency test; then the r06c measurements.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06d
TESTS="tests/test_gpu_group.py tests/test_gpu_cellcache.py tests/test_gpu_concurrency.py tests/test_gpu_device.py tests/test_gpu_sweep_clusters.py tests/test_gpu_index.py tests/test_gpu_configs.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 > gpurun_out/${R}_shapes.txt 2>&1 || exit 5
ENROL=1 timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 >> gpurun_out/${R}_shapes.txt 2>&1 || exit 6
GAP_MS=2 timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 >> gpurun_out/${R}_shapes.txt 2>&1 || exit 7
grep -v amdgpu.ids gpurun_out/${R}_shapes.txt
R=r06d bash scripts/diag/r06b.sh
