# Round 6: the GPU tests touched by the advisor fixes (coalescer re-runs, operational switches,
# long clips, group peer stats); the fingerprint launch on the C2 and C3-query shapes side by side
# (with and without the 100k-clip enrolment before it, item 4); then the r06b sweep A/B.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06c
TESTS="tests/test_gpu_concurrency.py tests/test_gpu_group.py tests/test_gpu_device.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 > gpurun_out/${R}_shapes.txt 2>&1 || exit 5
ENROL=1 timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 >> gpurun_out/${R}_shapes.txt 2>&1 || exit 6
GAP_MS=2 timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 >> gpurun_out/${R}_shapes.txt 2>&1 || exit 7
grep -v amdgpu.ids gpurun_out/${R}_shapes.txt
bash scripts/diag/r06b.sh
