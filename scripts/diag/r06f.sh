# Round 6: the configs suite (streaming at the 100k-clip DB, the C3 batch's sweep paths) and the
# sweep suite; then item 4 of the round-5 verdict: the fingerprint launch on the C2 and C3-query
# shapes in one process (alone; after the 100k-clip enrolment; with 2 ms idle gaps between launches),
# and GRBM_GUI_ACTIVE per dispatch of both shapes (the clock each ran at: GRBM / 8 / duration).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06f
TESTS="tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 > gpurun_out/${R}_shapes.txt 2>&1 || exit 5
ENROL=1 timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 >> gpurun_out/${R}_shapes.txt 2>&1 || exit 6
GAP_MS=2 timeout -k 10 300 python3 scripts/diag/fp_shapes.py 30 >> gpurun_out/${R}_shapes.txt 2>&1 || exit 7
grep -v amdgpu.ids gpurun_out/${R}_shapes.txt
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${R}_shapes_trace -o t -- python3 scripts/diag/fp_shapes.py 20 > gpurun_out/${R}_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "fingerprint8k_kernel" --output-format csv -d gpurun_out/${R}_shapes_pmc -o p -- python3 scripts/diag/fp_shapes.py 20 > gpurun_out/${R}_pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"; exit $rc
