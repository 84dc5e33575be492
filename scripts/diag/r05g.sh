# Round 5: the coefs=2 sweep's bin sort (wide_bins .. wide_dir_fill_bins) in place of the library
# sort on the speculative pass: the sweep tests, the C3 sweeps against the oracle, C3 timings of the
# bin sort vs the library sort (TFP_WIDE_LIBSORT), and a kernel trace of one tol 0.001 batch.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05g
TESTS="tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
for t in 0.001 0.01 0.1 0.45; do
  timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 9 >> gpurun_out/${R}_c3.txt 2>&1 || exit 4
  TFP_TEST_KNOBS=1 TFP_WIDE_LIBSORT=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 9 > gpurun_out/${R}_c3_lib.txt 2>&1 || exit 5
  sed 's/^/libsort /' gpurun_out/${R}_c3_lib.txt >> gpurun_out/${R}_c3.txt
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; exit $rc
