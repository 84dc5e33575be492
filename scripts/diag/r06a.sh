# Round 6: the sweep-r05p changes (fused directory fill, both-end bucket probes, checkpoint prefix
# rows) on main: the sweep and C3 config tests, C3 timings against the round-5 build (abv/r05,
# interleaved), a kernel trace of one coefs=2 tol 0.001 batch and of the coefs=1 batch.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06a
TESTS="tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r05 new; do
    L=""; [ $v = r05 ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/r05/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 7 $S > gpurun_out/${R}_one.txt 2>&1 || exit 4
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_c1_trace -o c1 -- python3 scripts/diag/c3_sweep.py 1 0.001 9 > gpurun_out/${R}_c1_trace.log 2>&1; rc=$?; echo "c1 trace rc=$rc"; exit $rc
