# Round 5: the directory fill fused into the bin sort (segk constants from the scan), bucket
# searches that probe both ends first, and prefix-count rows every 4 frames (kPStep; variant p1 =
# a row per frame, scripts/build_variant.sh p1 -DTFP_PSTEP=1): the sweep and C3 config tests, C3
# coefs=2 timings of both (interleaved), a kernel trace of one tol 0.001 batch, and a coefs=1 trace
# (the C3 query launch).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05p
TESTS="tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
for t in 0.001 0.01 0.1 0.45; do
  for v in base p1; do
    L=""; [ $v = p1 ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/p1/libtiresias_fp.so
    TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 9 > gpurun_out/${R}_one.txt 2>&1 || exit 4
    grep -v amdgpu.ids gpurun_out/${R}_one.txt | sed "s/^/$v /" >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; [ $rc = 0 ] || exit $rc
# the C3 query launch on its own (coefs=1 batches: fingerprints, then the vote)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_c1_trace -o c1 -- python3 scripts/diag/c3_sweep.py 1 0.001 9 > gpurun_out/${R}_c1_trace.log 2>&1; rc=$?; echo "c1 trace rc=$rc"; exit $rc
