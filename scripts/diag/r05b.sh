# Round 5: fingerprint8k_kernel<4> LDS-latency changes (filterbank reads pipelined by segment with
# its stores deferred; window and split-twiddle reads issued ahead of the syncs): bit-exactness on
# the full configs[1] batch and the kernel variants, then C2 A/B interleaved, then the bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05b
TESTS="tests/test_gpu_configs.py::test_configs1_full_batch_bit_exact tests/test_gpu_parity.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for r in 1 2 3; do
  for v in base fb fbwin all; do
    TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_ab.txt 2>&1 || exit 4
  done
done
grep "fp C2" gpurun_out/${R}_ab.txt
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/${R}_bench.err; exit $rc
