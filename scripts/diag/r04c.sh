cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W12=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/w12/libtiresias_fp.so
(ldconfig -p | grep -i -E "aubio|fftw" ; ls /usr/lib/x86_64-linux-gnu | grep -i -E "aubio|fftw"; true) > gpurun_out/r04c_aubio_probe.txt 2>&1
timeout -k 10 120 ./scripts/microbench/valu_issue > gpurun_out/r04c_valu.txt 2>&1 || exit 3
for r in 1 2; do
  timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04c_fpc2.txt 2>&1 || exit 4
  TFP_LIB_PATH=$W12 timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04c_fpc2.txt 2>&1 || exit 5
done
TFP_FP_BLOCKS_PER_CU=1 timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04c_fpc2.txt 2>&1 || exit 6
cat gpurun_out/r04c_fpc2.txt
TFP_LIB_PATH=$W12 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu -k "configs1 or fingerprint or golden" --timeout 240 --timeout-method thread > gpurun_out/r04c_w12_pytest.log 2>&1; rc=$?
echo "w12 parity rc=$rc $(tail -1 gpurun_out/r04c_w12_pytest.log)"; [ $rc = 0 ] || exit $rc
TAG=r04c bash scripts/gpu_tests.sh
