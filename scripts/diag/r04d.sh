# Round 4: the refactored default build's fingerprint parity, the 12-wave build under TFP_DEBUG_OCC
# (launch diagnostics), C2 timing of both on a real stream, then the whole GPU suite.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W12=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/w12/libtiresias_fp.so
K="configs1 or fingerprint or golden"
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu -k "$K" --timeout 240 --timeout-method thread > gpurun_out/r04d_base_pytest.log 2>&1; rc=$?
echo "base parity rc=$rc $(tail -1 gpurun_out/r04d_base_pytest.log)"; case $rc in 0|1) ;; *) exit $rc;; esac
TFP_DEBUG_OCC=1 TFP_LIB_PATH=$W12 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -s -m gpu -k configs1 --timeout 240 --timeout-method thread > gpurun_out/r04d_w12_pytest.log 2>&1; rc12=$?
echo "w12 parity rc=$rc12 $(tail -1 gpurun_out/r04d_w12_pytest.log)"; grep "\[tfp\]" gpurun_out/r04d_w12_pytest.log | head; case $rc12 in 0|1) ;; *) exit $rc12;; esac
for r in 1 2; do
  timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04d_fpc2.txt 2>&1 || exit 4
  if [ $rc12 = 0 ]; then TFP_LIB_PATH=$W12 timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04d_fpc2.txt 2>&1 || exit 5; fi
done
TFP_FP_BLOCKS_PER_CU=1 timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04d_fpc2.txt 2>&1 || exit 6
grep "fp C2" gpurun_out/r04d_fpc2.txt
[ $rc = 0 ] || exit 1
TAG=r04d bash scripts/gpu_tests.sh
