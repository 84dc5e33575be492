# The 12-wave fingerprint build after the asm early-clobber fix: small-launch check, configs[1]
# parity, then C2 timing interleaved with the default build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W12=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/w12/libtiresias_fp.so
for v in base w12; do
  L=""; [ $v = base ] || L=$W12
  TFP_LIB_PATH=$L timeout -k 10 120 python scripts/diag/fp_variant_check.py >> gpurun_out/r04f_check.txt 2>&1 || exit 3
done
grep -v amdgpu.ids gpurun_out/r04f_check.txt
TFP_LIB_PATH=$W12 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu -k "configs1 or fingerprint or golden" --timeout 240 --timeout-method thread > gpurun_out/r04f_w12_pytest.log 2>&1; rc=$?
echo "w12 parity rc=$rc $(tail -1 gpurun_out/r04f_w12_pytest.log)"; case $rc in 0|1) ;; *) exit $rc;; esac
for r in 1 2 3; do
  timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04f_fpc2.txt 2>&1 || exit 4
  TFP_LIB_PATH=$W12 timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/r04f_fpc2.txt 2>&1 || exit 5
done
grep "fp C2" gpurun_out/r04f_fpc2.txt
