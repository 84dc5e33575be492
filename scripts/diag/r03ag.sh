# Cross-key batches in the clip-major sweep: general-path parity (with the SQLite goldens), then C3
# coefs=2 timings of the default (16-clip windows) and 32-clip windows (abv/win32).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r03ag}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sweep_clusters.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_group.py -k "clusters or sweep or general or golden or pcm_vs_oracle or fallback or configs2 or group" > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log; [ $rc = 0 ] || exit $rc
for t in 0.001 0.01 0.1 0.45; do
  timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_xk16_$t.log 2>&1 || exit $?; echo "xk16 $(grep median gpurun_out/${T}_xk16_$t.log)"
  TFP_LIB_PATH=$PWD/asterisk-tiresias_amd/abv/win32/libtiresias_fp.so timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_xk32_$t.log 2>&1 || exit $?; echo "xk32 $(grep median gpurun_out/${T}_xk32_$t.log)"
done
