# coefs=2 at C3, A/B of the sweep forms: clip-major with 32-clip windows (default), 64-clip windows
# (abv/win64), and the key-major form (TFP_WIDE_GROUPS); after the general-path parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r03ab}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sweep_clusters.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "clusters or general or golden or pcm_vs_oracle or fallback or configs2" > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log; [ $rc = 0 ] || exit $rc
for t in 0.001 0.01 0.45; do
  timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_clip32_$t.log 2>&1 || exit $?; echo "clip32 $(grep median gpurun_out/${T}_clip32_$t.log)"
  TFP_LIB_PATH=$PWD/asterisk-tiresias_amd/abv/win64/libtiresias_fp.so timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_clip64_$t.log 2>&1 || exit $?; echo "clip64 $(grep median gpurun_out/${T}_clip64_$t.log)"
  TFP_WIDE_GROUPS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_groups_$t.log 2>&1 || exit $?; echo "groups $(grep median gpurun_out/${T}_groups_$t.log)"
done
