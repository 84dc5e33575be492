# 16-clip windows (abv/win16) against the default 32 at C3 coefs=2, then the full GPU check
# (tests, smoke, bench).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r03ac}
for t in 0.001 0.01 0.45; do
  timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_clip32_$t.log 2>&1 || exit $?; echo "clip32 $(grep median gpurun_out/${T}_clip32_$t.log)"
  TFP_LIB_PATH=$PWD/asterisk-tiresias_amd/abv/win16/libtiresias_fp.so timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_clip16_$t.log 2>&1 || exit $?; echo "clip16 $(grep median gpurun_out/${T}_clip16_$t.log)"
done
TAG=$T bash scripts/gpu_check.sh
