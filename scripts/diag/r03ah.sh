# Occupancy of the clip-major sweep: the default (82 VGPRs, 5 waves/SIMD) against builds cut for 6
# (abv/occ6) and 8 (abv/occ8, 12 VGPRs spilled) waves per SIMD, C3 coefs=2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r03ah}
for t in 0.001 0.01 0.45; do
  timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_occ5_$t.log 2>&1 || exit $?; echo "occ5 $(grep median gpurun_out/${T}_occ5_$t.log)"
  for v in occ6 occ8; do
    TFP_LIB_PATH=$PWD/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 7 > gpurun_out/${T}_${v}_$t.log 2>&1 || exit $?; echo "$v $(grep median gpurun_out/${T}_${v}_$t.log)"
  done
done
