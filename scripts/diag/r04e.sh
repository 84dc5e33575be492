# Which part of the 12-wave fingerprint build is wrong: the half-square layout at 4- and 8-wave
# workgroups (h4, h8) and the 12-wave build (w12), each on a small launch against the oracle.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base w12; do
  L=""; [ $v = base ] || L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
  TFP_LIB_PATH=$L timeout -k 10 120 python scripts/diag/fp_variant_check.py >> gpurun_out/r04e_check.txt 2>&1 || exit 3
done
grep -v amdgpu.ids gpurun_out/r04e_check.txt
