# Round 5: direct-PCM fingerprint kernel forms: dpcmp (first production form), dpt (buffer
# resource per tile), dpt_notw (dpt without the split twiddles' early read: 18 fewer hazard
# nops, 3 fewer VGPRs). Exactness (incl. ragged clips with odd starts and lengths), then C2 and
# C3-shaped launches interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05e
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for v in dpt dpt_notw; do
  TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_variant_check.py >> gpurun_out/${R}_check.txt 2>&1 || exit 3
done
grep -v amdgpu.ids gpurun_out/${R}_check.txt
for r in 1 2 3; do
  for v in w128 dpcmp dpt dpt_notw; do
    TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_ab.txt 2>&1 || exit 4
    FP_CLIPS=4096 FP_SECONDS=5 TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_ab.txt 2>&1 || exit 4
  done
done
grep "fp " gpurun_out/${R}_ab.txt
