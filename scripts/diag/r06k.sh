# Round 6: wide_clips A/B at C3 coefs 2 and batch-1: the committed tree before the window changes
# (abv/r06base), empty windows skipped with the 16 count rows cleared per window (abv/lazy0), and the
# tree (empty windows skipped, count rows written on a column's first add).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06k
S="2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r06base lazy0 new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c2_alt.py 200 > gpurun_out/${R}_alt.txt 2>&1 || { cat gpurun_out/${R}_alt.txt; exit 5; }
    grep batch-1 gpurun_out/${R}_alt.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
