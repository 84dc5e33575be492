# Round 6: wide_clips count rows per window: cleared always (abv/r06base), written on first add
# always (abv/lzall), or by the window's group count (first-add writes below 4 / 8 / 16 groups:
# abv/lz4, the tree, abv/lz16), at C3 coefs 2 and batch-1.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06l
S="2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r06base lzall lz4 new lz16; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c2_alt.py 200 > gpurun_out/${R}_alt.txt 2>&1 || { cat gpurun_out/${R}_alt.txt; exit 5; }
    grep batch-1 gpurun_out/${R}_alt.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
