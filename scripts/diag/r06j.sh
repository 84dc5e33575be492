# Round 6: wide_clips skipping windows where no used key has a group (the tree) against the
# committed sweep (abv/r06base) at C3 coefs 2, then kernel traces of the tree's coefs = 2 batch at
# tol 0.001 and 0.45.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06j
S="2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r06base new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
for t in 0.001 0.45; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_$t -o c3 -- python3 scripts/diag/c3_sweep.py 2 $t 5 > gpurun_out/${R}_wide_$t.log 2>&1; rc=$?; echo "trace $t rc=$rc"; [ $rc = 0 ] || exit $rc
done
