# Round 6: finish_db four values a thread (the tree) against one (abv/fd1): configs[1] parity and
# C2 steps; the bench on this tree (new legs: coefs=2 caches, group enrolment), then the sweep's
# prefix-count form A/B (checkpoint rows every 4 frames, the tree, against a row per frame, abv/p1,
# and the round-5 build abv/r05) at C3 coefs 1 / 2, then a coefs=2 tol 0.001 kernel trace of p1.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06g
TAG=${R}_ab bash scripts/ab_libs.sh base fd1; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/${R}_bench.err; [ $rc = 0 ] || exit $rc
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r05 new p1; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || exit 4
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
TFP_LIB_PATH=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/p1/libtiresias_fp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace_p1 -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; exit $rc
