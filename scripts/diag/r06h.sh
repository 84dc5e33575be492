# Round 6: the sweep's prefix-count form A/B at C3 (checkpoint rows every 4 frames: the tree; a row
# per frame: abv/p1; the round-5 build: abv/r05), then the coefs = 2 first-search-after-enrolment
# rounds (scripts/diag/c2_enrol.py) under a kernel trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06h
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r05 new p1; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_enrol_trace -o enrol -- python3 scripts/diag/c2_enrol.py 8 > gpurun_out/${R}_enrol.log 2>&1; rc=$?; echo "enrol trace rc=$rc"; grep -E "round|cache" gpurun_out/${R}_enrol.log; exit $rc
