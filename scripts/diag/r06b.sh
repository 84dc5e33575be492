# Round 6: the sweep-r05p changes split: checkpoint prefix rows every 4 frames (new) against a row
# per frame (abv/p1: -DTFP_PSTEP=1), both with the fused directory fill and the both-end probes,
# against the round-5 build (abv/r05); C3 batch times per setting, each setting's calls back to back.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${R:-r06b}
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
