# Round 6 (final tree): the clip sweep's wave clocks (abv/clk: -DTFP_BIN_CLOCKS=1 with TFP_DEBUG_BINS) at C3
# coefs = 2, tol 0.001 and 0.45: is wide_clips' time a tail of slow waves or the waves' mean?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for t in 0.001 0.45; do
  TFP_LIB_PATH=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/clk/libtiresias_fp.so TFP_TEST_KNOBS=1 TFP_DEBUG_BINS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 1 > gpurun_out/r06av_$t.log 2>&1 || { tail -20 gpurun_out/r06av_$t.log; exit 3; }
  echo "tol $t"; grep -E "clip sweep waves|  wave " gpurun_out/r06av_$t.log | tail -9
done
