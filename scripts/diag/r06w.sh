# Round 6: the bin sort's per-phase wave clocks and long-run directory buckets (abv/clk) at C3 coefs = 2.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TFP_LIB_PATH=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/clk/libtiresias_fp.so TFP_TEST_KNOBS=1 TFP_DEBUG_BINS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.001 1 > gpurun_out/r06w_bins.log 2>&1; rc=$?; grep -E "bin sort waves|cycles" gpurun_out/r06w_bins.log | tail -13; exit $rc
