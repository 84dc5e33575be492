# Round 6: the bin sort's chunk-0 bin and group sizes at C3 coefs = 2 (TFP_DEBUG_BINS), for the
# wide_bin_sort long tail (73 us for 10,112 waves of ~7 us each).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TFP_TEST_KNOBS=1 TFP_DEBUG_BINS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.001 1 > gpurun_out/r06s_bins.log 2>&1; rc=$?; grep -E "bins chunk|median|bin sort waves|cycles, frames" gpurun_out/r06s_bins.log | tail -20; exit $rc
