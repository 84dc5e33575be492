# Round 5: the bin sort's counts on one C3 coefs=2 batch (TFP_DEBUG_BINS).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TFP_TEST_KNOBS=1 TFP_DEBUG_BINS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.001 1 > gpurun_out/r05i.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05i.txt | tail -8; exit $rc
