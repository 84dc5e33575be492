# Fewer small launches ahead of the coefs=2 sweep (bad-frame count in the key pass, coalesced
# frame -> query map, chunk starts from the gather): the whole GPU suite, then C3 coefs=2 timing.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04o bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for tol in 0.001 0.01 0.1 0.45; do
    timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 2>/dev/null || exit 5
  done
done
