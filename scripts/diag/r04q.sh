# Packed keys-only sort for the coefs=2 sweep: the whole GPU suite, then C3 coefs=2 timing against
# TFP_WIDE_UNPACKED=1 (the pair sort), interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04q bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for tol in 0.001 0.01 0.1 0.45; do
    timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 2>/dev/null | sed "s/^/[packed] /" || exit 5
    TFP_WIDE_UNPACKED=1 timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 2>/dev/null | sed "s/^/[pairs] /" || exit 6
  done
done
