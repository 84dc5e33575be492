# Round-4 final tree: the GPU suite, C3 coefs=2 timing, smoke, bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r04v
TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
for tol in 0.001 0.01 0.1 0.45; do
  timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 2>/dev/null || exit 5
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${R}_bench.err; exit $rc
