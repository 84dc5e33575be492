# Round 5: the tree (direct-PCM fingerprint kernel, b128 filterbank weights): the GPU suite, smoke,
# then the bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05f
TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/${R}_bench.err; exit $rc
