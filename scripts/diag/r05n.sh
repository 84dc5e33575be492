# Round 5: smoke and the bench on the bin-sort tree (the -m gpu suite ran on it as r05k).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05n
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/${R}_bench.err; exit $rc
