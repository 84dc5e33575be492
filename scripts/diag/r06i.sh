# Round 6: coefs = 2 searches beside the index delta (the delta's own clip-set cache, no merge per
# enrolment) and the sweep's prefix rows back to a row per frame: the cache / index / sweep tests,
# configs (100k-clip DB: updated index, every sweep setting), the after-enrolment rounds, the bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06i
timeout -k 10 900 python -u -m pytest tests/test_gpu_cellcache.py tests/test_gpu_index.py tests/test_gpu_sweep_clusters.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest_a.log 2>&1; rc=$?; tail -3 gpurun_out/${R}_pytest_a.log; [ $rc = 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/${R}_pytest_b.log 2>&1; rc=$?; tail -3 gpurun_out/${R}_pytest_b.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/diag/c2_enrol.py 8 > gpurun_out/${R}_enrol.log 2>&1; rc=$?; grep -E "round|cache" gpurun_out/${R}_enrol.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; grep -E "coefs=2|sweep coefs=2" gpurun_out/${R}_bench.err; exit $rc
