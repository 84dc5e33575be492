# Round 6: the clip-set cache's build kernels with a thread's 16 consecutive rows (16-byte loads,
# one block scan) and the tile scan through LDS: cache / index / sweep / configs tests, then the
# first coefs = 2 searches at new tolerances under a kernel trace, then the wide_clips count-row A/B
# (scripts/diag/r06l.sh).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06m
timeout -k 10 900 python -u -m pytest tests/test_gpu_cellcache.py tests/test_gpu_index.py tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${R}_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_newtol -o nt -- python3 scripts/diag/c2_newtol.py > gpurun_out/${R}_newtol.log 2>&1; rc=$?; echo "newtol rc=$rc"; grep -E "tol|cache" gpurun_out/${R}_newtol.log; [ $rc = 0 ] || exit $rc
bash scripts/diag/r06l.sh
