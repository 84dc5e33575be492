# Round 6: the bin sort's crowded groups and directory runs of every length
# (test_bin_sort_crowd_groups_and_sparse_directory_runs) with the sweep's other tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep_clusters.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06ae_pytest.log 2>&1; rc=$?; tail -25 gpurun_out/r06ae_pytest.log; exit $rc
