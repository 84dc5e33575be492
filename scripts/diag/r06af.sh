# Round 6: a mutant library (dir_write's per-lane runs without their last 1-3 buckets, abv/mut)
# must fail test_bin_sort_crowd_groups_and_sparse_directory_runs (the test sees the directory).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TFP_LIB_PATH=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/mut/libtiresias_fp.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_sweep_clusters.py::test_bin_sort_crowd_groups_and_sparse_directory_runs" -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06af_pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed|assert got" gpurun_out/r06af_pytest.log | tail -6; [ $rc = 1 ] && echo "mutant killed" && exit 0; exit 3
