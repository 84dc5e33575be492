# Round 6: configs[3] as 8 gloo ranks on the one GPU (tests/test_gpu_c4.py) alone, with each side
# checked against the oracle first (the r06z suite run saw sharded != unsharded for queries >= 3585).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4.py -x -v -m gpu --timeout 850 --timeout-method thread > gpurun_out/r06q_c4.log 2>&1; rc=$?; tail -30 gpurun_out/r06q_c4.log; exit $rc
