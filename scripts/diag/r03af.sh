# The sweep tests (many keys per chunk, cluster gaps) on the default build, then the SQLite goldens
# on a debug build of the cross-key batching experiment (abv/xk, printf on a count underflow).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sweep_clusters.py > gpurun_out/r03af_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03af_pytest.log; [ $rc = 0 ] || exit $rc
TFP_LIB_PATH=$PWD/asterisk-tiresias_amd/abv/xk/libtiresias_fp.so timeout -k 10 300 python -u -m pytest -x -s -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k golden > gpurun_out/r03af_xk.log 2>&1; echo "xk rc=$?"; grep -m 20 XKBUG gpurun_out/r03af_xk.log; tail -3 gpurun_out/r03af_xk.log
exit 0
