# GPU test run: the -m gpu suite (or the tests named in $TESTS), one process, per-test timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-rX}
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -x -v -s -rs -m gpu --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/${TAG}_pytest.log | tail -3; exit $rc
