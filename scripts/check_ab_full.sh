# A/B of compile-flag variants (args), ending on the default build; then the full GPU suite and a
# short bench (match + stream legs at a reduced DB size).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/ab_flags.sh "$@" "" || exit $?
timeout -k 10 700 python -m pytest tests -x -q -m gpu > gpurun_out/full_pytest.log 2>&1; rc=$?
echo "full pytest rc=$rc $(tail -1 gpurun_out/full_pytest.log)"; case $rc in 0) ;; 1) tail -40 gpurun_out/full_pytest.log; exit 1;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --no-cpu --steps 5 --warmup 2 --db-clips 20000 > gpurun_out/short_bench.json 2> gpurun_out/short_bench.err; rc=$?
echo "bench rc=$rc"; tail -4 gpurun_out/short_bench.err; exit $rc
