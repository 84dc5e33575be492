set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: rc=$1 (fault/abort/timeout)"; exit "$1";; esac; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/r2_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r2_pytest.log; ok $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r2_smoke.log; ok $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --db-clips 10000 --queries 1024 --latency-queries 10 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/r2_bench.err; cat gpurun_out/r2_bench.json
