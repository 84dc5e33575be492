# GPU round trip: parity tests -> smoke -> bench -> rocprofv3 kernel stats. Stops on any fault.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-rX}
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: rc=$1 (fault/abort/timeout)"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -x -v -rs -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/${TAG}_pytest.log; ok $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; ok $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/${TAG}_bench.err; cat gpurun_out/${TAG}_bench.json; ok $rc
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ${PROF_ARGS} > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/${TAG}_prof.log
  find gpurun_out/${TAG}_prof -name "*stats*" | head; 
fi
