# Round evidence: rocprofv3 kernel-trace stats of the bench command, then PMC HBM bytes of the
# fingerprint kernel (FETCH_SIZE and WRITE_SIZE in separate passes, per MI355X_MICROARCH §HBM).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${R:-r01}
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace -o bench -- python3 bench.py ${BENCH_ARGS} > gpurun_out/${R}_trace.json 2> gpurun_out/${R}_trace.err; rc=$?; echo "trace rc=$rc"; tail -2 gpurun_out/${R}_trace.err; case $rc in 0) ;; *) exit $rc;; esac
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "fingerprint(8k)?_kernel|finish_db_kernel" --output-format csv -d gpurun_out/${R}_pmc_$c -o run -- python3 bench.py --no-match --no-cpu --no-strong --steps 5 --warmup 1 > gpurun_out/${R}_pmc_$c.log 2>&1; rc=$?; echo "pmc $c rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
