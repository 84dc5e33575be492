# coefs=2 C3 per-kernel trace and FETCH/WRITE passes on the final tree.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r04w
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; [ $rc = 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "wide_" --output-format csv -d gpurun_out/${R}_wide_pmc_$c -o run -- python3 scripts/diag/c3_sweep.py 2 0.001 3 > gpurun_out/${R}_wide_pmc_$c.log 2>&1; rc=$?; echo "wide pmc $c rc=$rc"; [ $rc = 0 ] || exit $rc
done
