# Round-3 evidence on the final build: the GPU check (tests, smoke, bench), the bench under a kernel
# trace with the fingerprint kernel's HBM PMC (profile_round.sh), and the coefs=2 general path at C3
# tol 0.001 (kernel trace, then FETCH_SIZE / WRITE_SIZE of the wide_* kernels in separate passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${R:-r03ae}
TAG=$R bash scripts/gpu_check.sh || exit $?
R=$R bash scripts/profile_round.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; tail -1 gpurun_out/${R}_wide_trace.log; [ $rc = 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "wide_" --output-format csv -d gpurun_out/${R}_wide_pmc_$c -o run -- python3 scripts/diag/c3_sweep.py 2 0.001 3 > gpurun_out/${R}_wide_pmc_$c.log 2>&1; rc=$?; echo "wide pmc $c rc=$rc"; [ $rc = 0 ] || exit $rc
done
