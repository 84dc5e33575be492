# coefs=2 general path at wide tolerances: kernel traces (tol 0.1, 0.45)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for tol in 0.1 0.45; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03o_$tol -o c3 -- python3 scripts/diag/c3_sweep.py 2 $tol 3 > gpurun_out/r03o_$tol.log 2>&1; rc=$?; echo "trace $tol rc=$rc"; grep coefs gpurun_out/r03o_$tol.log; [ $rc = 0 ] || exit $rc
done
