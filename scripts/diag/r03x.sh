# coefs=2 at C3 after the batched wide_final: kernel traces at tol 0.001 and 0.45, and the
# wide_groups work without its score writes (abv/noscore, timing only) at both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for t in 0.001 0.45; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03x_trace_$t -o c3 -- python3 scripts/diag/c3_sweep.py 2 $t 5 > gpurun_out/r03x_trace_$t.log 2>&1; rc=$?; echo "trace $t rc=$rc"; grep median gpurun_out/r03x_trace_$t.log; [ $rc = 0 ] || exit $rc
done
TFP_LIB_PATH=$PWD/asterisk-tiresias_amd/abv/noscore/libtiresias_fp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03x_noscore -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.45 5 > gpurun_out/r03x_noscore.log 2>&1; rc=$?; echo "noscore rc=$rc"; grep median gpurun_out/r03x_noscore.log; exit $rc
