# Round-6 profiles: the bench under a kernel trace + the fingerprint kernel's HBM PMC
# (profile_round.sh), its SQ issue counters (two passes), and the coefs=2 general path at C3 under a
# kernel trace at tol 0.001 and 0.45.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${R:-r06}
[ -n "$SKIP_BENCH" ] || R=$R bash scripts/profile_round.sh || exit $?
TAG=${R}_sq bash scripts/gpu_pmc.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" || exit $?
for t in 0.001 0.45; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_$t -o c3 -- python3 scripts/diag/c3_sweep.py 2 $t 5 > gpurun_out/${R}_wide_$t.log 2>&1; rc=$?; echo "wide trace $t rc=$rc"; tail -1 gpurun_out/${R}_wide_$t.log; [ $rc = 0 ] || exit $rc
done
