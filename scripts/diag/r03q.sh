# SQ counters of wide_groups_kernel at coefs=2 tol 0.45 (C3): instruction mix and wave-cycle split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03q
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "wide_groups" --output-format csv -d gpurun_out/r03q/p$i -o run -- python3 scripts/diag/c3_sweep.py 2 ${TOL:-0.45} 1 > gpurun_out/r03q/p$i.log 2>&1; rc=$?; echo "pass $i rc=$rc"; [ $rc = 0 ] || exit $rc
done
