# Round 5: SQ counters of the C3 query launch (fingerprint8k_kernel<4> over 4096 x 5 s queries,
# 643,072 frames) to set against the C2 launch's (profiles/r05/pmc_fingerprint8k_r05.json).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05m
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "fingerprint8k_kernel" --output-format csv -d gpurun_out/${R}/p$i -o run -- python3 scripts/diag/c3_sweep.py 1 0.001 3 > gpurun_out/${R}/p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"; [ $rc = 0 ] || exit $rc
done
FRAMES=643072 LAST=3 python3 scripts/tools/pmc_summary.py gpurun_out/${R}/p1 gpurun_out/${R}/p2 > gpurun_out/${R}_summary.json; cat gpurun_out/${R}_summary.json
