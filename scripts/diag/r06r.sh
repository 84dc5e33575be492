# Round 6: SQ counters of wide_clips at C3 coefs = 2 tol 0.001 and 0.45 (two passes each, one --pmc
# group per run, no tracing domains).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06r
for t in 0.001 0.45; do
  mkdir -p gpurun_out/${R}_$t
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "wide_clips|wide_bin_sort" --output-format csv -d gpurun_out/${R}_$t/p$i -o run -- python3 scripts/diag/c3_sweep.py 2 $t 3 > gpurun_out/${R}_$t/p$i.log 2>&1; rc=$?
    echo "tol $t pass $i rc=$rc"; [ $rc = 0 ] || exit $rc
  done
done
