# SQ counters of the coefs=2 sweep kernels at C3 tol 0.001 (two passes, no tracing domains).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "wide_clips|wide_dir_fill|wide_prefix" --output-format csv -d gpurun_out/r04i/p$i -o run -- python3 scripts/diag/c3_sweep.py 2 0.001 3 > gpurun_out/r04i_p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"; [ $rc = 0 ] || exit $rc
done
