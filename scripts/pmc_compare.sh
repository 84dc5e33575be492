# PMC counter passes of the fingerprint kernel for each build variant (args = EXTRA flags; "" = default).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
G3="SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC"
v=0
for fl in "$@"; do
  v=$((v+1))
  make -s -C asterisk-tiresias_amd clean && make -s -j16 -C asterisk-tiresias_amd EXTRA="$fl" > /dev/null 2>&1 || exit 3
  g=0
  for grp in "$G1" "$G2" "$G3"; do
    g=$((g+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "fingerprint(8k)?_kernel" --output-format csv -d gpurun_out/pmcc/v${v}g$g -o run -- python3 bench.py --no-match --no-cpu --steps 3 --warmup 1 > gpurun_out/pmcc/v${v}g$g.log 2>&1; rc=$?
    echo "[$fl] group $g rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
