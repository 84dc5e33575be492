# PMC counters per ablation variant of the fingerprint kernel (one counter group per run).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmca
for a in ${ABL:-0 2 4 8}; do
  TFP_ABLATE=$a timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "fingerprint(8k)?_kernel" --output-format csv -d gpurun_out/pmca/a$a -o run -- python3 bench.py --no-match --no-cpu --steps 3 --warmup 1 > gpurun_out/pmca/a$a.log 2>&1; rc=$?
  echo "ablate $a rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
