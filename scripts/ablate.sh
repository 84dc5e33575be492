# Phase ablation of the fingerprint kernel (timing only; outputs are wrong when TFP_ABLATE != 0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in ${ABL:-0 1 2 4 8 16 24 30 31}; do
  TFP_ABLATE=$a timeout -k 10 200 python bench.py --no-match --no-cpu --steps 20 --warmup 3 > /dev/null 2> gpurun_out/abl_$a.err; rc=$?
  echo "ablate=$a rc=$rc $(grep 'fingerprint:' gpurun_out/abl_$a.err)"; case $rc in 0) ;; *) exit $rc;; esac
done
