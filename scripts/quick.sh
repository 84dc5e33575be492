# parity tests (fingerprint/device/golden subset or full) + fingerprint timing (+ optional ablations)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu ${PYK:+-k "$PYK"} > gpurun_out/q_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/q_pytest.log)"; case $rc in 0) ;; 1) tail -30 gpurun_out/q_pytest.log; exit 1;; *) exit $rc;; esac
for a in ${ABL:-0}; do
  TFP_ABLATE=$a timeout -k 10 200 python bench.py --no-match --no-cpu --steps 20 --warmup 3 > /dev/null 2> gpurun_out/q_abl_$a.err; rc=$?
  echo "ablate=$a rc=$rc $(grep 'fingerprint:' gpurun_out/q_abl_$a.err)"; case $rc in 0) ;; *) exit $rc;; esac
done
