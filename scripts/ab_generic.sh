# GPU parity tests, then A/B of the 8 kHz specialized fingerprint kernel against the generic one
# (TFP_GENERIC=1) on the configs[1] bench leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/ab_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/ab_pytest.log)"; case $rc in 0) ;; 1) tail -40 gpurun_out/ab_pytest.log; exit 1;; *) exit $rc;; esac
for g in 0 1 0 1; do
  TFP_GENERIC=$g timeout -k 10 200 python bench.py --no-match --no-cpu --stream-channels 0 --steps 20 --warmup 3 > gpurun_out/ab_g$g.json 2> gpurun_out/ab_g$g.err; rc=$?
  echo "generic=$g rc=$rc $(grep 'fingerprint:' gpurun_out/ab_g$g.err)"; case $rc in 0) ;; *) tail -5 gpurun_out/ab_g$g.err; exit $rc;; esac
done
