# A/B of general-path library variants (scripts/build_variant.sh): coefs=2 parity sweeps at full
# DB size, then C3 timings at tol 0.001 / 0.01 / 0.45. Args: variant names ("base" = lib/).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
libof() { [ "$1" = base ] && echo "" || echo "$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$1/libtiresias_fp.so"; }
for n in "$@"; do
  TFP_LIB_PATH=$(libof $n) timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k "sweeps" --timeout 300 --timeout-method thread > gpurun_out/abw_$n.log 2>&1; rc=$?
  echo "[$n] parity rc=$rc $(tail -1 gpurun_out/abw_$n.log)"; [ $rc = 0 ] || exit $rc
  for tol in 0.001 0.01 0.45; do TFP_LIB_PATH=$(libof $n) timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 | sed "s/^/[$n] /" || exit $?; done
done
