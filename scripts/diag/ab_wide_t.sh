# timing-only A/B of general-path variants (experiment builds whose results are not checked)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
libof() { [ "$1" = base ] && echo "" || echo "$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$1/libtiresias_fp.so"; }
for n in "$@"; do
  for tol in ${TOLS:-0.001 0.45}; do TFP_LIB_PATH=$(libof $n) timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 | sed "s/^/[$n] /" || exit $?; done
done
