# A/B of fingerprint-kernel build variants on the GPU box: for each EXTRA flag set (args; "" =
# default), rebuild the library, check configs[1] full-size parity, time the C2 fingerprint leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
v=0
for fl in "$@"; do
  v=$((v+1))
  make -s -C asterisk-tiresias_amd clean && make -s -j16 -C asterisk-tiresias_amd EXTRA="$fl" > gpurun_out/$TAG/build$v.log 2>&1 || { echo "build $v failed"; exit 3; }
  timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k "configs1" --timeout 240 --timeout-method thread > gpurun_out/$TAG/test$v.log 2>&1; rc=$?
  echo "[$fl] parity rc=$rc $(tail -1 gpurun_out/$TAG/test$v.log)"; case $rc in 0) ;; *) exit $rc;; esac
  for rep in 1 2; do
    timeout -k 10 300 python bench.py --no-match --no-cpu --no-strong --steps 30 > gpurun_out/$TAG/bench$v.$rep.json 2> gpurun_out/$TAG/bench$v.$rep.err; rc=$?
    echo "[$fl] bench rc=$rc $(grep "avg launch\|blocks/CU" gpurun_out/$TAG/bench$v.$rep.err | tr "\\n" " ")"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
