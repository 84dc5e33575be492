# A/B of compile flags for the engine (rebuilt on the box), parity subset + fingerprint timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for fl in "$@"; do
  i=$((i+1))
  make -s -C asterisk-tiresias_amd clean && make -s -j16 -C asterisk-tiresias_amd EXTRA="$fl" > /dev/null 2>&1 || exit 3
  timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "fingerprint or golden" > gpurun_out/abf_$i.log 2>&1; rc=$?; echo "[$fl] pytest rc=$rc $(tail -1 gpurun_out/abf_$i.log)"; case $rc in 0|1) ;; *) exit $rc;; esac
  timeout -k 10 300 python bench.py --no-match --no-cpu --steps 50 --warmup 5 --clock-warmup-s 0.25 > /dev/null 2> gpurun_out/abf_$i.err; rc=$?; echo "[$fl] $(grep fingerprint: gpurun_out/abf_$i.err)"; case $rc in 0) ;; *) exit $rc;; esac
done
