# A/B of runtime knobs (env assignments, "" = default) on the configs[1] fingerprint leg, with the
# fingerprint parity tests run under each knob first. Usage: bash scripts/ab_env.sh "" "TFP_PIPE=1" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "fingerprint or golden or search" > gpurun_out/abe_$i.log 2>&1; rc=$?; echo "[$kv] pytest rc=$rc $(tail -1 gpurun_out/abe_$i.log)"; case $rc in 0|1) ;; *) exit $rc;; esac
  env $kv timeout -k 10 300 python bench.py --no-match --no-cpu --steps 50 --warmup 5 --clock-warmup-s 0.25 > /dev/null 2> gpurun_out/abe_$i.err; rc=$?; echo "[$kv] $(grep fingerprint: gpurun_out/abe_$i.err)"; case $rc in 0) ;; *) exit $rc;; esac
done
