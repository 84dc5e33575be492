# PMC counter passes for the fingerprint kernel (one --pmc group per run; no tracing domains).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/${TAG}
if [ -n "$LIST" ]; then rocprofv3 -L > gpurun_out/${TAG}/counters.txt 2>&1; echo "list rc=$?"; fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "fingerprint(8k)?_kernel" --output-format csv -d gpurun_out/${TAG}/p$i -o run -- python3 bench.py --no-match --no-cpu --no-strong --steps 3 --warmup 1 > gpurun_out/${TAG}/p$i.log 2>&1; rc=$?
  echo "pass $i [$grp] rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
