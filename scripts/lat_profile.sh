# Batch-1 search latency: plain run, then under rocprofv3 hip+kernel trace (API and kernel stats).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-lat}
timeout -k 10 300 python scripts/lat_probe.py ${ARGS} > gpurun_out/${T}.txt 2>&1; rc=$?; cat gpurun_out/${T}.txt | tail -2; case $rc in 0) ;; *) exit $rc;; esac
if [ -n "$PROF" ]; then
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 scripts/lat_probe.py ${ARGS} > gpurun_out/${T}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/${T}_prof.log
fi
