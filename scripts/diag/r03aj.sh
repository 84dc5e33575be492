# Enrol-then-first-search at 100k clips: the index-merge timings the engine logs (TFP_DEBUG_INDEX)
# and a kernel trace of the same bench leg, to split the 1.7 ms between host and kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TFP_DEBUG_INDEX=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03aj_trace -o b -- python3 bench.py --no-cpu --no-strong --no-sweeps --steps 3 --warmup 1 --stream-ticks 5 > gpurun_out/r03aj_bench.json 2> gpurun_out/r03aj_bench.err; rc=$?; echo "bench rc=$rc"; grep -E "enrol|index merge|full build" gpurun_out/r03aj_bench.err | tail -24; exit $rc
