# Full default bench (configs[1] fingerprint + configs[2] match) and a 2-rank rehearsal of the
# sharded path on the single GPU (gloo stands in for RCCL there).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/full_bench.err; cat gpurun_out/full_bench.json; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --clips 256 --db-clips 20000 --queries 1024 --latency-queries 5 --stream-channels 64 --stream-ticks 20 --dist-backend gloo > gpurun_out/dist2_bench.json 2> gpurun_out/dist2_bench.err; rc=$?; echo "dist2 rc=$rc"; tail -3 gpurun_out/dist2_bench.err; cat gpurun_out/dist2_bench.json
