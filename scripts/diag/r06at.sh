# Round 6 evidence (final tree: the DPP group mask), call 1: the whole GPU suite, smoke and the default bench (scripts/gpu_check.sh),
# then the 2-rank gloo rehearsal of the sharded path on the one GPU.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06at bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --clips 256 --db-clips 20000 --queries 1024 --latency-queries 20 --stream-channels 64 --stream-ticks 20 --dist-backend gloo > gpurun_out/r06at_dist2.json 2> gpurun_out/r06at_dist2.err; rc=$?; echo "dist2 rc=$rc"; tail -3 gpurun_out/r06at_dist2.err; exit $rc
