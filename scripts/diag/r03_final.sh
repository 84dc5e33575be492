# Round-3 evidence on the final build: the GPU check (tests, smoke, bench), the 2-rank gloo rehearsal
# of the sharded bench on the one GPU, the bench under a kernel
# trace with the fingerprint kernel's HBM PMC (profile_round.sh), and the coefs=2 general path at C3
# tol 0.001 (kernel trace, then FETCH_SIZE / WRITE_SIZE of the wide_* kernels in separate passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${R:-r03ae}
TAG=$R bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --clips 256 --db-clips 20000 --queries 1024 --latency-queries 20 --stream-channels 64 --stream-ticks 20 --dist-backend gloo > gpurun_out/${R}_dist2.json 2> gpurun_out/${R}_dist2.err; rc=$?; echo "dist2 rc=$rc"; tail -2 gpurun_out/${R}_dist2.err; [ $rc = 0 ] || exit $rc
R=$R bash scripts/profile_round.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; tail -1 gpurun_out/${R}_wide_trace.log; [ $rc = 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "wide_" --output-format csv -d gpurun_out/${R}_wide_pmc_$c -o run -- python3 scripts/diag/c3_sweep.py 2 0.001 3 > gpurun_out/${R}_wide_pmc_$c.log 2>&1; rc=$?; echo "wide pmc $c rc=$rc"; [ $rc = 0 ] || exit $rc
done
