# Round-4 GPU check on the tree as committed (256-query chunks, waves per chunk scaled): coefs=2
# parity, smoke, bench, the waves-per-chunk A/B, then the coefs=2 C3 per-kernel trace and
# FETCH/WRITE passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r04l
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_sweep_clusters.py tests/test_gpu_parity.py -x -q -m gpu -k "sweep or coefs2 or timed or updated or cluster or speculative" --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?
echo "parity rc=$rc $(tail -1 gpurun_out/${R}_pytest.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${R}_bench.err; [ $rc = 0 ] || exit $rc
for tol in 0.001 0.45; do
  timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 2>/dev/null | sed "s/^/[xw auto] /" || exit 5
  TFP_CLIP_XW=1024 timeout -k 10 300 python scripts/diag/c3_sweep.py 2 $tol 5 2>/dev/null | sed "s/^/[xw 1024] /" || exit 6
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; [ $rc = 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "wide_" --output-format csv -d gpurun_out/${R}_wide_pmc_$c -o run -- python3 scripts/diag/c3_sweep.py 2 0.001 3 > gpurun_out/${R}_wide_pmc_$c.log 2>&1; rc=$?; echo "wide pmc $c rc=$rc"; [ $rc = 0 ] || exit $rc
done
