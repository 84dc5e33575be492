# Edge passes of the throughput fingerprint kernel with a 16-byte fast path (TFP_FP_CHECKED_FAST) and
# the spread part_max: parity, then C2 and C3 timing against the previous edge fetch (oldedge).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OLD=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/oldedge/libtiresias_fp.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_sweep_clusters.py -x -q -m gpu -k "configs1 or fingerprint or golden or sweep or timed or cluster" --timeout 300 --timeout-method thread > gpurun_out/r04m_pytest.log 2>&1; rc=$?
echo "parity rc=$rc $(tail -1 gpurun_out/r04m_pytest.log)"; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 python scripts/diag/fp_c2.py 2>/dev/null | sed "s/^/[new] /" || exit 4
  TFP_LIB_PATH=$OLD timeout -k 10 120 python scripts/diag/fp_c2.py 2>/dev/null | sed "s/^/[old] /" || exit 5
  for c in 1 2; do
    timeout -k 10 300 python scripts/diag/c3_sweep.py $c 0.001 5 2>/dev/null | sed "s/^/[new] /" || exit 6
    TFP_LIB_PATH=$OLD timeout -k 10 300 python scripts/diag/c3_sweep.py $c 0.001 5 2>/dev/null | sed "s/^/[old] /" || exit 7
  done
done
