# wide_clips with the used keys' segment constants hoisted (TFP_CLIP_KEYPRE): coefs=2 parity at C3,
# then C3 timing against the build without it (nokp), interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_sweep_clusters.py -x -q -m gpu -k "sweep or coefs2 or timed or updated or cluster" --timeout 300 --timeout-method thread > gpurun_out/r04j_pytest.log 2>&1; rc=$?
echo "parity rc=$rc $(tail -1 gpurun_out/r04j_pytest.log)"; [ $rc = 0 ] || exit $rc
TOLS="0.001 0.01 0.45" bash scripts/diag/ab_wide_t.sh base nokp wpre grp base nokp wpre grp > gpurun_out/r04j_ab.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r04j_ab.txt; exit $rc
