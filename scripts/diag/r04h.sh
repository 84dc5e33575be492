# Index delta with carried bitsets (tests + the bench's enrol leg), then the round-4 profiles
# (bench kernel trace, fingerprint HBM and SQ PMC, coefs=2 C3 kernel trace + FETCH/WRITE).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_configs.py -x -q -m gpu -k "index or updated" --timeout 300 --timeout-method thread > gpurun_out/r04h_pytest.log 2>&1; rc=$?
echo "index tests rc=$rc $(tail -1 gpurun_out/r04h_pytest.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu --no-strong --no-sweeps --steps 3 --warmup 1 --stream-ticks 5 > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err; rc=$?
echo "bench rc=$rc"; grep -E "enrol" gpurun_out/r04h_bench.err | tail -3; [ $rc = 0 ] || exit $rc
R=r04 bash scripts/profile_r04.sh
