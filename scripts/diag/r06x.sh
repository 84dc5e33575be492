# Round 6: the directory's runs up to 256 buckets by their own lane (16-byte stores), on top of
# r06v: per-phase wave clocks (abv/clk), C3 A/B against the committed tree (abv/pre), then the
# sweep's GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06x
TFP_LIB_PATH=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/clk/libtiresias_fp.so TFP_TEST_KNOBS=1 TFP_DEBUG_BINS=1 timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 0.001 1 > gpurun_out/${R}_bins.log 2>&1 || { tail -20 gpurun_out/${R}_bins.log; exit 3; }
grep -E "bin sort waves|cycles" gpurun_out/${R}_bins.log | tail -13
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in pre new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/${R}_pytest.log; exit $rc
