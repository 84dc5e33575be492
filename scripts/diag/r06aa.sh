# Round 6: the clip sweep's uniform-lane shuffles as readlane (abv/rl), its lane scans through DPP
# (abv/dpp), and windows in blocks of 4 (the tree) against the committed tree (abv/base) at C3, then the sweep's GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06aa
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in base rl dpp new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_cellcache.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/${R}_pytest.log; exit $rc
