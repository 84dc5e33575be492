# Round 6: the key pass's segment stats by each frame's own lane (the tree) against one segment a
# step per wave (abv/k0) at C3, then the sweep's GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06ab
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in k0 new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_cellcache.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/${R}_pytest.log; exit $rc
