# Round 6: the clip sweep's batch groups from a DPP-reduced mask of their starts (the tree) against
# the binary lifting (abv/base = the committed tree) at C3, kernel traces, then GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06as
S="1:0.001 2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in base new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
for v in base new; do
  L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
  export TFP_LIB_PATH=$L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace_$v -o t -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_trace_$v.log 2>&1 || { tail gpurun_out/${R}_trace_$v.log; exit 5; }
done
unset TFP_LIB_PATH
for v in base new; do grep -h "wide_clips" gpurun_out/${R}_trace_$v/t_kernel_stats.csv | cut -d, -f1-5 | sed "s/^/$v /"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py tests/test_gpu_cellcache.py tests/test_gpu_parity.py tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${R}_pytest.log; exit $rc
