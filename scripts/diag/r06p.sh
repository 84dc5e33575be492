# Round 6: cache builds with one key box per thread when its rows share a key index, sparse points
# written where they fall (dense ones staged in LDS): cache / index / sweep / configs
# tests, the first coefs = 2 searches at new tolerances under a kernel trace, then C3 coefs 2 and
# batch-1 against the committed sweep (abv/r06base).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06p
timeout -k 10 900 python -u -m pytest tests/test_gpu_cellcache.py tests/test_gpu_index.py tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${R}_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_newtol -o nt -- python3 scripts/diag/c2_newtol.py > gpurun_out/${R}_newtol.log 2>&1; rc=$?; echo "newtol rc=$rc"; grep -E "^tol|^cache" gpurun_out/${R}_newtol.log; [ $rc = 0 ] || exit $rc
S="2:0.001 2:0.01 2:0.1 2:0.45"
for rep in 1 2; do
  for v in r06base new; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_multi.py 9 $S > gpurun_out/${R}_one.txt 2>&1 || { cat gpurun_out/${R}_one.txt; exit 4; }
    grep coefs gpurun_out/${R}_one.txt >> gpurun_out/${R}_c3.txt
    TAG=$v TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c2_alt.py 200 > gpurun_out/${R}_alt.txt 2>&1 || { cat gpurun_out/${R}_alt.txt; exit 5; }
    grep batch-1 gpurun_out/${R}_alt.txt >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
