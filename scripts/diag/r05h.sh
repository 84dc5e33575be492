# Round 5: the bin sort with per-workgroup segment stats; directory scale A/B (TFP_DIR_SCALE 0 / 1
# builds against the default 2) on the C3 coefs=2 sweeps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05h
TESTS="tests/test_gpu_sweep_clusters.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for t in 0.001 0.45; do
  for v in base ds0 ds1; do
    if [ $v = base ]; then L=""; else L=$A/$v/libtiresias_fp.so; fi
    TFP_LIB_PATH=$L timeout -k 10 300 python3 scripts/diag/c3_sweep.py 2 $t 9 > gpurun_out/${R}_one.txt 2>&1 || exit 4
    sed "s/^/$v /" gpurun_out/${R}_one.txt | grep -v amdgpu.ids >> gpurun_out/${R}_c3.txt
  done
done
cat gpurun_out/${R}_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_wide_trace -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 5 > gpurun_out/${R}_wide_trace.log 2>&1; rc=$?; echo "wide trace rc=$rc"; exit $rc
