# Round 6: the GPU tests of this round's changes (groups, caches, sweep paths, configs), then the
# software-pipelined fingerprint loop (abv/pipe: -DTFP_FP8_PIPE=1) against the tree's build:
# configs[1] parity and interleaved C2 launch timings.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r06e
TESTS="tests/test_gpu_sweep_clusters.py tests/test_gpu_group.py tests/test_gpu_cellcache.py tests/test_gpu_concurrency.py tests/test_gpu_device.py tests/test_gpu_index.py" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
TAG=${R}_ab bash scripts/ab_libs.sh base pipe; rc=$?; [ $rc = 0 ] || exit $rc
for v in base pipe; do
  L=""; [ $v != base ] && L=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$v/libtiresias_fp.so
  TFP_LIB_PATH=$L FP_CLIPS=4096 FP_SECONDS=5 timeout -k 10 120 python3 scripts/diag/fp_c2.py 40 2>&1 | grep -v amdgpu.ids
done
