# Round 5: the GPU suite on the tree, C2 A/B of the hoisted table reads' placement (all: before the
# syncs; all2 = the tree: after them), then the bench with the new legs.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05c
TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for r in 1 2 3; do
  for v in base all all2; do
    TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_ab.txt 2>&1 || exit 4
  done
done
grep "fp C2" gpurun_out/${R}_ab.txt
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -8 gpurun_out/${R}_bench.err; exit $rc
