# Round 5, first GPU call: the -m gpu suite on the pruned tree (key-major sweep and the 12-wave
# fingerprint form removed, test knobs behind TFP_TEST_KNOBS), then the fingerprint phase-cost
# ablations of scripts/diag/r05_ablate.py (C2 launch, interleaved with the unmodified HEAD build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05a
TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for r in 1 2; do
  for v in base nosqrtfix noconst nologs nofb norare notrans nobperm base; do
    TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_abl.txt 2>&1 || exit 4
  done
done
grep "fp C2" gpurun_out/${R}_abl.txt
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${R}_bench.err; exit $rc
