# Round 5: fingerprint8k_kernel<4> variants: filterbank weights as one ds_read_b128 per two step
# pairs (w128), inline edge fetches for throughput launches too (w128inl), PCM loaded straight
# into registers by buffer loads (dpcm). Exactness of each against the oracle (fp_variant_check),
# then C2 and C3-shaped (4096 x 5 s) launches interleaved. Then the tree (w128 + the sweep's
# per-segment constants table, segc): its sweep tests, and C3 coefs=2 timing against all2.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05d
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for v in all2 w128 w128inl dpcm dpcmp; do
  TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_variant_check.py >> gpurun_out/${R}_check.txt 2>&1 || exit 3
done
grep -v amdgpu.ids gpurun_out/${R}_check.txt
for r in 1 2 3; do
  for v in all2 w128 dpcm dpcmp; do
    TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_ab.txt 2>&1 || exit 4
    FP_CLIPS=4096 FP_SECONDS=5 TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 120 python scripts/diag/fp_c2.py >> gpurun_out/${R}_ab.txt 2>&1 || exit 4
  done
done
grep "fp " gpurun_out/${R}_ab.txt
TESTS="tests/test_gpu_sweep_clusters.py tests/test_gpu_configs.py::test_configs2_sweeps_vs_sorted_oracle" TAG=$R bash scripts/gpu_tests.sh; rc=$?; [ $rc = 0 ] || exit $rc
for v in all2 segc all2 segc; do
  echo "[$v]" >> gpurun_out/${R}_c3.txt
  TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 300 python scripts/diag/c3_sweep.py 2 0.001 7 >> gpurun_out/${R}_c3.txt 2>&1 || exit 5
done
grep -v amdgpu.ids gpurun_out/${R}_c3.txt
