# Round 5: wide_bin_sort's duration with and without its sorts (scripts/diag/r05_ablate.py
# binsort_nosort: the batch is redone with the library sort, only the kernel's own time counts).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=r05o
A=$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv
for v in base binsort_nosort; do
  TFP_LIB_PATH=$A/$v/libtiresias_fp.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${R}_$v -o c3 -- python3 scripts/diag/c3_sweep.py 2 0.001 3 > gpurun_out/${R}_$v.log 2>&1; rc=$?; echo "$v rc=$rc"; [ $rc = 0 ] || exit $rc
done
