# A/B of the fingerprint kernel's register budget (2 vs 3 waves/SIMD), built and timed on the box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for w in 2 3; do
  make -s -C asterisk-tiresias_amd clean && make -s -j16 -C asterisk-tiresias_amd FP_WAVES=$w > /dev/null 2>&1 || exit 3
  timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "fingerprint or device or golden" > gpurun_out/ab_w${w}_pytest.log 2>&1; rc=$?; echo "w=$w pytest rc=$rc $(tail -1 gpurun_out/ab_w${w}_pytest.log)"; case $rc in 0|1) ;; *) exit $rc;; esac
  timeout -k 10 300 python bench.py --no-match --no-cpu --steps 30 --warmup 3 > gpurun_out/ab_w${w}.json 2> gpurun_out/ab_w${w}.err; rc=$?; echo "w=$w bench rc=$rc"; grep "fingerprint:" gpurun_out/ab_w${w}.err; case $rc in 0) ;; *) exit $rc;; esac
done
