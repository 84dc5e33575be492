# A/B of prebuilt library variants (built in the container: scripts/build_variant.sh NAME FLAGS ->
# asterisk-tiresias_amd/abv/NAME/libtiresias_fp.so). For each NAME ("base" = lib/): configs[1]
# parity, then the C2 fingerprint leg twice, interleaved over the variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-abl}
mkdir -p gpurun_out/$TAG
libof() { [ "$1" = base ] && echo "" || echo "$GRAFT_REPO_ROOT/asterisk-tiresias_amd/abv/$1/libtiresias_fp.so"; }
for n in "$@"; do
  TFP_LIB_PATH=$(libof $n) timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k "configs1" --timeout 240 --timeout-method thread > gpurun_out/$TAG/test_$n.log 2>&1; rc=$?
  echo "[$n] parity rc=$rc $(tail -1 gpurun_out/$TAG/test_$n.log)"; [ $rc = 0 ] || exit $rc
done
for rep in 1 2 3; do
  for n in "$@"; do
    TFP_LIB_PATH=$(libof $n) timeout -k 10 300 python bench.py --no-match --no-cpu --no-strong --steps 30 > gpurun_out/$TAG/bench_$n.$rep.json 2> gpurun_out/$TAG/bench_$n.$rep.err; rc=$?
    echo "[$n] rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_$n.$rep.json'));print('%.4f ms/step, kernel %.4f ms' % (d['ms_per_step'], d['roofline']['avg_launch_ms']))")"; [ $rc = 0 ] || exit $rc
  done
done
