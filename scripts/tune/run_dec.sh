# decode step timing for a few engine knobs (+ the GPU engine tests first)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dropin_gpu.py -q -m "gpu and not slow" -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/dec.tests.log 2>&1
rc=$?; tail -3 gpurun_out/dec.tests.log; [ $rc -eq 0 ] || exit 1
OUT=gpurun_out/dec.log
: > $OUT
for a in "" "--split-keys 64" "--split-o 1" "--split-o 4"; do
  timeout -k 10 240 python scripts/tune/decode_step.py $a >> $OUT 2>> gpurun_out/dec.err || exit 1
done
cut -c1-200 $OUT
