set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_engine_gpu.py tests/test_dropin_gpu.py -q -m "gpu and not slow" -p no:cacheprovider -x > gpurun_out/v7.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/v7.tests.log; [ $rc -eq 0 ] || exit 1
OUT=gpurun_out/v7.variants.log
: > $OUT
timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/v7.err || exit 1
cat $OUT
bash scripts/tune/prof_decode.sh v7p
