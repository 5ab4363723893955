# fp8 lm_head with 4 tiles per wave: tests + pt-896 x32 decode A/B vs PG_GEMV8_NT4=0 (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-nt4}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "gemv8 or mx_ or fp8" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in "" scripts/tune/libs/nt4off.so; do
    PGHIP_LIB=$lib timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | tee -a $O/decode.jsonl || exit 1
  done
done
