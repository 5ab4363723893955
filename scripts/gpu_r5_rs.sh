# q|k|v fp8 GEMV row split: fp8 tests (kernel, tiny engine, full-size pt-896) + pt-896 x32 decode A/B (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rs}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_large_gpu.py -k "gemv8 or mx_ or fp8" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "emulated" $O/tests.log | head -3; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in "" scripts/tune/libs/rsq.so; do
    PGHIP_LIB=$lib timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | tee -a $O/decode.jsonl || exit 1
  done
done
