# round 5: MX norms (tests + pt-896 x32 fp8 decode A/B) and the in-kernel prefill split merge (tests + A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-mxn}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py \
  -k "${SEL:-mx_ or gemv8 or gemm8 or fp8 or attention or attn or key_split or pt224}" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -15; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for m in 1 0; do
    PG_MX_NORM=$m timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"mx_norm\": $m, /" | tee -a $O/decode896.jsonl || exit 1
  done
done
for r in 1 2 3; do
  for lib in "" scripts/tune/libs/pfm0.so; do
    PGHIP_LIB=$lib timeout -k 10 200 python scripts/tune/prefill_ms.py 2>> $O/err.log | tee -a $O/prefill.jsonl || exit 1
  done
done
