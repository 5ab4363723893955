# round 5: MX decode MLP rows (tests + pt-896 x32 fp8 decode A/B) and the pending prefill / lm_head A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-mx}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py \
  -k "${SEL:-mx_h or gemv8 or gemm8 or fp8 or quant}" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for m in 1 0; do
    PG_MX_H=$m timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"mx\": $m, /" | tee -a $O/decode896.jsonl || exit 1
  done
done
[ -n "$SKIP_AB2" ] && exit 0
bash scripts/gpu_r5_ab2.sh ${1:-mx}/ab2
