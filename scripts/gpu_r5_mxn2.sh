# round 5: MX norms after the row-factor prologue loads (tests + timelines + pt-896 x32 fp8 decode A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-mxn}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "${SEL:-mx_ or gemv8 or gemm8 or fp8}" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -6; [ $rc -eq 0 ] || exit 1
CASES="mx1|PG_MX_NORM=1|--config pt-896 --batch 32 --fp8;mx0|PG_MX_NORM=0|--config pt-896 --batch 32 --fp8" bash scripts/gpu_timeline.sh ${1:-mxn}/tl || exit 1
for r in 1 2 3; do
  for m in 1 0; do
    PG_MX_NORM=$m timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"mx_norm\": $m, /" | tee -a $O/decode896.jsonl || exit 1
  done
done
