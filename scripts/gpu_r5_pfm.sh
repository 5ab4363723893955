# round 5: in-kernel prefill key-split merge (tests + prefill A/B vs PG_PF_MERGE=0) and the Infinity Cache probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pfm}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "${SEL:-attention or attn or prefill or pt224}" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in "" scripts/tune/libs/pfm0.so; do
    PGHIP_LIB=$lib timeout -k 10 200 python scripts/tune/prefill_ms.py 2>> $O/err.log | tee -a $O/prefill.jsonl || exit 1
  done
done
bash scripts/gpu_mall_probe.sh ${1:-pfm}/mall
