# prefill tuning on the product build (gpurun_out/$1): small-GEMM tile / split sweep and batch-1 prefill time;
# with PGHIP_LIB set, the same on a variant build first checked by the kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tune}; mkdir -p $O
if [ -n "$PGHIP_LIB" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_variant.log 2>&1
  rc=$?; tail -n 3 $O/tests_variant.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 400 python scripts/tune/small_gemm_sweep.py > $O/sweep.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/tune/prefill_time.py > $O/prefill.txt 2>&1 || exit 1
tail -n 2 $O/prefill.txt
