# gemm256: staggered wave groups (var_stagger.so) vs default; correctness first (GEMM + engine tests on the variant)
set -o pipefail
cd $GRAFT_REPO_ROOT
PGHIP_LIB=scripts/tune/var_stagger.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -m "gpu" -k "gemm or prefill or parity" > gpurun_out/stg.tests.log 2>&1
rc=$?; tail -2 gpurun_out/stg.tests.log; [ $rc -eq 0 ] || exit 1
echo "== stagger"; PGHIP_LIB=scripts/tune/var_stagger.so timeout -k 10 200 python scripts/tune/gemm_bench.py && \
echo "== default" && timeout -k 10 200 python scripts/tune/gemm_bench.py
