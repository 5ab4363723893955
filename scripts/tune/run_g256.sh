set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/g256.tests.log 2>&1
rc=$?; tail -3 gpurun_out/g256.tests.log; [ $rc -eq 0 ] || exit 1
echo "== prefetch"; timeout -k 10 200 python scripts/tune/gemm_bench.py && \
echo "== base" && PGHIP_LIB=scripts/tune/var_nopf.so timeout -k 10 200 python scripts/tune/gemm_bench.py
