# flash attention: two 16-row groups per wave (default build) vs one (var_rpw1.so); tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/fa.tests.log 2>&1
rc=$?; tail -2 gpurun_out/fa.tests.log; [ $rc -eq 0 ] || exit 1
echo "== rpw2"; timeout -k 10 200 python scripts/tune/attn_bench.py && \
echo "== rpw1" && PGHIP_LIB=scripts/tune/var_rpw1.so timeout -k 10 200 python scripts/tune/attn_bench.py
