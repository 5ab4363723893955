set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "attention" > gpurun_out/attn.tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn.tests.log; [ $rc -eq 0 ] || exit 1
echo "== fa"; timeout -k 10 120 python scripts/tune/attn_bench.py && \
echo "== old" && PGHIP_LIB=scripts/tune/var_nofa.so timeout -k 10 120 python scripts/tune/attn_bench.py
