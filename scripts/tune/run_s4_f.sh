set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4f.tests.log 2>&1
rc=$?; tail -3 gpurun_out/s4f.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/tune/gemm_bench.py > gpurun_out/s4f_gemm.log 2>&1
rc=$?; cat gpurun_out/s4f_gemm.log; exit $rc
