set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/tune/gemm_bench.py > gpurun_out/s4_gemm.log 2>&1
rc=$?; cat gpurun_out/s4_gemm.log; exit $rc
