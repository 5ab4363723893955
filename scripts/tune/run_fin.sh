set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "finalize or qkv_rope or gemm" > gpurun_out/fin.tests.log 2>&1
rc=$?; tail -3 gpurun_out/fin.tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_check3.sh
