# fp8 path: kernel + engine tests, then the pt-896 x32 fp8 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m "gpu and not slow" > gpurun_out/fp8t.log 2>&1
rc=$?; tail -3 gpurun_out/fp8t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --fp8 > gpurun_out/b896_fp8.log 2>&1 && tail -1 gpurun_out/b896_fp8.log | cut -c1-1200
