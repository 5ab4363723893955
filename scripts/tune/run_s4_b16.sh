# argmax / engine GPU tests, then the pt-448 x16 decode step over split-KV targets
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_tp_gpu.py -q -x -m "gpu and not slow" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s4d.tests.log 2>&1
rc=$?; tail -3 gpurun_out/s4d.tests.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/s4d.log
for t in 256 512 1024; do
  timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-target $t >> gpurun_out/s4d.log 2>&1 || exit 1
done
timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 >> gpurun_out/s4d.log 2>&1
