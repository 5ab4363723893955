# batched decode (pt-448 x16): attention combine + split size sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/b16.tests.log 2>&1
rc=$?; tail -2 gpurun_out/b16.tests.log; [ $rc -eq 0 ] || exit 1
for t in 1024 256 128 64; do
  timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-target $t > gpurun_out/b16_$t.log 2>&1 || exit 1
  echo "target $t: $(tail -1 gpurun_out/b16_$t.log | cut -c1-150)"
done
