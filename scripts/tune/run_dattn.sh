# decode attention K ring (default build) vs the previous one-block form (var_base.so): B=1, 16, 32
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/da.tests.log 2>&1
rc=$?; tail -2 gpurun_out/da.tests.log; [ $rc -eq 0 ] || exit 1
for lib in pghip/libpghip.so ../scripts/tune/var_base.so; do
  L=paligemma-multimodal-system_amd/$lib
  PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config pt-224 --batch 1 --steps 100 > gpurun_out/da.log 2>&1 || exit 1
  echo "$lib B=1: $(tail -1 gpurun_out/da.log | cut -c90-140)"
  PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 > gpurun_out/da.log 2>&1 || exit 1
  echo "$lib B=16: $(tail -1 gpurun_out/da.log | cut -c90-140)"
  PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config pt-896 --batch 32 --steps 20 --fp8 > gpurun_out/da.log 2>&1 || exit 1
  echo "$lib B=32: $(tail -1 gpurun_out/da.log | cut -c90-140)"
done
