# fused attention + o_proj (pg_attn_oproj): engine/drop-in GPU tests, then the decode step time
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_dropin_gpu.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/ao.tests.log 2>&1
rc=$?; tail -3 gpurun_out/ao.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python scripts/tune/decode_step.py > gpurun_out/ao.log 2>&1 && cut -c1-200 gpurun_out/ao.log
