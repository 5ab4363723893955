# attention kernel tests (12-wave flash path) + pt-448 x16 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s4i.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4i.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s4i.b448.json 2> gpurun_out/s4i.b448.err || { tail -20 gpurun_out/s4i.b448.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/s4i.b448.json')); print(d['value'], d['prefill_ms'], d['prefill_mfma_frac'], d['decode_ms_per_token'])"
timeout -k 10 300 python scripts/tune/attn_bench.py > gpurun_out/s4i.attn.log 2>&1; tail -12 gpurun_out/s4i.attn.log
