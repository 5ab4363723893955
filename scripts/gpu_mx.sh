# round 6: MX prefill h -- kernel / engine fp8 tests, then the configs[4] bench line with PG_MX_PREFILL=1 / 0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-mx6}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "mx or fp8 or gemv8" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40; [ $rc -eq 0 ] || exit 1
for m in 1 0; do
  PG_MX_PREFILL=$m timeout -k 10 400 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline --no-tp-curve \
    --steps 2 --warmup 1 > $O/bench_mx$m.json 2>> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python -c "import json;o=json.load(open('$O/bench_mx$m.json'));print('MX_PREFILL=$m', o['prefill_ms'], o['decode_ms_per_token'], o['value'])"
done
