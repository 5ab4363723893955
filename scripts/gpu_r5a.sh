# round 5: fixed-point decode residual + configs[4] at its shape (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_dropin_gpu.py \
  -k "${SEL:-fx or bit_reproducible or pt224_free_running or end_to_end}" \
  > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40; [ $rc -eq 0 ] || exit 1
for m in fx both fx both; do
  PG_DECODE_ADD=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-tp-curve > $O/bench_$m.json 2>> $O/bench.err || exit 1
  python -c "import json,sys;o=json.load(open('$O/bench_$m.json'));print('$m',o['decode_ms_per_token'],o['decode_hbm_frac'],o['prefill_ms'])"
done
