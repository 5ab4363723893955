# row-block split of ragged fp32-slab GEMMs: kernel + engine tests, then pt-448 x16 prefill A/B (PG_ROW_BLOCKS)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4o.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4o.tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PG_ROW_BLOCKS=$v timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/s4o.$v.json 2> gpurun_out/s4o.$v.err || { tail -20 gpurun_out/s4o.$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s4o.$v.json')); print('row_blocks=$v', d['prefill_ms'], d['prefill_mfma_frac'])"
done
