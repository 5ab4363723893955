# row-block tails with their own split: tests, prefill A/B (PG_TAIL_SPLIT), full-size greedy ids with / without row blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4u.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4u.tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PG_ROW_BLOCKS_GU=$v timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/s4u.$v.json 2> gpurun_out/s4u.$v.err || { tail -20 gpurun_out/s4u.$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s4u.$v.json')); print('row_blocks_gu=$v', d['prefill_ms'], d['prefill_mfma_frac'])"
done
for v in 1 0; do
  PG_ROW_BLOCKS=$v timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 20 > gpurun_out/s4u.ids$v 2>&1 || { tail -5 gpurun_out/s4u.ids$v; exit 1; }
  echo "row_blocks=$v $(tail -1 gpurun_out/s4u.ids$v | grep -o '"ids16".*')"
done
