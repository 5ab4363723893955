# SigLIP ragged-N GEMMs as column blocks: tests, then prefill A/B (PG_COL_BLOCKS) at pt-448 x16 and pt-896 x32
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4p.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4p.tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PG_COL_BLOCKS=$v timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/s4p.$v.json 2> gpurun_out/s4p.$v.err || { tail -20 gpurun_out/s4p.$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s4p.$v.json')); print('pt-448 col_blocks=$v', d['prefill_ms'], d['prefill_mfma_frac'])"
done
for v in 1 0; do
  PG_COL_BLOCKS=$v timeout -k 10 600 python bench.py --config pt-896 --batch 32 --steps 1 --warmup 1 --gen-tokens 8 --fp8 --no-cpu-baseline > gpurun_out/s4p.896_$v.json 2> gpurun_out/s4p.896_$v.err || { tail -20 gpurun_out/s4p.896_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s4p.896_$v.json')); print('pt-896 col_blocks=$v', d['prefill_ms'], d['prefill_mfma_frac'])"
done
