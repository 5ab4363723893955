# A/B in one call: 12-wave flash attention (product) vs 8-wave (var_now12.so): attention shapes + pt-448 x16 prefill
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/tune/attn_bench.py --only gemma448x16,gemma896x32 > gpurun_out/s4j.attn.log 2>&1 || exit 1
PGHIP_LIB=scripts/tune/var_now12.so timeout -k 10 300 python scripts/tune/attn_bench.py --only gemma448x16,gemma896x32 > gpurun_out/s4j.attn8.log 2>&1 || exit 1
for v in prod now12 prod now12; do
  if [ $v = prod ]; then L=""; else L=scripts/tune/var_now12.so; fi
  PGHIP_LIB=$L timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/s4j.$v.json 2> gpurun_out/s4j.$v.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/s4j.$v.json')); print('$v', d['prefill_ms'], d['prefill_mfma_frac'])"
done
grep -h gemma gpurun_out/s4j.attn.log gpurun_out/s4j.attn8.log
