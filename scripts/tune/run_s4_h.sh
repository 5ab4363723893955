# bench with the captured prefill (pt-224 twice, eager-prefill once) and pt-448 x16
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s4h.b224_$i.json 2> gpurun_out/s4h.b224_$i.err || { tail -20 gpurun_out/s4h.b224_$i.err; exit 1; }
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager-prefill > gpurun_out/s4h.b224e.json 2> gpurun_out/s4h.b224e.err || exit 1
timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s4h.b448.json 2> gpurun_out/s4h.b448.err || { tail -20 gpurun_out/s4h.b448.err; exit 1; }
grep -h "capture failed" gpurun_out/s4h.*.err
for f in gpurun_out/s4h.*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['prefill_ms'], d['prefill_mfma_frac'], d['decode_ms_per_token'], d['config'].get('prefill'))"; done
