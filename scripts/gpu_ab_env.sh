# Interleaved A/B of one environment knob on the bench line:
#   gpurun -- bash scripts/gpu_ab_env.sh <out> <VAR> "<v1 v2 ...>" <rounds> [bench args...]
# prints decode ms/token, prefill ms and tokens/s per run (gpurun_out/<out>/ab.jsonl)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; VAR=$2; VALS=$3; R=$4; shift 4
mkdir -p $O
for r in $(seq $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 240 python bench.py --no-cpu-baseline --no-tp-curve "$@" > $O/run.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "
import json,sys; o=json.loads(open('$O/run.json').read().strip().splitlines()[-1])
print(json.dumps({'$VAR': '$v', 'round': $r, 'decode_ms': o['decode_ms_per_token'], 'prefill_ms': o['prefill_ms'], 'value': o['value'], 'hbm': o['decode_hbm_frac']}))" | tee -a $O/ab.jsonl
  done
done
