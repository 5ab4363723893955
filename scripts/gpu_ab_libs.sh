# Interleaved A/B of library variants x one env knob on the bench line:
#   gpurun -- bash scripts/gpu_ab_libs.sh <out> "<lib1.so|product> ..." <VAR> "<v1 v2 ...>" <rounds> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; LIBS=$2; VAR=$3; VALS=$4; R=$5; shift 5
mkdir -p $O
for r in $(seq $R); do
  for lib in $LIBS; do
    for v in $VALS; do
      if [ "$lib" = product ]; then L=""; else L=$lib; fi
      env PGHIP_LIB=$L $VAR=$v timeout -k 10 240 python bench.py --no-cpu-baseline --no-tp-curve "$@" > $O/run.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
      python -c "
import json,sys; o=json.loads(open('$O/run.json').read().strip().splitlines()[-1])
print(json.dumps({'lib': '$lib'.split('/')[-1], '$VAR': '$v', 'round': $r, 'decode_ms': o['decode_ms_per_token'], 'prefill_ms': o['prefill_ms'], 'value': o['value'], 'hbm': o['decode_hbm_frac']}))" | tee -a $O/ab.jsonl
    done
  done
done
