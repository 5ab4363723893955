# batched decode: fused attention (pg_attn_decode) vs split kernel + combine, interleaved (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abf}; mkdir -p $O
for rnd in 1 2; do
  for cfg in "pt-448 16" "pt-224 16"; do
    set -- $cfg
    for mr in 2 99; do
      PG_FUSED_MIN_ROUNDS=$mr timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 2 --warmup 1 --no-cpu-baseline > $O/r.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
      python -c "import json; d=json.load(open('$O/r.json')); print('$1 x$2 min_rounds=$mr decode', d['decode_ms_per_token'], 'prefill', d['prefill_ms'])"
    done
  done
done
