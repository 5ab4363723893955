# batched decode: split-KV target (keys per split) A/B at pt-448 x16 and pt-224 x16 (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-splt}; mkdir -p $O
for rnd in 1 2; do
  for t in 1024 512 256; do
    timeout -k 10 300 python scripts/tune/bench_knob.py DECODE_SPLIT_TARGET=$t -- --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 32 --no-cpu-baseline > $O/d448_${t}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    timeout -k 10 300 python scripts/tune/bench_knob.py DECODE_SPLIT_TARGET=$t -- --config pt-224 --batch 16 --steps 2 --warmup 1 --gen-tokens 32 --no-cpu-baseline > $O/d224_${t}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; a=json.load(open('$O/d448_${t}_$rnd.json')); b=json.load(open('$O/d224_${t}_$rnd.json')); print('target $t pt448x16 decode', a['decode_ms_per_token'], 'pt224x16 decode', b['decode_ms_per_token'])"
  done
done
