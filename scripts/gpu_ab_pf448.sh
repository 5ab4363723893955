# pt-448 x16 prefill A/B over library variants (gpurun_out/$1): product, then each PGHIP_LIB given
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab448}; mkdir -p $O; shift
for rnd in 1 2; do
  timeout -k 10 300 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/product_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/product_$rnd.json')); print('product', d['prefill_ms'])"
  for v in "$@"; do
    PGHIP_LIB=$v timeout -k 10 300 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/$(basename $v .so)_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$(basename $v .so)_$rnd.json')); print('$v', d['prefill_ms'])"
  done
done
