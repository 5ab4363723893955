# flash-attention change vs the previous commit's library (scripts/tune/fa_head.so): attention kernel tests,
# attn_bench twice interleaved, pt-448 x16 prefill (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-faab2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tk.log 2>&1; tail -2 $O/tk.log; grep -q " passed" $O/tk.log && ! grep -q failed $O/tk.log || exit 1
for rnd in 1 2; do
  for v in product fa_head; do
    L=""; [ $v = product ] || L=scripts/tune/$v.so
    PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/attn_bench.py > $O/ab_${v}_$rnd.txt 2>&1 || { tail -3 $O/ab_${v}_$rnd.txt; exit 1; }
    echo "== $v $rnd"; grep '^[gs]' $O/ab_${v}_$rnd.txt
  done
done
for rnd in 1 2; do
  for v in product fa_head; do
    L=""; [ $v = product ] || L=scripts/tune/$v.so
    PGHIP_LIB=$L timeout -k 10 300 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/pf448_${v}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/pf448_${v}_$rnd.json')); print('pt448x16 prefill $v', d['prefill_ms'])"
  done
done
