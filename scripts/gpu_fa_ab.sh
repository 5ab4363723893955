# flash-attention change: attention kernel tests, attn_bench new vs old library, pt-448 x16 / pt-224 prefill A/B (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-faab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tk.log 2>&1; tail -2 $O/tk.log; grep -q " passed" $O/tk.log && ! grep -q failed $O/tk.log || exit 1
timeout -k 10 200 python scripts/tune/attn_bench.py > $O/ab_new.txt 2>&1 || { tail -3 $O/ab_new.txt; exit 1; }
PGHIP_LIB=scripts/tune/fa_old.so timeout -k 10 200 python scripts/tune/attn_bench.py > $O/ab_old.txt 2>&1 || { tail -3 $O/ab_old.txt; exit 1; }
echo new; cat $O/ab_new.txt; echo old; cat $O/ab_old.txt
for rnd in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L=scripts/tune/fa_old.so
    PGHIP_LIB=$L timeout -k 10 300 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/pf448_${v}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/pf448_${v}_$rnd.json')); print('pt448x16 $v', d['prefill_ms'], d['value'])"
  done
done
