# pipelined flash kernel + permlane reductions + one-instruction bf16 packs: kernel tests, attn_bench product vs
# variants, pt-448 x16 prefill A/B, pt-224 prefill + decode (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fapipe}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tk.log 2>&1; tail -2 $O/tk.log; grep -q " passed" $O/tk.log && ! grep -q failed $O/tk.log || exit 1
for v in product fa_nopipe fa_w8; do
  L=""; [ $v = product ] || L=scripts/tune/$v.so
  PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/attn_bench.py > $O/ab_$v.txt 2>&1 || { tail -3 $O/ab_$v.txt; exit 1; }
  echo "== $v"; grep '^[gs]' $O/ab_$v.txt
done
for rnd in 1 2; do
  for v in product fa_nopipe fa_w8; do
    L=""; [ $v = product ] || L=scripts/tune/$v.so
    PGHIP_LIB=$L timeout -k 10 300 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/pf448_${v}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/pf448_${v}_$rnd.json')); print('pt448x16 $v prefill', d['prefill_ms'])"
  done
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/b224.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
cat $O/b224.json
