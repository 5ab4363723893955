# flash-attention tuning variants after the LDS read fix: attn_bench per library, pt-224 prefill with / without key splits (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-favar}; mkdir -p $O
for v in product fa_rpw2 fa_w8 fa_deep fa_small; do
  L=""; [ $v = product ] || L=scripts/tune/$v.so
  PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/attn_bench.py > $O/ab_$v.txt 2>&1 || { tail -3 $O/ab_$v.txt; exit 1; }
  echo "== $v"; grep '^[gs]' $O/ab_$v.txt
done
for ks in 1 0 1 0; do
  PG_PF_KEYSPLIT=$ks timeout -k 10 200 python scripts/tune/prefill_time.py --reps 20 > $O/pt_ks$ks.txt 2>&1 || { tail -3 $O/pt_ks$ks.txt; exit 1; }
  echo "keysplit=$ks $(grep 'TILE_M1=1 prefill' $O/pt_ks$ks.txt | head -2 | tr '\n' ' ')"
done
