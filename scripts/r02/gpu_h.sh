# round 2, call H: MALL-warm vs cold GEMV, o_proj split 1 vs 2 in the decode step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 200 python scripts/r02/gemv_bench.py > $O/gemv.log 2>&1 || { cat $O/gemv.log; exit 1; }
tail -1 $O/gemv.log
for v in 1 2 1 2; do
  PG_SPLIT_O=$v timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 > $O/one 2>&1 || { cat $O/one; exit 1; }
  echo "split_o=$v $(tail -1 $O/one | grep -o '"ms_per_token": [0-9.]*') $(tail -1 $O/one | grep -o '"ids16": \[[0-9]*, [0-9]*, [0-9]*')" >> $O/ab.log
done
cat $O/ab.log
