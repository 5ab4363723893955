# round 2, call V: pt-224 B=1 decode: o_proj split (1 = unsplit, merge of all 8 heads per workgroup; 8 = one head each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02v; mkdir -p $O
for r in a b; do
for so in 1 2 4 8; do
  if [ $so = 1 ]; then E=""; else E="PG_SPLIT_O=$so"; fi
  env $E timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/so${so}_$r.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "split_o $so ($r): $(python -c "import json;d=json.load(open('$O/so${so}_$r.json'));print(d['ms_per_token'], d['split_o'])")"
done
done
