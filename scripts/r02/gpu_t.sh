# round 2, call T: pt-224 B=1 decode: keys per attention split (2/4-block splits = the LDS-merged kernel, fewer
# partials for the o_proj merge prologue) x down split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02t; mkdir -p $O
for r in a b; do
for sk in 32 64 128; do
for sd in 4 8; do
  timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 --split-keys $sk --split-down $sd > $O/sk${sk}_sd${sd}_$r.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "sk $sk sd $sd ($r): $(python -c "import json;d=json.load(open('$O/sk${sk}_sd${sd}_$r.json'));print(d['ms_per_token'], d['ids16'][:6])")"
done
done
done
