# round 2, call S: pt-224 B=1 decode: down-projection split sweep (graph-timed step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s; mkdir -p $O
for r in a b; do
for sd in 2 4 8; do
  timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 --split-down $sd > $O/sd${sd}_$r.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "split_down $sd ($r): $(python -c "import json;d=json.load(open('$O/sd${sd}_$r.json'));print(d['ms_per_token'], d['all'])")"
done
done
