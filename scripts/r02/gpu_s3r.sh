# round 2, session 3, call R: decode split-K re-sweep on the final code (o_proj / down), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3r; mkdir -p $O
for v in "PG_SPLIT_O=2" "X=0" "PG_SPLIT_O=2" "X=0" "PG_SPLIT_O=2" "X=0" "PG_SPLIT_O=2" "X=0" "PG_SPLIT_O=2" "X=0"; do
  env $v timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('$O/step.json'));print(d['ms_per_token'], d['all'])")"
done
