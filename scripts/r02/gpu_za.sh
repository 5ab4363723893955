# round 2, call ZA: keys per decode-attention split at B = 1 (o_proj prologue merge re-read vs attention waves)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02za; mkdir -p $O
for sk in 32 64 128 256; do
  PG_SK_SMALL=$sk timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_$sk.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "sk=$sk $(python -c "import json;d=json.load(open('$O/step_$sk.json'));print(d['ms_per_token'])")"
done
for sk in 32 128; do
  PG_SK_SMALL=$sk timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step2_$sk.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "sk=$sk $(python -c "import json;d=json.load(open('$O/step2_$sk.json'));print(d['ms_per_token'])")"
done
