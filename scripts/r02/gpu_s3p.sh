# round 2, session 3, call P: GEMV ring depth re-check on the final code (PG_GEMV_D_NT1 / PG_GEMV_D_NT2), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3p; mkdir -p $O
for v in "X=0" "PG_GEMV_D_NT1=6" "PG_GEMV_D_NT2=3" "X=0" "PG_GEMV_D_NT1=6" "PG_GEMV_D_NT2=3" "PG_GEMV_D_NT2=2"; do
  env $v timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('$O/step.json'));print(d['ms_per_token'], d['all'])")"
done
