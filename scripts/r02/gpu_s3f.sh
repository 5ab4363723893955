# round 2, session 3, call F: Infinity-Cache-resident q|k|v / o_proj weights (PG_GEMV_HOT variants: those GEMVs read
# with default-policy loads, every other weight stream non-temporal) -- graph-replayed pt-224 decode step, A/B/A
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3f; mkdir -p $O
for lib in "" scripts/tune/var_hot1.so scripts/tune/var_hot2.so scripts/tune/var_hot3.so "" scripts/tune/var_hot1.so scripts/tune/var_hot2.so; do
  PGHIP_LIB=$lib timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "lib=${lib:-product} $(python -c "import json;d=json.load(open('$O/step.json'));print(d['ms_per_token'], d['all'])")"
done
