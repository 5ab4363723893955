# round 2, session 3, call K: pg_argmax_embed as one launch (ticketed last workgroup) -- parity tests, then graph-
# replayed pt-224 decode step A/B/A/B (PG_ARGMAX_ONEPASS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_dropin_gpu.py -k "argmax or chained or greedy or full_size or tiny or dropin or inference or batched" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0 1 0; do
  PG_ARGMAX_ONEPASS=$v timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "onepass=$v $(python -c "import json;d=json.load(open('$O/step.json'));print(d['ms_per_token'], d['all'], d['ids16'][:6])")"
done
