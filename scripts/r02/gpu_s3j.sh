# round 2, session 3, call J: the argmax's first pass folded into the batch-1 lm_head GEMV (PG_FUSE_ARGMAX) --
# parity tests, then graph-replayed pt-224 decode step A/B/A/B and the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py tests/test_dropin_gpu.py -k "fused_argmax or chained or greedy or full_size or tiny or dropin or inference" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PG_FUSE_ARGMAX=$v timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "fuse_argmax=$v $(python -c "import json;d=json.load(open('$O/step.json'));print(d['ms_per_token'], d['all'], d['ids16'][:6])")"
done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['prefill_ms'], d['decode_ms_per_token'], d['decode_hbm_frac'])"
