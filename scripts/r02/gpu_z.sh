# round 2, call Z: chained argmax + next-step embed (pg_argmax_embed): parity, decode step on/off, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "argmax or chained or greedy or batched" > $O/test.log 2>&1 || { tail -15 $O/test.log; exit 1; }
tail -1 $O/test.log
for c in 1 0; do
  PG_CHAIN_EMBED=$c timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_$c.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "chain=$c $(python -c "import json;d=json.load(open('$O/step_$c.json'));print(d['ms_per_token'])")"
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
