# round 2, call K: the one-launch decode MLP block (pg_decode_mlp_block): bit-exact test, A/B bench, step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "mlp_block" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
PG_MLP_BLOCK=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_on.json 2> $O/bench_on.err || { tail -5 $O/bench_on.err; exit 1; }
PG_MLP_BLOCK=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_off.json 2> $O/bench_off.err || { tail -5 $O/bench_off.err; exit 1; }
PG_MLP_BLOCK=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_on2.json 2> $O/bench_on2.err || { tail -5 $O/bench_on2.err; exit 1; }
for f in on off on2; do python -c "import json,sys; d=json.load(open('$O/bench_$f.json')); print('$f', d['value'], d['decode_ms_per_token'], d['prefill_ms'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/dprof.log 2>&1 || { tail -5 $O/dprof.log; exit 1; }
python scripts/step_timeline.py $O/dprof/run_kernel_trace.csv > $O/decode_step_timeline.txt
cat $O/decode_step_timeline.txt
