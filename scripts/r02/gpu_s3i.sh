# round 2, session 3, call I: batch-1 down projection as tile pairs (PG_FIN_NT2) -- parity tests with it on, then
# graph-replayed pt-224 decode step A/B/A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3i; mkdir -p $O
PG_FIN_NT2=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py -k "full_size or greedy or tiny or chained or two_stream" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
  PG_FIN_NT2=$v timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "fin_nt2=$v $(python -c "import json;d=json.load(open('$O/step.json'));print(d['ms_per_token'], d['all'], d['ids16'][:6])")"
done
PG_FIN_NT2=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/dprof.log 2>&1 || exit 1
python scripts/step_timeline.py $O/dprof/run_kernel_trace.csv
