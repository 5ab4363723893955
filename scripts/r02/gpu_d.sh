# round 2, call D: GPU tests, GEMV micro-bench CPW on/off, decode step + timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 200 python scripts/r02/gemv_bench.py >> $O/gemv.log 2>&1 || exit 1
  PG_GEMV_CPW_OFF=1 timeout -k 10 200 python scripts/r02/gemv_bench.py >> $O/gemv.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/gemv.log
for r in 1 2; do
  timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 > $O/one 2>&1 || { cat $O/one; exit 1; }
  echo "prod $(tail -1 $O/one | grep -o '"ms_per_token": [0-9.]*') $(tail -1 $O/one | grep -o '"ids16": \[[0-9]*, [0-9]*, [0-9]*')" >> $O/ab.log
done
cat $O/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/prof.log 2>&1 || exit 1
python scripts/step_timeline.py $O/prof/run_kernel_trace.csv
