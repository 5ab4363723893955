# round 2, call F: fused decode attention block -- bit-exact test first, then the GPU suite, decode timing, timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py -k fused_decode_block > $O/fused.log 2>&1
rc=$?; tail -15 $O/fused.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PG_FUSE_BLOCK=$v timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 > $O/one 2>&1 || { cat $O/one; exit 1; }
  echo "fuse=$v $(tail -1 $O/one | grep -o '"ms_per_token": [0-9.]*') $(tail -1 $O/one | grep -o '"ids16": \[[0-9]*, [0-9]*, [0-9]*')" >> $O/ab.log
done
cat $O/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/prof.log 2>&1 || exit 1
python scripts/step_timeline.py $O/prof/run_kernel_trace.csv
