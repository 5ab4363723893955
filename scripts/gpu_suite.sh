# GPU suite + smoke + the default bench line (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 500 python bench.py --config pt-448 --batch 16 --no-cpu-baseline --no-tp-curve > $O/bench_pt448_b16.json 2> $O/bench448.err || { tail -5 $O/bench448.err; exit 1; }
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline --no-tp-curve > $O/bench_pt896_b32_fp8.json 2> $O/bench896.err || { tail -5 $O/bench896.err; exit 1; }
