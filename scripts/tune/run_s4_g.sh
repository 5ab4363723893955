# engine GPU tests on the row-major prefill copies, pt-448 x16 bench, pt-224 prefill with/without the copies at M=264
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4g.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4g.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s4g.b448.json 2> gpurun_out/s4g.b448.err || { tail -20 gpurun_out/s4g.b448.err; exit 1; }
cut -c 1-20,700-900 gpurun_out/s4g.b448.json
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s4g.b224.json 2> gpurun_out/s4g.b224.err || exit 1
PG_ROWMAJOR_MIN_M=256 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s4g.b224r.json 2> gpurun_out/s4g.b224r.err || exit 1
grep -o '"prefill_ms": [0-9.]*' gpurun_out/s4g.b224.json gpurun_out/s4g.b224r.json gpurun_out/s4g.b448.json
