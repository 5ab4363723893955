# Re-entry check: GPU parity tests, default bench line, kernel-trace stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m "gpu and not slow" -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/c2.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/c2.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/c2.bench.json 2> gpurun_out/c2.bench.err || { tail -20 gpurun_out/c2.bench.err; exit 1; }
cat gpurun_out/c2.bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/c2prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c2.prof.log 2>&1
echo "prof rc=$?"
