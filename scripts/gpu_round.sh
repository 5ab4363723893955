# usage: bash scripts/gpu_round.sh TAG   -- GPU tests (not slow), bench, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests -q -m "gpu and not slow" -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/$TAG.tests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit 1
cat gpurun_out/$TAG.bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.prof.log 2>&1
echo "prof rc=$?"
