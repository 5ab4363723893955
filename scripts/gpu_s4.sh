# usage: bash scripts/gpu_s4.sh TAG -- full GPU suite, smoke(), pt-224 bench + kernel stats, pt-448 x16 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-s4}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { tail -20 gpurun_out/$TAG.smoke.log; exit 1; }
tail -1 gpurun_out/$TAG.smoke.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/$TAG.b224.json 2> gpurun_out/$TAG.b224.err || { tail -30 gpurun_out/$TAG.b224.err; exit 1; }
cat gpurun_out/$TAG.b224.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$TAG.p224 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.p224.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.b448.json 2> gpurun_out/$TAG.b448.err || { tail -30 gpurun_out/$TAG.b448.err; exit 1; }
cat gpurun_out/$TAG.b448.json
