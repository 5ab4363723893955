# usage: bash scripts/gpu_check.sh TAG -- GPU tests (incl. slow) + 1-GPU bench; exits at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail -20 gpurun_out/$TAG.bench.err; exit 1; }
cat gpurun_out/$TAG.bench.json
