# Targeted GPU tests: gpurun -- bash scripts/gpu_tests.sh <out-name> <per-test timeout s> <pytest selection args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-t}; T=${2:-300}; shift 2
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -m gpu -v --timeout $T --timeout-method thread -p no:cacheprovider "$@" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40; exit $rc
