# Run a pytest selection against a tuning library build (gpurun_out/$1): PGHIP_LIB=$2
#   gpurun -- bash scripts/gpu_lib_tests.sh <out> <lib.so> <pytest args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; L=$2; shift 2
mkdir -p $O
PGHIP_LIB=$L timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -12; exit $rc
