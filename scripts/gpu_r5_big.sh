# round 5: full-size fp8 parity (single rank and TP=8 on one GPU) on the MX decode path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-big}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -m gpu -v -s --timeout 900 --timeout-method thread -p no:cacheprovider \
  tests/test_large_gpu.py tests/test_tp_gpu.py -k "${SEL:-fp8}" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|emulated|ratio" $O/tests.log | tail -30; exit $rc
