# round 6: the tiny TP suite (2 queues per rank, the test default), then ONE run of the 8-rank xGMI exchange test with
# 4 hardware queues per rank (the round-5 timeout condition) to record the exchange diagnostics if it times out
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tp6}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v -rP --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_tp_gpu.py -k "tp_engine_on_one_device or xgmi_allreduce" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -20; [ $rc -eq 0 ] || exit 1
TP_HW_QUEUES=4 timeout -k 10 300 python -u -m pytest -m gpu -v -rA --timeout 240 --timeout-method thread \
  -p no:cacheprovider "tests/test_tp_gpu.py::test_xgmi_allreduce_ranks_on_one_device[8]" > $O/q4.log 2>&1
echo "4-queue run rc=$?"; grep -E "PASSED|FAILED|diag|err" $O/q4.log | tail -8
