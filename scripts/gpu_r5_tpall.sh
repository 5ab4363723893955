# round 5: every tensor-parallel GPU test (ranks sharing one device), with a heartbeat (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tpall}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1100 python -u -m pytest -m gpu -v -s --timeout 1000 --timeout-method thread -p no:cacheprovider \
  tests/test_tp_gpu.py -k "${SEL:-tp}" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -20; grep -o '{"rank": 0.*' $O/tests.log | cut -c1-500; exit $rc
