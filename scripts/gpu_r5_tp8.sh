# round 5: TP=8 pt-896 x32 fp8 (eight ranks on one GPU) with the MX decode path on, then off (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tp8}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
for mx in ${MXS:-1 0}; do
  PG_MX_H=$mx PG_MX_NORM=$mx timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 850 --timeout-method thread \
    -p no:cacheprovider tests/test_tp_gpu.py -k "tp8_pt896_fp8_batch32" > $O/tests_mx$mx.log 2>&1
  rc=$?; echo "mx=$mx rc=$rc"; grep -o '{"rank": 0.*' $O/tests_mx$mx.log | head -1 | cut -c1-600
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
