# FIN / fx kernel tests, then round 5 vs round 4 decode A/B (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "fin or fx or bit_reproducible or pt448 or batched" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_r5_r4ab.sh ${1:-r4ab}
