# batched q|k|v GEMV with one tile per workgroup (product) vs two (var_qkvnt2.so): parity, then decode step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -q -x -m "gpu" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s4l.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4l.tests.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/s4l.log
for v in prod nt2 prod nt2; do
  if [ $v = prod ]; then L=""; else L=scripts/tune/var_qkvnt2.so; fi
  for B in 16 8; do
    PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch $B --steps 50 > gpurun_out/s4l.one 2>&1 || { cat gpurun_out/s4l.one; exit 1; }
    echo "$v B=$B $(tail -1 gpurun_out/s4l.one | cut -c1-200)" >> gpurun_out/s4l.log
  done
done
cut -c1-150 gpurun_out/s4l.log
