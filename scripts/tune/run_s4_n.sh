# split-KV decode attention: waves per workgroup 1 (product) / 2 / 4 (consecutive splits share a CU's L2 lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s4n.tests.log 2>&1 || { tail -5 gpurun_out/s4n.tests.log; exit 1; }
PGHIP_LIB=scripts/tune/var_sw2.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -x -k "attention or decode" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s4n.tests2.log 2>&1 || { tail -5 gpurun_out/s4n.tests2.log; exit 1; }
rm -f gpurun_out/s4n.log
for v in prod sw2 sw4 prod sw2 sw4; do
  if [ $v = prod ]; then L=""; else L=scripts/tune/var_$v.so; fi
  for B in 16 1; do
    C=pt-448; [ $B = 1 ] && C=pt-224
    PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config $C --batch $B --steps 50 > gpurun_out/s4n.one 2>&1 || { cat gpurun_out/s4n.one; exit 1; }
    echo "$v B=$B $(tail -1 gpurun_out/s4n.one | cut -c100-160)" >> gpurun_out/s4n.log
  done
done
cat gpurun_out/s4n.log
