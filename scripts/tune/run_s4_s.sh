# decode split-KV with paired 32-key blocks (product) vs single blocks (var_nopair.so), 64- and 32-key splits
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -x -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s4s2.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4s2.tests.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/s4s2.log
for r in 1 2; do
for v in prod nopair; do
  if [ $v = prod ]; then L=""; else L=scripts/tune/var_$v.so; fi
  for t in 256 1024; do
    PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-target $t > gpurun_out/s4s2.one 2>&1 || { cat gpurun_out/s4s2.one; exit 1; }
    echo "$v target=$t $(tail -1 gpurun_out/s4s2.one | grep -o '"ms_per_token": [0-9.]*') $(tail -1 gpurun_out/s4s2.one | grep -o '"ids16": \[[0-9]*, [0-9]*, [0-9]*')" >> gpurun_out/s4s2.log
  done
done
PGHIP_LIB= timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 > gpurun_out/s4s2.one 2>&1 || exit 1
echo "prod B=1 $(tail -1 gpurun_out/s4s2.one | grep -o '"ms_per_token": [0-9.]*')" >> gpurun_out/s4s2.log
done
cat gpurun_out/s4s2.log
