# split-KV merge with the O partials prefetched (product) vs loaded after the weights (var_nopf.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4x.tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4x.tests.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/s4x.log
for r in 1 2; do
for v in prod nopf; do
  if [ $v = prod ]; then L=""; else L=scripts/tune/var_$v.so; fi
  for B in 16 8; do
    PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch $B --steps 50 > gpurun_out/s4x.one 2>&1 || { cat gpurun_out/s4x.one; exit 1; }
    echo "$v B=$B $(tail -1 gpurun_out/s4x.one | grep -o '"ms_per_token": [0-9.]*') $(tail -1 gpurun_out/s4x.one | grep -o '"ids16": \[[0-9]*, [0-9]*, [0-9]*')" >> gpurun_out/s4x.log
  done
done
done
cat gpurun_out/s4x.log
