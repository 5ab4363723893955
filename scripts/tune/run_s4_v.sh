# small-grid prefill attention: flash kernel (product) vs the register / LDS-staged kernels (var_nofa.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in prod nofa prod nofa; do
  if [ $v = prod ]; then L=""; else L=scripts/tune/var_$v.so; fi
  PGHIP_LIB=$L timeout -k 10 200 python scripts/tune/attn_bench.py --only gemma224,siglip224 > gpurun_out/s4v.one 2>&1 || { cat gpurun_out/s4v.one; exit 1; }
  grep -h "224" gpurun_out/s4v.one | sed "s/^/$v /"
done
