# prefill GEMM tuning (gpurun_out/$1): the product build's tile / split sweep with the hipBLASLt yardstick, the deep
# staging variant, the no-MFMA / no-load probes on the unsplit shapes, and the batch-1 prefill time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tune}; mkdir -p $O
L=scripts/tune/lib
timeout -k 10 400 python scripts/tune/small_gemm_sweep.py > $O/sweep.txt 2>&1 || { tail -n 5 $O/sweep.txt; exit 1; }
if [ -f $L/deep.so ]; then
  PGHIP_LIB=$L/deep.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm" > $O/tests_deep.log 2>&1
  rc=$?; tail -n 2 $O/tests_deep.log; [ $rc -eq 0 ] || exit 1
  PGHIP_LIB=$L/deep.so SWEEP_BLAS=0 SWEEP_TILES=t64,n64 SWEEP_KS=1,2,3,4,6 timeout -k 10 400 python scripts/tune/small_gemm_sweep.py > $O/sweep_deep.txt 2>&1 || { tail -n 5 $O/sweep_deep.txt; exit 1; }
fi
for p in probe1 probe2; do
  [ -f $L/$p.so ] || continue
  PGHIP_LIB=$L/$p.so SWEEP_BLAS=0 SWEEP_KS=1 timeout -k 10 300 python scripts/tune/small_gemm_sweep.py > $O/sweep_$p.txt 2>&1 || { tail -n 5 $O/sweep_$p.txt; exit 1; }
done
timeout -k 10 300 python scripts/tune/prefill_time.py > $O/prefill.txt 2>&1 || exit 1
tail -n 2 $O/prefill.txt
