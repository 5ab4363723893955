# A/B of a variant library (scripts/tune/lib/$2.so) against the product build (gpurun_out/$1): the variant's GEMM
# kernel tests, the small-GEMM sweep on both (tiles t64 / n64), batch-1 prefill time on both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
V=$PWD/scripts/tune/lib/$2.so
PGHIP_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm" > $O/tests_variant.log 2>&1
rc=$?; tail -n 2 $O/tests_variant.log; [ $rc -eq 0 ] || exit 1
SWEEP_BLAS=0 SWEEP_TILES=t64,n64 SWEEP_KS=${KS:-1,2,3,6} timeout -k 10 400 python scripts/tune/small_gemm_sweep.py > $O/sweep_base.txt 2>&1 || { tail -n 5 $O/sweep_base.txt; exit 1; }
PGHIP_LIB=$V SWEEP_BLAS=0 SWEEP_TILES=t64,n64 SWEEP_KS=${KS:-1,2,3,6} timeout -k 10 400 python scripts/tune/small_gemm_sweep.py > $O/sweep_var.txt 2>&1 || { tail -n 5 $O/sweep_var.txt; exit 1; }
timeout -k 10 300 python scripts/tune/prefill_time.py > $O/prefill_base.txt 2>&1 || exit 1
PGHIP_LIB=$V timeout -k 10 300 python scripts/tune/prefill_time.py > $O/prefill_var.txt 2>&1 || exit 1
tail -n 1 $O/prefill_base.txt; tail -n 1 $O/prefill_var.txt
