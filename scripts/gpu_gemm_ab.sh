# bf16 prefill GEMM A/B over library builds (gpurun_out/$1): scripts/tune/gemm_bench.py per lib, interleaved
#   gpurun -- bash scripts/gpu_gemm_ab.sh <out> "<lib.so|product> ..." <rounds> <shapes>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; LIBS=$2; R=$3; SH=$4
mkdir -p $O
for r in $(seq $R); do
  for lib in $LIBS; do
    if [ "$lib" = product ]; then L=""; else L=$lib; fi
    echo "== $lib round $r" | tee -a $O/ab.txt
    env PGHIP_LIB=$L timeout -k 10 150 python scripts/tune/gemm_bench.py --only $SH >> $O/ab.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
cat $O/ab.txt
