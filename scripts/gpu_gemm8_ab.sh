# fp8 prefill GEMM A/B over library builds at the pt-896 x32 shapes (gpurun_out/$1)
#   gpurun -- bash scripts/gpu_gemm8_ab.sh <out> "<lib.so|product> ..." <rounds>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; LIBS=$2; R=$3
mkdir -p $O
for r in $(seq $R); do
  for lib in $LIBS; do
    if [ "$lib" = product ]; then L=""; else L=$lib; fi
    echo "== $lib round $r" | tee -a $O/ab.txt
    env PGHIP_LIB=$L timeout -k 10 150 python scripts/tune/gemm8_big.py >> $O/ab.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
cat $O/ab.txt
