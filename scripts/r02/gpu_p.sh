# round 2, call P: skinny-M prefill GEMM (one 256/288-row tile per 128 columns) vs the product routing, pt-224 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02p2; mkdir -p $O
timeout -k 10 300 python scripts/tune/skinny_bench.py > $O/base.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
PGHIP_LIB=scripts/tune/skinny.so timeout -k 10 300 python scripts/tune/skinny_bench.py > $O/skinny.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
paste -d'|' <(head -n -1 $O/base.txt) <(head -n -1 $O/skinny.txt)
