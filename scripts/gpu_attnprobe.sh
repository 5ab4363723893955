# decode-attention A/B: product library vs a variant build (gpurun_out/$1); PGHIP_LIB variants listed after $1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-attn}; mkdir -p $O; shift
timeout -k 10 240 python scripts/tune/decode_attn_bench.py > $O/product.txt 2>&1 || { tail -5 $O/product.txt; exit 1; }
for v in "$@"; do
  PGHIP_LIB=$v timeout -k 10 240 python scripts/tune/decode_attn_bench.py > $O/$(basename $v .so).txt 2>&1 || { tail -5 $O/$(basename $v .so).txt; exit 1; }
done
tail -n 1 $O/*.txt
