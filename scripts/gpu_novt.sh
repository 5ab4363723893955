# decode timing with / without the row-major K and V^T cache writes in the q|k|v epilogue (timing only: the
# variant's prefill attention reads unwritten K / V^T) (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-novt}; mkdir -p $O
for rnd in 1 2; do
  for v in product novt; do
    L=""; [ $v = product ] || L=scripts/tune/$v.so
    PGHIP_LIB=$L timeout -k 10 300 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --gen-tokens 32 --no-cpu-baseline > $O/d448_${v}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    PGHIP_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/d224_${v}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; a=json.load(open('$O/d448_${v}_$rnd.json')); b=json.load(open('$O/d224_${v}_$rnd.json')); print('$v pt448x16 decode', a['decode_ms_per_token'], 'pt224x1 decode', b['decode_ms_per_token'])"
  done
done
