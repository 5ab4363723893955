# fp8 row copy from the one-launch decode attention (ABI 7): whole GPU suite, then pt-896 x32 fp8 with / without
# it, interleaved (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-a8}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for rnd in 1 2; do
  for v in 1 0; do
    PG_ATTN_FP8_OUT=$v timeout -k 10 400 python bench.py --config pt-896 --batch 32 --fp8 --steps 2 --warmup 1 --gen-tokens 32 --no-cpu-baseline > $O/d896_${v}_$rnd.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; b=json.load(open('$O/d896_${v}_$rnd.json')); print('attn_fp8_out=$v pt896x32 decode', b['decode_ms_per_token'], 'prefill', b['prefill_ms'])"
  done
done
