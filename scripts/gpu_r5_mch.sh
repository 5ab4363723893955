# decode attention merge: 8 vs 16 partials per round trip (tests + pt-896 x32 / pt-448 x16 decode A/B) (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-mch}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "attn_decode_fused" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in "" scripts/tune/libs/share0.so; do
    PGHIP_LIB=$lib timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"cfg\": \"pt896x32\", /" | tee -a $O/decode.jsonl || exit 1
  done
done
