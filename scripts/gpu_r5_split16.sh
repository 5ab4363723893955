# round 5: batched decode attention split cap re-checked after the shared merge (pt-896 x32 fp8, pt-448 x16)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-split16}; mkdir -p $O
for r in 1 2; do
  for s in 8 12 16; do
    PG_DECODE_MAX_SPLITS=$s timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"max_splits\": $s, \"cfg\": \"pt896x32\", /" | tee -a $O/splits.jsonl || exit 1
    PG_DECODE_MAX_SPLITS=$s timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"max_splits\": $s, \"cfg\": \"pt448x16\", /" | tee -a $O/splits.jsonl || exit 1
  done
done
