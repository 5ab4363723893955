# round 5: o / down K splits of the finalised batched decode GEMVs re-checked on the final tree (pt-448 x16)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fin16}; mkdir -p $O
for r in 1 2; do
  for sd in 4 8 2; do
    for so in 1 2; do
      PG_SPLIT_O=$so PG_SPLIT_DOWN=$sd timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 \
        2>> $O/err.log | sed "s/^{/{\"cfg\": \"pt448x16\", /" | tee -a $O/splits.jsonl || exit 1
    done
  done
done
