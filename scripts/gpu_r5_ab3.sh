# round 5: decode attention split cap A/B (pt-896 x32 fp8) + pending prefill / lm_head library A/B (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab3}; mkdir -p $O
for r in 1 2; do
  for s in 8 6 12; do
    PG_DECODE_MAX_SPLITS=$s timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"max_splits\": $s, /" | tee -a $O/splits896.jsonl || exit 1
  done
done
bash scripts/gpu_r5_ab2.sh ${1:-ab3}/ab2
