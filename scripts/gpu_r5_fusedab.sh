# pt-448 x16: one-launch decode attention (min rounds 2) vs split + combine (3), interleaved; timelines (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fab}; mkdir -p $O
for r in 1 2 3; do
  for fr in 2 3; do
    PG_FUSED_MIN_ROUNDS=$fr timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"fused_min_rounds\": $fr, /" | tee -a $O/ab.jsonl || exit 1
  done
done
CASES="pt448x16||--config pt-448 --batch 16;pt896x32||--config pt-896 --batch 32 --fp8" bash scripts/gpu_timeline.sh ${1:-fab}/tl
