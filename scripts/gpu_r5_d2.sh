# round 5: ring depth of the two-tile bf16 GEMV (gate/up, finalised down at pt-448 x16): kernel timelines + step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-d2}; mkdir -p $O
CASES="base||--config pt-448 --batch 16;d6|PGHIP_LIB=scripts/tune/libs/d6.so|--config pt-448 --batch 16;d8|PGHIP_LIB=scripts/tune/libs/d8.so|--config pt-448 --batch 16" \
  bash scripts/gpu_timeline.sh ${1:-d2} || exit 1
for r in 1 2; do
  for v in base d6 d8; do
    L=""; [ $v != base ] && L=scripts/tune/libs/$v.so
    PGHIP_LIB=$L timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 \
      2>> $O/err.log | sed "s/^{/{\"v\": \"$v\", /" | tee -a $O/ab.jsonl || exit 1
  done
done
