# round 5: the finalised batched down GEMV at pt-448 x16 -- two or four tiles per workgroup (fin4 variant,
# PG_GEMV_FIN_NT=4) and its K split (PG_SPLIT_DOWN), o_proj split 1 / 2; graph-replayed decode steps + a timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fin16}; mkdir -p $O
for r in 1 2; do
  for v in base fin4; do
    L=""; [ $v != base ] && L=scripts/tune/libs/$v.so
    for sd in 4 8; do
      for so in 1 2; do
        PGHIP_LIB=$L PG_SPLIT_O=$so PG_SPLIT_DOWN=$sd timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 \
          --batch 16 --steps 50 2>> $O/err.log | sed "s/^{/{\"v\": \"$v\", /" | tee -a $O/splits.jsonl || exit 1
      done
    done
  done
done
CASES="fin4_8|PGHIP_LIB=scripts/tune/libs/fin4.so PG_SPLIT_O=1 PG_SPLIT_DOWN=8|--config pt-448 --batch 16;base_4|PG_SPLIT_O=1 PG_SPLIT_DOWN=4|--config pt-448 --batch 16" \
  bash scripts/gpu_timeline.sh ${1:-fin16}
