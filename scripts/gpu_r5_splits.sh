# round 5: pt-896 x32 fp8 decode split sweep (o_proj / down_proj split-K) on the MX path (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-splits}; mkdir -p $O
for sd in 8 16 4; do
  for so in 2 1 4; do
    timeout -k 10 300 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 50 --split-o $so \
      --split-down $sd 2>> $O/err.log | tee -a $O/splits.jsonl || exit 1
  done
done
