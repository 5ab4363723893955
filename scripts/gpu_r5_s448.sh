# pt-448 x16 decode: split sweep + timeline (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s448}; mkdir -p $O
for sd in 8 4 16; do
  for so in 2 1 4; do
    timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-o $so \
      --split-down $sd 2>> $O/err.log | tee -a $O/splits.jsonl || exit 1
  done
done
CASES="pt448x16||--config pt-448 --batch 16" bash scripts/gpu_timeline.sh ${1:-s448}/tl
