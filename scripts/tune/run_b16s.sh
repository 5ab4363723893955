# batched decode (pt-448 x16, fin path): o / down split-K sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
for so in 2 4; do for sd in 4 8; do
  timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-o $so --split-down $sd > gpurun_out/b16s.log 2>&1 || exit 1
  echo "so=$so sd=$sd: $(tail -1 gpurun_out/b16s.log | cut -c90-150)"
done; done
