# pt-224 B=1 decode: o / down split-K sweep on the current library
set -o pipefail
cd $GRAFT_REPO_ROOT
for sd in 4 8 16; do for so in 2 4; do
  timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 --split-o $so --split-down $sd >> gpurun_out/s4_splits.log 2>&1 || exit 1
done; done
for sd in 4 8; do
  timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-down $sd >> gpurun_out/s4_splits.log 2>&1 || exit 1
done
