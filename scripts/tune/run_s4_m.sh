# batched decode (pt-448 x16): o / down split-K sweep on the current library
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/s4m.log
for a in "2 4" "2 8" "4 4" "4 8" "2 4"; do
  set -- $a
  timeout -k 10 200 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 50 --split-o $1 --split-down $2 > gpurun_out/s4m.one 2>&1 || { cat gpurun_out/s4m.one; exit 1; }
  echo "so=$1 sd=$2 $(tail -1 gpurun_out/s4m.one | cut -c100-160)" >> gpurun_out/s4m.log
done
cat gpurun_out/s4m.log
