set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/splits.log
: > $OUT
for a in "--split-o 2 --split-down 4" "--split-o 4 --split-down 4" "--split-o 8 --split-down 4" "--split-o 4 --split-down 8" "--split-o 2 --split-down 8" "--split-o 4 --split-down 2" "--split-o 1 --split-down 4"; do
  timeout -k 10 240 python scripts/tune/decode_step.py $a >> $OUT 2>> gpurun_out/splits.err || exit 1
done
cat $OUT
