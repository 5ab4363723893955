set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/splits2.log
: > $OUT
for a in "--split-o 2 --split-down 4" "--split-o 4 --split-down 4" "--split-o 2 --split-down 8" "--split-o 4 --split-down 8" "--split-o 1 --split-down 4" "--split-o 2 --split-down 2"; do
  timeout -k 10 240 python scripts/tune/decode_step.py $a >> $OUT 2>> gpurun_out/splits.err || exit 1
done
for v in nomerge nofin d6; do
  PGHIP_LIB=scripts/tune/var_$v.so timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/splits.err || exit 1
done
cat $OUT
