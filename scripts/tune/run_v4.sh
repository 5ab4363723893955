set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/v4.variants.log
: > $OUT
timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/v4.err || exit 1
cat $OUT
bash scripts/tune/prof_decode.sh v4p
