set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/v2.variants.log
: > $OUT
for v in all hw hw_aw4; do
  PGHIP_LIB=scripts/tune/var_$v.so timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/v2.err || exit 1
done
cat $OUT
bash scripts/tune/prof_decode.sh v2p
