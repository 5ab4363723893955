set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/v3.variants.log
: > $OUT
for v in base nt nopro nopro_nt; do
  PGHIP_LIB=scripts/tune/var_$v.so timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/v3.err || exit 1
done
cat $OUT
