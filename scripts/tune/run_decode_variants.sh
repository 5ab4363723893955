# usage: bash scripts/tune/run_decode_variants.sh TAG  -- decode-step ms/token per library variant / split setting
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1.variants.log
: > $OUT
ERR=gpurun_out/$1.variants.err
run() { timeout -k 10 240 python scripts/tune/decode_step.py "$@" >> $OUT 2>> $ERR || { echo "FAILED $*" >> $OUT; exit 1; }; }
for v in base prew mv2 aw1 all; do
  PGHIP_LIB=scripts/tune/var_$v.so run
done
PGHIP_LIB=scripts/tune/var_all.so run --split-o 4
PGHIP_LIB=scripts/tune/var_all.so run --split-o 1
PGHIP_LIB=scripts/tune/var_all.so run --split-down 8
PGHIP_LIB=scripts/tune/var_all.so run --split-down 2
PGHIP_LIB=scripts/tune/var_all.so run --split-keys 64
cat $OUT
