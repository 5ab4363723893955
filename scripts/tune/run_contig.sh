set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/contig.log
: > $OUT
for v in base contig; do
  PGHIP_LIB=scripts/tune/var_$v.so timeout -k 10 200 python scripts/tune/gateup_time.py >> $OUT 2>> gpurun_out/contig.err || exit 1
  PGHIP_LIB=scripts/tune/var_$v.so timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/contig.err || exit 1
done
cat $OUT
