set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ao2.log
: > $OUT
timeout -k 10 240 python scripts/tune/decode_step.py --no-fuse-ao >> $OUT 2>> gpurun_out/ao2.err || exit 1
timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/ao2.err || exit 1
PGHIP_LIB=scripts/tune/var_ao2.so timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/ao2.err || exit 1
PGHIP_LIB=scripts/tune/var_ao4.so timeout -k 10 240 python scripts/tune/decode_step.py >> $OUT 2>> gpurun_out/ao2.err || exit 1
cut -c1-230 $OUT
