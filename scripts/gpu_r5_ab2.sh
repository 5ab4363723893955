# prefill A/B (norm weights early, finalize RoPE early) + lm_head depth A/B (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab2}; mkdir -p $O
for r in 1 2 3; do
  for lib in "" scripts/tune/libs/norm0.so scripts/tune/libs/fin0.so; do
    PGHIP_LIB=$lib timeout -k 10 200 python scripts/tune/prefill_ms.py 2>> $O/err.log | tee -a $O/prefill.jsonl || exit 1
  done
done
bash scripts/gpu_ab_libs.sh ${1:-ab2}/lm "product scripts/tune/libs/lmd8.so" PG_DECODE_ADD "fx" 3
