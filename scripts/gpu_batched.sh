# batched-decode bench lines (BASELINE configs[2] / configs[4] shapes on one GPU) + decode-attention microbench
# (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-batched}; mkdir -p $O
PG_FUSED_ONLY=1 timeout -k 10 300 python scripts/tune/decode_attn_bench.py > $O/attn_bench.txt 2>&1 || { tail -5 $O/attn_bench.txt; exit 1; }
grep -v amdgpu.ids $O/attn_bench.txt | grep -v '^{'
timeout -k 10 400 python bench.py --config pt-448 --batch 16 --no-cpu-baseline > $O/pt448_b16.json 2> $O/pt448_b16.err || { tail -5 $O/pt448_b16.err; exit 1; }
cat $O/pt448_b16.json
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline > $O/pt896_b32_fp8.json 2> $O/pt896_b32_fp8.err || { tail -5 $O/pt896_b32_fp8.err; exit 1; }
cat $O/pt896_b32_fp8.json
