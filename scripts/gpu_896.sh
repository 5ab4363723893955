# BASELINE configs[4] shapes on one MI355X: pt-896 (4096 image tokens) batch 32, bf16 and fp8 Gemma linears
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --fp8 > gpurun_out/b896_fp8.log 2>&1 && tail -1 gpurun_out/b896_fp8.log | cut -c1-2000 &&
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b896_bf16.log 2>&1 && tail -1 gpurun_out/b896_bf16.log | cut -c1-2000
