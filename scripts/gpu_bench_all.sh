# bench lines for profiles/: default (pt-224 B=1), pt-448 x16, pt-896 x32 fp8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_pt224.log 2>&1 && tail -1 gpurun_out/bench_pt224.log | cut -c1-300 &&
timeout -k 10 400 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_pt448.log 2>&1 && tail -1 gpurun_out/bench_pt448.log | cut -c1-300 &&
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --fp8 > gpurun_out/bench_pt896.log 2>&1 && tail -1 gpurun_out/bench_pt896.log | cut -c1-300
