set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 && \
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -q -m slow -p no:cacheprovider > gpurun_out/slow1.log 2>&1
echo rc=$?
