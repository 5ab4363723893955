# pt-448 batch 16 (BASELINE configs[2]) bench line + kernel trace of one request
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b448.json 2> gpurun_out/b448.err || { tail -30 gpurun_out/b448.err; exit 1; }
cat gpurun_out/b448.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/p448 -o run --output-format csv -- python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/p448.log 2>&1
echo "prof rc=$?"
