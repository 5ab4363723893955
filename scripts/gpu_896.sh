set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --config pt-896 --batch 32 --gen-tokens 32 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b896.json 2> gpurun_out/b896.err || { tail -30 gpurun_out/b896.err; exit 1; }
cat gpurun_out/b896.json
