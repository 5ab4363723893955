# round refresh: full GPU suite, smoke(), pt-224 bench (+ CPU baseline) and kernel stats, pt-448 x16 bench and
# one request's kernel trace, pt-896 x32 fp8 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-s4r}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/$T.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1 || { tail -20 gpurun_out/$T.smoke.log; exit 1; }
tail -1 gpurun_out/$T.smoke.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/$T.b224.json 2> gpurun_out/$T.b224.err || { tail -30 gpurun_out/$T.b224.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$T.p224 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T.p224.log 2>&1 || { echo "prof224 failed"; exit 1; }
timeout -k 10 600 python bench.py --config pt-448 --batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T.b448.json 2> gpurun_out/$T.b448.err || { tail -30 gpurun_out/$T.b448.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$T.p448 -o run --output-format csv -- python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/$T.p448.log 2>&1 || { echo "prof448 failed"; exit 1; }
timeout -k 10 600 python bench.py --config pt-896 --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --fp8 > gpurun_out/$T.b896.json 2> gpurun_out/$T.b896.err || { tail -30 gpurun_out/$T.b896.err; exit 1; }
for f in b224 b448 b896; do python -c "
import json; d=json.load(open('gpurun_out/$T.$f.json')); print('$f', d['value'], d['prefill_ms'], d['prefill_mfma_frac'], d['decode_ms_per_token'], d['roofline']['frac'])"; done
