# round 2, call J: pt-448 x16 prefill kernel breakdown (one request) + pt-224 prefill breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p448 -o run --output-format csv -- python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --no-cpu-baseline --gen-tokens 4 > $O/p448.log 2>&1 || { tail -5 $O/p448.log; exit 1; }
python scripts/prefill_breakdown.py $O/p448/run_kernel_trace.csv > $O/prefill_448x16.txt
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p224 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --gen-tokens 4 > $O/p224.log 2>&1 || { tail -5 $O/p224.log; exit 1; }
python scripts/prefill_breakdown.py $O/p224/run_kernel_trace.csv > $O/prefill_224.txt
cat $O/prefill_448x16.txt
