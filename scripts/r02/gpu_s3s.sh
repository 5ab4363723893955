# round 2, session 3, call S: rocprofv3 kernel stats of the default bench and the decode-step timeline, final code
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3s; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/dprof.log 2>&1 || exit 1
python scripts/step_timeline.py $O/dprof/run_kernel_trace.csv | tee $O/decode_step_timeline.txt
