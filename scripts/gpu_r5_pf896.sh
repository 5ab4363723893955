# round 5: pt-896 x32 fp8 prefill kernel breakdown (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pf896}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/d -o run --output-format csv -- python scripts/tune/prefill_big.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python scripts/prefill_breakdown.py $O/d/run_kernel_trace.csv > $O/breakdown.txt; head -30 $O/breakdown.txt
