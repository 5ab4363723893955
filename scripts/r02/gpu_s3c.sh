# round 2, session 3, call C: kernel timeline of the two-stream decode step (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3c; mkdir -p $O
PG_DECODE_BANK=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python -u scripts/tune/decode_step.py --steps 20 > $O/step.log 2>&1 || { tail -5 $O/step.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python scripts/r02/bank_timeline.py $f > $O/timeline.txt && head -60 $O/timeline.txt && tail -40 $O/timeline.txt
