# decode step timelines, fixed-point (fx) vs float-atomic (both) residual adds (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fxprof}; mkdir -p $O
for m in fx both; do
PG_DECODE_ADD=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d_$m -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-224 --batch 1 --steps 20 > $O/d_$m.log 2>&1 || { tail -5 $O/d_$m.log; exit 1; }
python scripts/step_timeline.py $O/d_$m/run_kernel_trace.csv > $O/timeline_$m.txt; echo "== $m"; cat $O/timeline_$m.txt
done
