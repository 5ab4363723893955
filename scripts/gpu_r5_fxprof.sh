# decode step timelines, fixed-point (fx) vs float-atomic (both) residual adds (gpurun_out/$1); MODES = run order
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fxprof}; mkdir -p $O
i=0
for m in ${MODES:-fx both}; do
i=$((i+1)); D=$O/d_${m}_$i
PG_DECODE_ADD=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-224 --batch 1 --steps 20 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
python scripts/step_timeline.py $D/run_kernel_trace.csv > $O/timeline_${m}_$i.txt; echo "== $m $i"; head -3 $O/timeline_${m}_$i.txt; grep "step wall" $O/timeline_${m}_$i.txt
done
