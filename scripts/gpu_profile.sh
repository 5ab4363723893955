# Profiling pass (gpurun_out/$1): pt-224 batch-1 prefill kernel breakdown and decode step timeline, plus the batched
# long-KV decode step timelines (pt-448 x 16, pt-896 x 32 fp8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf -o run --output-format csv -- python scripts/tune/prefill_time.py --reps 4 > $O/pf.log 2>&1 || { tail -5 $O/pf.log; exit 1; }
python scripts/prefill_breakdown.py $O/pf/run_kernel_trace.csv > $O/prefill_breakdown_pt224.txt; tail -n 3 $O/prefill_breakdown_pt224.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d224 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-224 --batch 1 --steps 20 > $O/d224.log 2>&1 || { tail -5 $O/d224.log; exit 1; }
python scripts/step_timeline.py $O/d224/run_kernel_trace.csv > $O/decode_step_timeline_224x1.txt; cat $O/decode_step_timeline_224x1.txt
if [ "$2" = "long" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d896 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 10 > $O/d896.log 2>&1 || { tail -5 $O/d896.log; exit 1; }
python scripts/step_timeline.py $O/d896/run_kernel_trace.csv > $O/decode_step_timeline_896x32_fp8.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d448 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 20 > $O/d448.log 2>&1 || { tail -5 $O/d448.log; exit 1; }
python scripts/step_timeline.py $O/d448/run_kernel_trace.csv > $O/decode_step_timeline_448x16.txt
fi
