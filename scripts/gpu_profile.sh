# Round-3 profiling pass (gpurun_out/$1): batch-1 prefill kernel breakdown, batched long-KV decode step timelines,
# the small-GEMM sweep, and the batch-1 flash-attention A/B (PG_FA_SMALL variant library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf -o run --output-format csv -- python scripts/tune/prefill_time.py --reps 4 --knob VISION_DP > $O/pf.log 2>&1 || { tail -5 $O/pf.log; exit 1; }
python scripts/prefill_breakdown.py $O/pf/run_kernel_trace.csv > $O/prefill_breakdown_pt224.txt; tail -3 $O/prefill_breakdown_pt224.txt
timeout -k 10 200 python scripts/tune/prefill_time.py --reps 20 --knob VISION_DP > $O/pf_time_fa1.json 2>&1 || exit 1
PGHIP_LIB=scripts/tune/fa_small0.so timeout -k 10 200 python scripts/tune/prefill_time.py --reps 20 --knob VISION_DP > $O/pf_time_fa0.json 2>&1 || exit 1
tail -1 $O/pf_time_fa1.json $O/pf_time_fa0.json
timeout -k 10 300 python scripts/tune/small_gemm_sweep.py > $O/small_gemm_sweep.txt 2>&1 || { tail -3 $O/small_gemm_sweep.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d896 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 10 > $O/d896.log 2>&1 || { tail -5 $O/d896.log; exit 1; }
python scripts/step_timeline.py $O/d896/run_kernel_trace.csv > $O/decode_step_timeline_896x32_fp8.txt; cat $O/decode_step_timeline_896x32_fp8.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d448 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 20 > $O/d448.log 2>&1 || { tail -5 $O/d448.log; exit 1; }
python scripts/step_timeline.py $O/d448/run_kernel_trace.csv > $O/decode_step_timeline_448x16.txt; cat $O/decode_step_timeline_448x16.txt
