# round 2, call Q: decode-step timelines at pt-896 x32 (fp8) and pt-448 x16: where the batched decode time goes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/d896 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 10 > $O/d896.log 2>&1 || { tail -5 $O/d896.log; exit 1; }
python scripts/step_timeline.py $O/d896/run_kernel_trace.csv > $O/decode_step_timeline_896x32_fp8.txt
cat $O/decode_step_timeline_896x32_fp8.txt
tail -1 $O/d896.log | cut -c1-200
