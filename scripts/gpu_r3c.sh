# kernel tests, fused decode-attention plan sweep, pt-448 x16 prefill kernel profile (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tk.log 2>&1; tail -2 $O/tk.log; grep -q " passed" $O/tk.log && ! grep -q failed $O/tk.log || exit 1
PG_FUSED_ONLY=1 timeout -k 10 300 python scripts/tune/decode_attn_bench.py > $O/dab.txt 2>&1 || { tail -3 $O/dab.txt; exit 1; }
grep fused $O/dab.txt | grep -v '^{'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf448 -o run --output-format csv -- python bench.py --config pt-448 --batch 16 --steps 1 --warmup 0 --gen-tokens 2 --no-cpu-baseline > $O/pf448.log 2>&1 || { tail -5 $O/pf448.log; exit 1; }
python scripts/prefill_breakdown.py $O/pf448/run_kernel_trace.csv > $O/prefill_breakdown_pt448x16.txt; head -16 $O/prefill_breakdown_pt448x16.txt; tail -1 $O/prefill_breakdown_pt448x16.txt
