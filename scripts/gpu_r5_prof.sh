# prefill breakdown + decode timeline on the product library, then an lm_head variant A/B (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf -o run --output-format csv -- python scripts/tune/prefill_time.py --reps 4 > $O/pf.log 2>&1 || { tail -5 $O/pf.log; exit 1; }
python scripts/prefill_breakdown.py $O/pf/run_kernel_trace.csv > $O/prefill_breakdown_pt224.txt; cat $O/prefill_breakdown_pt224.txt
bash scripts/gpu_ab_libs.sh ${1:-r5prof}/ab "product scripts/tune/libs/lm2d4.so scripts/tune/libs/lm2d6.so" PG_DECODE_ADD "fx" 3
