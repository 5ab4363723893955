# round 2, call ZE: pt-224 batch-1 prefill kernel breakdown (after PG_TILE_M1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ze; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -T -d $O/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python scripts/prefill_breakdown.py $f > $O/breakdown.txt && cat $O/breakdown.txt
