# round 2, session 3, call G: q|k|v MALL-hot default + in-launch split-K finalisation (pg_gemm_splitk) -- kernel /
# engine GPU tests; o_proj merge-prologue cost (PG_T_NOMERGE timing variant: x = 0) A/B/A; batch-1 prefill with the
# in-launch finalisation on / off; fresh pt-224 batch-1 prefill kernel breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3g; mkdir -p $O
for v in 1 0 1 0; do
  PG_SPLITK_INLAUNCH=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  echo "splitk_inlaunch=$v $(python -c "import json;d=json.load(open('$O/bench_$v.json'));print(d['value'], d['prefill_ms'], d['decode_ms_per_token'])")"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python scripts/prefill_breakdown.py $f > $O/breakdown.txt && cat $O/breakdown.txt
