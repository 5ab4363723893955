# The round's measurement evidence (gpurun_out/$1): the default bench line; rocprofv3 --kernel-trace --stats of the
# same bench command; the roofline kernel's PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes); the configs[2] and
# configs[4] single-GPU bench lines; the batch-1 prefill breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-evid}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/b -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
bash scripts/gpu_pmc_gateup.sh ${1:-evid}/pmc || exit 1
timeout -k 10 500 python bench.py --config pt-448 --batch 16 --no-cpu-baseline --no-tp-curve > $O/pt448_b16.json 2> $O/err448.log || { tail -5 $O/err448.log; exit 1; }
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline --no-tp-curve > $O/pt896_b32_fp8.json 2> $O/err896.log || { tail -5 $O/err896.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/pf -o run --output-format csv -- python scripts/tune/prefill_time.py --reps 4 > $O/pf.log 2>&1 || { tail -5 $O/pf.log; exit 1; }
python scripts/prefill_breakdown.py $O/pf/run_kernel_trace.csv > $O/prefill_breakdown_pt224.txt
rm -rf $O/pf/*.csv
for f in pt448_b16 pt896_b32_fp8; do python -c "import json;o=json.load(open('$O/$f.json'));print('$f', o['value'], o['prefill_ms'], o['decode_ms_per_token'], o['decode_hbm_frac'])"; done
tail -1 $O/prefill_breakdown_pt224.txt
