# round 2, call W: round-end refresh of the measurements on the final code: headline bench (+ CPU baseline),
# rocprofv3 kernel stats of it, PMC traffic of the roofline kernel, decode-step timelines, secondary configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_pt224_b1.json 2> $O/bench_pt224_b1.err || { tail -5 $O/bench_pt224_b1.err; exit 1; }
echo "bench ok: $(cut -c1-200 $O/bench_pt224_b1.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo "prof ok"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_f -o run --output-format csv -- python scripts/pmc_gateup.py > $O/pmc_f.log 2>&1 || { tail -5 $O/pmc_f.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_w -o run --output-format csv -- python scripts/pmc_gateup.py > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 1; }
python scripts/pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_gateup.json
echo "pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/dprof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/dprof.log 2>&1 || { tail -5 $O/dprof.log; exit 1; }
python scripts/step_timeline.py $O/dprof/run_kernel_trace.csv > $O/decode_step_timeline.txt
cat $O/decode_step_timeline.txt
timeout -k 10 400 python bench.py --config pt-448 --batch 16 --no-cpu-baseline > $O/bench_pt448_b16.json 2> $O/bench_pt448_b16.err || { tail -5 $O/bench_pt448_b16.err; exit 1; }
echo "448: $(cut -c1-120 $O/bench_pt448_b16.json)"
timeout -k 10 300 python bench.py --batch 16 --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_pt224_b16.json 2> $O/bench_pt224_b16.err || { tail -5 $O/bench_pt224_b16.err; exit 1; }
echo "224x16 ok"
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_pt896_b32_fp8.json 2> $O/bench_pt896_b32_fp8.err || { tail -5 $O/bench_pt896_b32_fp8.err; exit 1; }
echo "896 ok"
