# round 2, session 3, final: whole GPU suite, smoke, headline bench, rocprofv3 kernel stats of the bench, PMC traffic
# of the roofline kernel, decode-step timeline, pt-224 x16 / pt-448 x16 / pt-896 x32 fp8 benches (gpurun_out/r02f,
# copied to profiles/ by the caller)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 400 python bench.py > $O/bench_pt224_b1.json 2> $O/bench_pt224_b1.err || { tail -5 $O/bench_pt224_b1.err; exit 1; }
cat $O/bench_pt224_b1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo "prof ok"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_f -o run --output-format csv -- python scripts/pmc_gateup.py > $O/pmc_f.log 2>&1 || { tail -5 $O/pmc_f.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_w -o run --output-format csv -- python scripts/pmc_gateup.py > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 1; }
python scripts/pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_gateup.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > $O/dprof.log 2>&1 || exit 1
python scripts/step_timeline.py $O/dprof/run_kernel_trace.csv > $O/decode_step_timeline.txt
cat $O/decode_step_timeline.txt
timeout -k 10 400 python bench.py --batch 16 --no-cpu-baseline > $O/bench_pt224_b16.json 2> $O/bench_pt224_b16.err || { tail -5 $O/bench_pt224_b16.err; exit 1; }
timeout -k 10 400 python bench.py --batch 64 --no-cpu-baseline --steps 2 --warmup 1 > $O/bench_pt224_b64.json 2> $O/bench_pt224_b64.err || { tail -5 $O/bench_pt224_b64.err; exit 1; }
echo "224x64 ok"
timeout -k 10 400 python bench.py --config pt-448 --batch 16 --no-cpu-baseline > $O/bench_pt448_b16.json 2> $O/bench_pt448_b16.err || { tail -5 $O/bench_pt448_b16.err; exit 1; }
echo "448 ok"
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_pt896_b32_fp8.json 2> $O/bench_pt896_b32_fp8.err || { tail -5 $O/bench_pt896_b32_fp8.err; exit 1; }
echo "896 ok"
