# Round profile set: PMC traffic of the roofline kernel (separate FETCH_SIZE / WRITE_SIZE passes), the default
# bench line (reads that traffic), and the kernel-trace stats of the same bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run --output-format csv -- python scripts/pmc_gateup.py > gpurun_out/pmc_f.log 2>&1 || { tail -5 gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_w -o run --output-format csv -- python scripts/pmc_gateup.py > gpurun_out/pmc_w.log 2>&1 || { tail -5 gpurun_out/pmc_w.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_f gpurun_out/pmc_w profiles/r01_pmc_gateup.json || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/pf.bench.json 2> gpurun_out/pf.bench.err || { tail -20 gpurun_out/pf.bench.err; exit 1; }
cat gpurun_out/pf.bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/pfprof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pfprof.log 2>&1
echo "prof rc=$?"
