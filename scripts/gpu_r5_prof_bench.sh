# round 5: rocprofv3 --stats of the default bench command + PMC traffic of its roofline kernel (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-profb}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/b -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
bash scripts/gpu_pmc_gateup.sh ${1:-profb}/pmc
