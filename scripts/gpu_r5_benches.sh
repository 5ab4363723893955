# round 5: the configs[2] and configs[4] single-GPU bench lines (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-benches}; mkdir -p $O
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python bench.py --config pt-896 --batch 32 --fp8 --no-cpu-baseline --no-tp-curve > $O/pt896_b32_fp8.json 2> $O/err896.log || { tail -5 $O/err896.log; exit 1; }
cat $O/pt896_b32_fp8.json
timeout -k 10 500 python bench.py --config pt-448 --batch 16 --no-cpu-baseline --no-tp-curve > $O/pt448_b16.json 2> $O/err448.log || { tail -5 $O/err448.log; exit 1; }
cat $O/pt448_b16.json
