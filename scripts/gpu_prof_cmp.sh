# Prefill kernel breakdowns (rocprofv3 --kernel-trace, scripts/prefill_breakdown.py) of scripts/tune/prefill_big.py under
# two values of an environment knob:
#   gpurun -- bash scripts/gpu_prof_cmp.sh <out> <VAR> "<v1 v2>" [prefill_big.py args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; VAR=$2; VALS=$3; shift 3
mkdir -p $O
for v in $VALS; do
  D=$O/${VAR}_$(basename $v)
  export $VAR=$v
  timeout -k 10 600 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 scripts/tune/prefill_big.py \
    --reps 2 "$@" > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python3 scripts/prefill_breakdown.py $D/run_kernel_trace.csv > $D.txt
  rm -rf $D
  echo "== $VAR=$v"; head -14 $D.txt; tail -1 $D.txt
done
