# decode step kernel timeline (rocprofv3 kernel trace) for each "name|decode_step.py args" case in CASES
#   gpurun -- 'CASES="pt896x32|--config pt-896 --batch 32 --fp8;pt448x16|--config pt-448 --batch 16" bash scripts/gpu_timeline.sh <out>'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-timeline}; mkdir -p $O
IFS=';' read -ra CS <<< "$CASES"
for c in "${CS[@]}"; do
  name=${c%%|*}; args=${c#*|}; D=$O/d_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python scripts/tune/decode_step.py $args --steps 20 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python scripts/step_timeline.py $D/run_kernel_trace.csv > $O/timeline_$name.txt; echo "== $name"; cat $O/timeline_$name.txt
done
