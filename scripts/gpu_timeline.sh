# decode step kernel timeline (rocprofv3 kernel trace) for each "name|ENV=VAL ...|decode_step.py args" case in CASES
#   gpurun -- 'CASES="mx1|PG_MX_NORM=1|--config pt-896 --batch 32 --fp8;mx0|PG_MX_NORM=0|--config pt-896 --batch 32 --fp8" bash scripts/gpu_timeline.sh <out>'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-timeline}; mkdir -p $O
IFS=';' read -ra CS <<< "$CASES"
for c in "${CS[@]}"; do
  IFS='|' read -r name envs args <<< "$c"; D=$O/d_$name
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python scripts/tune/decode_step.py $args --steps 20 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python scripts/step_timeline.py $D/run_kernel_trace.csv > $O/timeline_$name.txt; echo "== $name"; cat $O/timeline_$name.txt
done
