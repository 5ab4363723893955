# round 2, session 3, call H: does the decode step time depend on the prefill's allocation pattern? (in-launch split-K
# finalisation on / off, and off with its ticket buffer allocated anyway)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3h; mkdir -p $O
for v in "PG_SPLITK_INLAUNCH=1" "PG_SPLITK_INLAUNCH=0" "PG_SPLITK_INLAUNCH=0 PG_TK_ALWAYS=1" "PG_SPLITK_INLAUNCH=1" "PG_SPLITK_INLAUNCH=0" "PG_SPLITK_INLAUNCH=0 PG_TK_ALWAYS=1"; do
  env $v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['prefill_ms'], d['decode_ms_per_token'])")"
done
