# round 2, session 3, call L: batch-1 prefill eager vs captured (bench.py --graph-prefill), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3l; mkdir -p $O
for v in "" "--graph-prefill" "" "--graph-prefill" "" "--graph-prefill"; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $v > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "mode=${v:-eager} $(python -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['prefill_ms'], d['decode_ms_per_token'])")"
done
