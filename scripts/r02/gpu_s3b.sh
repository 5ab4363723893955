# round 2, session 3, call B: two-stream decode (pg_gateup_bank + pro-7 q|k|v): kernel + engine bit-exactness, then
# the graph-replayed pt-224 decode step with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3b; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py -k "gateup_bank or two_stream" > $O/test.log 2>&1
rc=$?; tail -5 $O/test.log; [ $rc -eq 0 ] || exit 1
for v in "PG_DECODE_BANK=0" "PG_DECODE_BANK=0 PG_SK_SMALL=64" "PG_DECODE_BANK=1" "PG_DECODE_BANK=0" "PG_DECODE_BANK=1"; do
  env $v timeout -k 10 200 python -u scripts/tune/decode_step.py --steps 100 > $O/step.json 2> $O/step.err || { tail -5 $O/step.err; exit 1; }
  echo "$v $(cat $O/step.json)"
done
