# round 2, call ZC: PG_TILE_M1 batch-1 prefill GEMMs: kernel test, pt-224 engine parity, bench prefill on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zc; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "tile_m1 or pt224 or greedy" > $O/test.log 2>&1 || { tail -15 $O/test.log; exit 1; }
tail -1 $O/test.log
for m in 1 0 1 0; do
  PG_TILE_M1=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $O/bench_$m.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  echo "tile_m1=$m $(python -c "import json;d=json.load(open('$O/bench_$m.json'));print(d['value'], d['prefill_ms'])")"
done
