# round 2, call X: the persistent MLP engine (pg_decode_mlp_engine): parity test, stamps, graph-timed decode step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "mlp_engine" > $O/test.log 2>&1; rc=$?
tail -15 $O/test.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/r02/engine_stamps.py > $O/stamps.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
cat $O/stamps.txt
PG_MLP_ENGINE=1 timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_on.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_off.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
echo "on $(cut -c1-150 $O/step_on.json)"; echo "off $(cut -c1-150 $O/step_off.json)"
