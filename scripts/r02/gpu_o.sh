# round 2, call O: MLP block defaults re-check (test + timing) and the pt-448 B=16 decode step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "mlp_block" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
PG_MLP_BLOCK=1 timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_on.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_off.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
echo "on $(cut -c1-120 $O/step_on.json)"; echo "off $(cut -c1-120 $O/step_off.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d16 -o run --output-format csv -- python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 20 > $O/d16.log 2>&1 || { tail -5 $O/d16.log; exit 1; }
python scripts/step_timeline.py $O/d16/run_kernel_trace.csv > $O/decode_step_timeline_448x16.txt
cat $O/decode_step_timeline_448x16.txt
