# round 2, call Y: MLP engine variants (loader thinning during the gather, gather sweep interval)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "mlp_engine" > $O/test.log 2>&1 || { tail -15 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in base; do
  if [ $v = base ]; then L=""; else L=scripts/tune/en_$v.so; fi
  PGHIP_LIB=$L timeout -k 10 200 python scripts/r02/engine_stamps.py > $O/stamps_$v.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  PGHIP_LIB=$L PG_MLP_ENGINE=1 timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_$v.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('$O/step_$v.json'));print(d['ms_per_token'])")"; tail -1 $O/stamps_$v.txt
done
timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_off.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
echo "off $(python -c "import json;d=json.load(open('$O/step_off.json'));print(d['ms_per_token'])")"
