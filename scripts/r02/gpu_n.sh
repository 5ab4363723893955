# round 2, call N: decode MLP block ring-depth variants: in-kernel stamps + graph-timed decode step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_off.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
echo "off $(cat $O/step_off.json)"
for v in base s32 s32c s127c s8c; do
  if [ $v = base ]; then L=""; else L=scripts/tune/mlp_$v.so; fi
  PGHIP_LIB=$L PG_MLP_BLOCK=1 timeout -k 10 200 python scripts/tune/decode_step.py --steps 50 > $O/step_$v.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  PGHIP_LIB=$L timeout -k 10 200 python scripts/r02/mlp_stamps.py > $O/stamps_$v.txt 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$v $(cat $O/step_$v.json)"
  tail -1 $O/stamps_$v.txt
done
