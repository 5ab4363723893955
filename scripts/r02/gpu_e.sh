# round 2, call E: GEMV ring-depth / CPW variants (graph-timed micro-bench) + decode step per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02e; mkdir -p $O
run() {  # env assignments..., then the tag
  env "$@" timeout -k 10 200 python scripts/r02/gemv_bench.py > $O/one 2>&1 || { cat $O/one; return 1; }
  echo "$* $(tail -1 $O/one)" >> $O/gemv.log
  env "$@" timeout -k 10 200 python scripts/tune/decode_step.py --steps 100 > $O/one 2>&1 || { cat $O/one; return 1; }
  echo "$* $(tail -1 $O/one | grep -o '"ms_per_token": [0-9.]*') $(tail -1 $O/one | grep -o '"ids16": \[[0-9]*, [0-9]*, [0-9]*')" >> $O/dec.log
}
for r in 1 2; do
  run X=0 || exit 1
  run PG_GEMV_CPW_OFF=1 || exit 1
  run PG_GEMV_D_NT2=3 || exit 1
  run PG_GEMV_D_NT2=2 || exit 1
  run PG_GEMV_D_NT1=6 || exit 1
  run PG_GEMV_D_NT1=4 || exit 1
done
cat $O/gemv.log $O/dec.log
