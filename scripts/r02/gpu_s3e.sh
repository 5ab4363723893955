# round 2, session 3, call E: two-stream decode variants with per-layer GEMV / bank-kernel stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s3e; mkdir -p $O
i=0
for v in "PG_DECODE_BANK=0" "PG_DECODE_BANK=1 PG_BANK_INFL=0" "PG_DECODE_BANK=1 PG_BANK_INFL=8" "PG_DECODE_BANK=1 PG_BANK_INFL=4" "PG_DECODE_BANK=1 PG_BANK_INFL=16" "PG_DECODE_BANK=1 PG_BANK_INFL=8 PG_BANK_QKV_WAIT=0"; do
  i=$((i+1))
  env $v timeout -k 10 200 python -u scripts/r02/bank_probe2.py > $O/v$i.txt 2>&1 || { tail -5 $O/v$i.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/v$i.txt | head -1; sed -n '3,6p;12,13p' $O/v$i.txt
done
