# PMC pass over the prefill flash attention at the long shapes (gpurun_out/$1): wave-cycle breakdown, MFMA busy, LDS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmca}; mkdir -p $O
REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/p -o run --output-format csv -- python scripts/tune/attn_bench.py --only gemma448x16,siglip448x16,gemma896x32,siglip896x32 > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
grep -v amdgpu $O/p.log | tail -4
python - $O/p <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(float)); names = {}
for r in csv.DictReader(open(f)):
    d = int(r["Dispatch_Id"]); per[d][r["Counter_Name"]] += float(r["Counter_Value"]); names[d] = r["Kernel_Name"][:60]
for d in sorted(per):
    v = per[d]
    if "attn_fa" not in names[d]: continue
    wc = v["SQ_WAVE_CYCLES"] or 1
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print(names[d], "mfma_busy/(cu*4 simd*cyc) %.3f" % (v["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * cyc)),
          "wait_any %.2f wait_inst %.2f active %.2f wait_lds %.3f lds_conflict/idx %.3f" % (
          v["SQ_WAIT_ANY"] / wc, v["SQ_WAIT_INST_ANY"] / wc, v["SQ_ACTIVE_INST_ANY"] / wc, v["SQ_WAIT_INST_LDS"] / wc,
          v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"])))
PY
