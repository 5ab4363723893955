# PMC pass over the pt-224 batch-1 prefill (gpurun_out/$1): per kernel type MFMA busy, wave-cycle breakdown,
# LDS bank conflicts, summed over its dispatches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcp}; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/p -o run --output-format csv -- python scripts/tune/prefill_time.py --reps 2 > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
python - $O/p <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(float)); names = {}
for r in csv.DictReader(open(f)):
    d = int(r["Dispatch_Id"]); per[d][r["Counter_Name"]] += float(r["Counter_Value"]); names[d] = r["Kernel_Name"][:60]
agg = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(int)
for d, v in per.items():
    cnt[names[d]] += 1
    for k, x in v.items(): agg[names[d]][k] += x
rows = sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"])
for n, v in rows[:16]:
    wc = v["SQ_WAVE_CYCLES"] or 1; cyc = v["GRBM_GUI_ACTIVE"] / 8
    print("%-60s n=%3d cyc/disp %7.0f mfma %.3f wait_any %.2f wait_inst %.2f active %.2f lds_conf %.3f" % (
        n, cnt[n], cyc / cnt[n], v["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * cyc), v["SQ_WAIT_ANY"] / wc,
        v["SQ_WAIT_INST_ANY"] / wc, v["SQ_ACTIVE_INST_ANY"] / wc, v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"])))
PY
