# PMC pass over the prefill GEMMs (bf16 gemm256 / fp8 gemm8) at the pt-448 x16 Gemma shapes and square shapes
# (gpurun_out/$1): MFMA busy, wave-cycle breakdown, LDS bank conflicts per kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcg}; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/p -o run --output-format csv -- python scripts/tune/gemm8_bench.py > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
grep -v amdgpu $O/p.log | tail -8
python - $O/p <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(float)); names = {}
for r in csv.DictReader(open(f)):
    d = int(r["Dispatch_Id"]); per[d][r["Counter_Name"]] += float(r["Counter_Value"]); names[d] = r["Kernel_Name"][:70]
seen = defaultdict(int)
for d in sorted(per):
    v = per[d]
    if "gemm" not in names[d] or v["GRBM_GUI_ACTIVE"] < 8 * 20000: continue
    seen[names[d]] += 1
    if seen[names[d]] > 2: continue
    wc = v["SQ_WAVE_CYCLES"] or 1
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print(names[d], "cyc %.0f mfma_busy %.3f wait_any %.2f wait_inst %.2f active %.2f wait_lds %.3f lds_conflict/idx %.3f" % (
          cyc, v["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * cyc), v["SQ_WAIT_ANY"] / wc, v["SQ_WAIT_INST_ANY"] / wc,
          v["SQ_ACTIVE_INST_ANY"] / wc, v["SQ_WAIT_INST_LDS"] / wc, v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"])))
PY
