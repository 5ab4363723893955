"""MFMA busy fraction over one prefill (the kernels from an im2col to the next argmax_final) of a rocprofv3
--pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass (scripts/gpu_pmc_prefill.sh):
  sum(SQ_VALU_MFMA_BUSY_CYCLES) / sum(GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs), by kernel family too."""
import csv
import json
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
disp = defaultdict(dict)
for r in rows:
    d = disp[int(r["Dispatch_Id"])]
    d[r["Counter_Name"]] = float(r["Counter_Value"])
    d["name"] = r["Kernel_Name"]
    d["t"] = int(r["Start_Timestamp"])
    d["wall"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
order = sorted(disp, key=lambda k: disp[k]["t"])
starts = [i for i, k in enumerate(order) if disp[k]["name"].startswith("im2col")]
i0 = starts[-1]
i1 = next(i for i in range(i0 + 1, len(order)) if disp[order[i]]["name"].startswith("argmax_final"))
fam = defaultdict(lambda: [0.0, 0.0, 0.0])
for k in order[i0:i1 + 1]:
    d = disp[k]
    f = d["name"].split("<")[0].split("(")[0].replace("void ", "")
    fam[f][0] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    fam[f][1] += d.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 256 * 4
    fam[f][2] += d["wall"]
tot_b = sum(v[0] for v in fam.values())
tot_c = sum(v[1] for v in fam.values())
tot_w = sum(v[2] for v in fam.values())
out = {"prefill_kernel_us": round(tot_w, 1), "mfma_busy_frac": round(tot_b / tot_c, 4),
       "by_kernel": {f: {"us": round(v[2], 1), "mfma_busy_frac": round(v[0] / v[1], 4) if v[1] else None}
                     for f, v in sorted(fam.items(), key=lambda kv: -kv[1][2])}}
print(json.dumps(out, indent=1))
