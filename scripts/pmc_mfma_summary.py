"""MFMA utilisation of the gemm256 dispatches from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_BUSY_CU_CYCLES pass (scripts/gpu_pmc_mfma.sh).  Per dispatch:
  clock     = GRBM_GUI_ACTIVE / 8 XCDs / wall  (MI355X_MICROARCH.md, DVFS give-back)
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)
and, beside it, the flop-derived fraction 2*M*N*K / wall / 2.5 PF/s from the shape each dispatch ran."""
import csv
import json
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
by = defaultdict(dict)
meta = {}
for r in rows:
    if "gemm256" not in r["Kernel_Name"]:
        continue
    d = int(r["Dispatch_Id"])
    by[d][r["Counter_Name"]] = float(r["Counter_Value"])
    meta[d] = (int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
shapes = {8320 * 512: ("gemma_gu_nofrag (16512x32768x2048)", 2 * 16512 * 32768 * 2048),  # grid = tiles * 512
          1024 * 512: ("sq8192", 2 * 8192 ** 3)}
out = {}
for d in sorted(by):
    c, (grid, wall) = by[d], meta[d]
    if "GRBM_GUI_ACTIVE" not in c or "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
        continue
    name, flops = shapes.get(grid, (f"grid{grid}", None))
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 256 * 4)
    rec = out.setdefault(name, [])
    rec.append({"wall_us": round(wall * 1e6, 1), "clock_ghz": round(cyc / wall / 1e9, 3), "mfma_busy_frac": round(util, 4),
                "flop_frac_of_2.5PF": round(flops / wall / 2.5e15, 4) if flops else None})
print(json.dumps({k: v[-3:] for k, v in out.items()}, indent=1))
