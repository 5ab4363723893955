"""Analyse a rocprofv3 kernel trace of scripts/tune/mall_probe.py (phases split at the 1024-WG flush kernels)."""
import csv
import sys

NAMES = sys.argv[2].split(",") if len(sys.argv) > 2 else \
    ["gu_cold", "gu_warm", "dn_cold", "dn_warm", "chain", "chain_pf32", "chain_pf64", "chain_pf128", "chain_pf256", "end"]
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void prefetch_kernel") or
         r["Kernel_Name"].startswith("prefetch_kernel")]
marks = [i for i in marks if rows[i]["Grid_Size_X"] == str(1024 * 256)]
marks = marks[-len(NAMES):]
for n, (a, b) in zip(NAMES, zip(marks, marks[1:] + [len(rows)])):
    seg = rows[a + 1:b]
    if not seg:
        continue
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    agg = {}
    for r in seg:
        k = (r["Kernel_Name"].split("(")[0].replace("void ", "")[:26], r["Grid_Size_X"], r["Grid_Size_Y"])
        agg.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"== {n}: span {(t1 - t0) / 1e3:9.1f} us, {len(seg)} kernels")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        print(f"   {k[0]:26s} grid={k[1]:>7s},{k[2]:>2s} n={len(v):3d} med={v[len(v) // 2]:7.2f} min={v[0]:7.2f}")
