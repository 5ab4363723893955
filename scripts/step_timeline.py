"""Print one decode step's kernel timeline from a rocprofv3 kernel_trace.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("embed_merge") and int(r["Grid_Size_X"]) <= 16384]
if len(idx) < 3:    # chained greedy decode (no embed launch): steps end at the argmax's final launch
    idx = [i + 1 for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("argmax_final", "argmax_embed_onepass"))]
segs = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]), a, b) for a, b in zip(idx, idx[1:])]
segs = sorted(s for s in segs if s[2] - s[1] < 400)   # decode steps only (prefill spans hundreds of kernels)
_, i0, i1 = segs[len(segs) // 2]
t0 = int(rows[i0]["Start_Timestamp"])
agg = {}
for r in rows[i0:i1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = (r["Kernel_Name"][:28], r["Grid_Size_X"], r["Grid_Size_Y"])
    agg.setdefault(k, []).append(d)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:28s} grid={k[1]:>7s},{k[2]:>2s} n={len(v):3d} avg={sum(v)/len(v):7.2f}us tot={sum(v):8.1f}us")
print("step wall", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, "us")
