"""Aggregate one prefill's kernels (the segment between the image-rank scan and the next decode step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("im2col")]
i0 = starts[len(starts) // 2]
i1 = next(i for i in range(i0 + 1, len(rows)) if rows[i]["Kernel_Name"].startswith("argmax_final"))
agg = {}
for r in rows[i0:i1 + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = (r["Kernel_Name"][:26], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"],
         r["LDS_Block_Size"])
    agg.setdefault(k, []).append(d)
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{k[0]:26s} wgs={k[1]:6d} y={k[2]:>3s} z={k[3]:>3s} lds={k[4]:>6s} n={len(v):3d} avg={sum(v)/len(v):7.2f}us "
          f"tot={sum(v):8.1f}us")
print("sum of kernel time", round(tot, 1), "us; wall", (int(rows[i1]["End_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3)
