"""Print one decode step of a rocprofv3 kernel_trace.csv as a timeline (start / end relative to the step's first
kernel, both streams interleaved): python scripts/r02/bank_timeline.py <kernel_trace.csv> [step index from the end]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ends = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("argmax_final")]
a, b = ends[-1 - back], ends[-back]
t0 = int(rows[a + 1]["Start_Timestamp"])
for r in rows[a + 1: b + 1]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{r['Kernel_Name'][:34]:34s} q={r.get('Queue_Id', r.get('Stream_Id', '?')):>3s} "
          f"grid={r['Grid_Size_X']:>7s} start={s:8.2f} end={e:8.2f} dur={e - s:6.2f}")
print("step", (int(rows[b]["End_Timestamp"]) - t0) / 1e3, "us")
