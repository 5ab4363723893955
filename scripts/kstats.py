"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{r['Name'][:60]:60s} calls={int(r['Calls']):7d} avg_us={float(r['AverageNs'])/1e3:9.2f} "
          f"tot_ms={float(r['TotalDurationNs'])/1e6:9.2f} {100*float(r['TotalDurationNs'])/tot:5.1f}%")
