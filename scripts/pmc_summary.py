"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of scripts/pmc_gateup.py into
profiles/<out>.json: per-launch HBM bytes of the gate/up GEMV, FETCH_SIZE doubled (gfx950: FETCH_SIZE
reports half the bytes of 16-B-per-lane streaming reads, MI355X_MICROARCH.md § HBM)."""
import csv
import glob
import json
import sys


def per_dispatch(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter and r["Kernel_Name"].startswith("void gemv_kernel<2"):
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sorted(vals.values())


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
med = lambda v: v[len(v) // 2]  # noqa: E731
alg = 2 * 16384 * 2048 * 2 + 2048 * 2 + 16384 * 2
rec = {"kernel": "gemv_kernel<GELU_MUL,2> decode gate/up (bench.py roofline kernel)",
       "launches": len(fetch), "fetch_size_kb_median": med(fetch), "write_size_kb_median": med(write),
       "fetch_bytes_per_launch": med(fetch) * 1024 * 2, "write_bytes_per_launch": med(write) * 1024,
       "algorithmic_bytes_per_launch": alg,
       "note": "FETCH_SIZE x2 (gfx950 half-count of 16-B streaming reads); separate --pmc passes"}
rec["traffic_bytes_per_launch"] = rec["fetch_bytes_per_launch"] + rec["write_bytes_per_launch"]
rec["traffic_over_algorithmic"] = rec["traffic_bytes_per_launch"] / alg
json.dump(rec, open(sys.argv[3], "w"), indent=1)
print(json.dumps(rec))
