"""Per-kernel HBM traffic of the batch-1 decode step from rocprofv3 --pmc passes of scripts/pmc_decode.py:
    python scripts/pmc_decode_summary.py <FETCH_SIZE dir> <WRITE_SIZE dir> <TCC_HIT/MISS dir> out.json
FETCH_SIZE is doubled (gfx950 counts half the bytes of 16-B-per-lane streaming reads, MI355X guide § HBM; the
decode GEMVs, attention and merge all read 16 B per lane).  Only the decode-step dispatches (the last 6 steps'
kernels, identified by name) are kept; per kernel the median over its launches."""
import csv
import glob
import json
import sys
from collections import defaultdict

KERNELS = {  # name prefix -> label
    "void gemv_kernel<2,": "gate/up GEMV (+gelu*up)",
    "void gemv_kernel<7, 1, 2, 8, 0": "down GEMV split 8 (+F32_FIN)",
    "void gemv_kernel<7, 1, 2, 8, 2": "o_proj GEMV + split-KV merge prologue (+F32_FIN)",
    "void gemv_kernel<6,": "q|k|v GEMV (+RoPE, KV append)",
    "void gemv_kernel<3,": "lm_head GEMV",
    "void attn_decode_kernel": "split-KV attention",
}


def load(d, counters):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] in counters:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return per, names


def label(name):
    for k, v in KERNELS.items():
        if name.startswith(k):
            return v
    return None


def by_label(per, names, counter, scale=1.0):
    out = defaultdict(list)
    for d, vals in per.items():
        lb = label(names[d])
        if lb and counter in vals:
            out[lb].append(vals[counter] * scale)
    return {k: sorted(v)[len(v) // 2] for k, v in out.items()}


fper, fnames = load(sys.argv[1], {"FETCH_SIZE"})
wper, wnames = load(sys.argv[2], {"WRITE_SIZE"})
hper, hnames = load(sys.argv[3], {"TCC_HIT_sum", "TCC_MISS_sum"})
fetch = by_label(fper, fnames, "FETCH_SIZE", 2 * 1024)
write = by_label(wper, wnames, "WRITE_SIZE", 1024)
hit = by_label(hper, hnames, "TCC_HIT_sum")
miss = by_label(hper, hnames, "TCC_MISS_sum")
alg = {"gate/up GEMV (+gelu*up)": 2 * 16384 * 2048 * 2, "down GEMV split 8 (+F32_FIN)": 2048 * 16384 * 2,
       "o_proj GEMV + split-KV merge prologue (+F32_FIN)": 2048 * 2048 * 2,
       "q|k|v GEMV (+RoPE, KV append)": 2560 * 2048 * 2, "lm_head GEMV": 257216 * 2048 * 2,
       "split-KV attention": None}
rec = {}
for lb in KERNELS.values():
    if lb not in fetch:
        continue
    r = {"fetch_bytes": round(fetch[lb]), "write_bytes": round(write.get(lb, 0)),
         "tcc_hit": hit.get(lb), "tcc_miss": miss.get(lb)}
    if hit.get(lb) is not None and miss.get(lb) is not None and hit[lb] + miss[lb] > 0:
        r["tcc_hit_rate"] = round(hit[lb] / (hit[lb] + miss[lb]), 4)
    if alg.get(lb):
        r["weight_bytes"] = alg[lb]
        r["fetch_over_weights"] = round(fetch[lb] / alg[lb], 4)
    rec[lb] = r
rec["note"] = ("FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; medians over the eager decode steps of scripts/pmc_decode.py; "
               "separate --pmc passes; the Infinity Cache is memory-side, so MALL hits count as fetched bytes")
json.dump(rec, open(sys.argv[4], "w"), indent=1)
print(json.dumps(rec, indent=1))
