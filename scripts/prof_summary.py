"""Per-kernel totals from a rocprofv3 SQLite result (rocprofv3 -d DIR -o run, default output format):
    python scripts/prof_summary.py gpurun_out/p896/run_results.db [top]
Kernel names are shortened to the template head; rows: total ms, launches, average us, share."""
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([\w:]+)(<[^()]*>)?", name)
    head = m.group(1) if m else name[:60]
    targs = (m.group(2) or "")[:60] if m else ""
    return head + targs


def main():
    db, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: [0, 0])
    total = 0
    for name, dur in c.execute("select name, duration from kernels"):
        k = short(name)
        agg[k][0] += dur
        agg[k][1] += 1
        total += dur
    print(f"{'kernel':80s} {'total ms':>10s} {'n':>7s} {'avg us':>9s} {'share':>6s}")
    for k, (d, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{k[:80]:80s} {d / 1e6:10.2f} {n:7d} {d / n / 1e3:9.1f} {d / total:6.1%}")
    print(f"{'total':80s} {total / 1e6:10.2f}")


if __name__ == "__main__":
    main()
