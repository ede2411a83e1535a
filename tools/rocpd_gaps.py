#!/usr/bin/env python3
"""Inter-kernel gaps from a rocprofv3 kernel-trace DB: for each consecutive kernel pair
(A -> B on the same queue order) the median idle time between A's end and B's start,
plus the median duration of each kernel.  Shows how much of a step is launch seams.

usage: rocpd_gaps.py run_results.db [--skip N]   (ignore the first N dispatches: warm-up)
"""
import re
import sqlite3
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    return re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0][:40]


def main():
    db = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 200
    rows = list(sqlite3.connect(db).execute("select name, start, end from kernels order by start"))[skip:]
    gaps, durs = defaultdict(list), defaultdict(list)
    for (n0, s0, e0), (n1, s1, e1) in zip(rows, rows[1:]):
        gaps[(short(n0), short(n1))].append((s1 - e0) / 1e3)
    for n, s, e in rows:
        durs[short(n)].append((e - s) / 1e3)
    print("| kernel | median duration us |")
    print("|---|---|")
    for k, v in sorted(durs.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"| {k} | {statistics.median(v):.2f} |")
    print("\n| seam (A -> B) | count | median gap us |")
    print("|---|---|---|")
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        if len(v) >= 10:
            print(f"| {a} -> {b} | {len(v)} | {statistics.median(v):.2f} |")
    span = (rows[-1][2] - rows[0][1]) / 1e3
    busy = sum(e - s for _, s, e in rows) / 1e3
    print(f"\nwall {span:.0f} us, kernels busy {busy:.0f} us ({100 * busy / span:.1f} %)")


if __name__ == "__main__":
    main()
