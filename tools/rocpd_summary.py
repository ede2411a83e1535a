#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite DB (kernel-trace) as a markdown table.

usage: rocpd_summary.py run_results.db [--last N]   (N = only the last N dispatches of each kernel)
"""
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:60]


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration, grid_x, grid_y, workgroup_x, vgpr_count, accum_vgpr_count, lds_size from kernels order by start"))
    agg = defaultdict(list)
    meta = {}
    for name, dur, gx, gy, wx, v, a, lds in rows:
        k = short(name)
        agg[k].append(dur)
        meta[k] = (gx // max(wx, 1), gy, wx, v, a, lds)
    tot = sum(sum(v) for v in agg.values())
    print("| kernel | calls | mean us | median us | % time | grid(blocks x y) | block | vgpr/agpr | LDS B |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        v2 = sorted(v)
        m = meta[k]
        print(f"| {k} | {len(v)} | {sum(v)/len(v)/1e3:.2f} | {v2[len(v2)//2]/1e3:.2f} | {100*sum(v)/tot:.1f} | {m[0]}x{m[1]} | {m[2]} | {m[3]}/{m[4]} | {m[5]} |")
    print(f"\ntotal kernel time {tot/1e6:.2f} ms over {len(rows)} dispatches")


if __name__ == "__main__":
    main()
