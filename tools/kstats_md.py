#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv as a markdown table (top-N kernels).

usage: kstats_md.py run_kernel_stats.csv [--top N] [--steps S]   (S: divide totals by S -> ms/step)
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"at::native::", "", name)
    if name.startswith(("Cijk_", "Custom_Cijk_")):
        mt = re.search(r"MT\d+x\d+x\d+", name)
        return name.split("_BBS")[0].split("_UserArgs")[0][:32] + (f" {mt.group(0)}" if mt else "") + " (hipBLASLt)"
    return name.split("(")[0][:90] if not name.startswith("void") else name[5:].split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=float, default=1.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(int(r["TotalDurationNs"]) for r in rows)
    steps = a.steps if a.steps > 0 else 1.0  # 0: no per-step division
    print(f"total kernel time {tot / 1e6:.1f} ms over {a.steps:g} steps = {tot / 1e6 / steps:.1f} ms/step\n")
    print("| kernel | calls | mean us | ms/step | % time |")
    print("|---|---|---|---|---|")
    for r in rows[: a.top]:
        t = int(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{t / 1e6 / steps:.2f} | {100 * t / tot:.2f} |")


if __name__ == "__main__":
    main()
