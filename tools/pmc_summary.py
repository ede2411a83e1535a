#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc csv outputs (counter_collection.csv) per kernel (mean per dispatch)."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return n.split("(")[0][:40]


def main(paths):
    vals = defaultdict(lambda: defaultdict(list))
    for p in paths:
        per = defaultdict(lambda: defaultdict(float))
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), d in per.items():
            for c, v in d.items():
                vals[k][c].append(v)
    ctrs = sorted({c for k in vals for c in vals[k]})
    for k in sorted(vals):
        print(f"== {k}")
        for c in ctrs:
            if c in vals[k]:
                v = vals[k][c]
                print(f"   {c:28s} {sum(v)/len(v):14.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
