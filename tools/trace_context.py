#!/usr/bin/env python3
"""List the kernels of ONE steady-state step that match a regex, in launch order, with grid size,
duration and the kernels launched just before / after them (where in the step they sit).

usage: trace_context.py <kernel_trace.csv> <match-regex> <step-marker-regex> <total-steps> [min_us]
(the marker, e.g. the optimizer kernel, launches the same number of times every step)
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::|at::native::", "", n)
    return (n[5:] if n.startswith("void ") else n).split("(")[0][:70]


def main():
    path, pat, marker = sys.argv[1], sys.argv[2], sys.argv[3]
    total = int(sys.argv[4])
    min_us = float(sys.argv[5]) if len(sys.argv) > 5 else 0.0
    ks = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(ks) if re.search(marker, r["Kernel_Name"])]
    per = len(marks) // total
    if per < 1 or len(marks) % total:
        raise SystemExit(f"{len(marks)} marker kernels do not divide into {total} steps")
    lo, hi = marks[-per - 1] + 1, marks[-1] + 1  # the last whole step
    for i in range(lo, hi):
        r = ks[i]
        if not re.search(pat, r["Kernel_Name"]):
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if us < min_us:
            continue
        g = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        print(f"{i - lo:4d} {us:8.1f} us grid={g:>9} {short(r['Kernel_Name'])}\n"
              f"       before: {short(ks[i - 1]['Kernel_Name'])}\n       after:  {short(ks[i + 1]['Kernel_Name'])}")


if __name__ == "__main__":
    main()
