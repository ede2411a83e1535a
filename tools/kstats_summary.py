#!/usr/bin/env python3
"""Group a rocprofv3 kernel_stats.csv by kernel family and print the top kernels.

usage: kstats_summary.py <kernel_stats.csv> [steps]   (per-step ms when steps is given)
       kstats_summary.py --trace <kernel_trace.csv> <marker-regex> <last-n-steps> <total-steps>
The --trace form keeps only the kernels of the last n steps: the marker (e.g. the optimizer
kernel) launches the same number of times every step (total markers / total steps), and the
window starts after the marker launch that ends step total-n.  One-off work such as MIOpen's
algorithm search at start-up then does not pollute the steady-state picture.
"""
import csv
import re
import sys

FAMILIES = [
    ("batch-norm", r"batch_norm|batchnorm|MIOpenBatchNorm|\bbn_|::bn_"),
    ("conv bwd-weight", r"bwd_weight|wrw"), ("conv bwd-data", r"bwd_data|igemm_bwd|naive_conv.*_bwd_"),
    ("conv fwd", r"conv.*fwd|fwd.*conv|igemm|xdl.*conv"), ("gemm", r"Cijk|gemm|hipblaslt"),
    ("sgd/optimizer", r"sgd|multi_tensor|foreach|_fused_"), ("reduce", r"reduce"),
    ("elementwise", r"elementwise|vectorized|unrolled"), ("pool", r"pool"),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name, re.I):
            return fam
    return "other"


def from_trace(path, marker, last_n, total_steps):
    ks = list(csv.DictReader(open(path)))
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(ks) if re.search(marker, r["Kernel_Name"])]
    per = len(marks) // total_steps
    if per < 1 or len(marks) % total_steps or last_n >= total_steps:
        raise SystemExit(f"{len(marks)} marker kernels do not divide into {total_steps} steps")
    keep = ks[marks[-last_n * per - 1] + 1:marks[-1] + 1]
    agg = {}
    for r in keep:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg.setdefault(r["Kernel_Name"], [0, 0])
        a[0] += 1
        a[1] += d
    span = int(keep[-1]["End_Timestamp"]) - int(keep[0]["Start_Timestamp"])
    print(f"steady state: {last_n} steps, {len(keep)} kernels, {span / 1e6 / last_n:.2f} ms/step first-start to last-end\n")
    return [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": t / c} for n, (c, t) in agg.items()]


def main():
    if sys.argv[1] == "--trace":
        rows = from_trace(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
        steps = float(sys.argv[4])
    else:
        rows = list(csv.DictReader(open(sys.argv[1])))
        steps = float(sys.argv[2]) if len(sys.argv) > 2 else None
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = {}
    for r in rows:
        f = family(r["Name"])
        fam[f] = fam.get(f, 0.0) + float(r["TotalDurationNs"])
    unit = f"ms/step over {steps:g} steps" if steps else "ms total"
    div = 1e6 * (steps or 1)
    print(f"| family | {unit} | share |\n|---|---|---|")
    for f, t in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"| {f} | {t / div:.2f} | {100 * t / tot:.1f} % |")
    print(f"| total | {tot / div:.2f} | |\n")
    print(f"| kernel | calls | {unit} | avg us |\n|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
        n = r["Name"]
        n = (n[:110] + "...") if len(n) > 113 else n
        print(f"| `{n}` | {r['Calls']} | {float(r['TotalDurationNs']) / div:.2f} | {float(r['AverageNs']) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
