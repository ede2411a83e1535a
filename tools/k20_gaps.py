#!/usr/bin/env python3
"""Break a short timed region (bench.py --steps 20 --warmup 5) into host launch latency,
GPU busy time, inter-kernel gaps and the host's synchronize tail, from a rocprofv3
``--kernel-trace --hip-runtime-trace --output-format csv`` run (tools/gpu/profile.sh with --hip-runtime-trace added).

The timed region is the last run of hipGraphLaunch calls followed by a synchronize."""
import csv
import glob
import json
import sys


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main(d):
    api = rows(f"{d}/**/*hip_api_trace.csv")
    ker = rows(f"{d}/**/*kernel_trace.csv")
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    ker.sort(key=lambda r: int(r["Start_Timestamp"]))
    launches = [i for i, r in enumerate(api) if r["Function"] == "hipGraphLaunch"]
    # last block of consecutive graph launches
    last = launches[-1]
    first = last
    while first - 1 in launches or (first - 1 >= 0 and api[first - 1]["Function"] == "hipGraphLaunch"):
        first -= 1
    syncs = [r for r in api[last + 1:] if "Synchronize" in r["Function"]]
    t_l0 = int(api[first]["Start_Timestamp"])
    t_l1 = int(api[last]["End_Timestamp"])
    t_sync_end = int(syncs[0]["End_Timestamp"])
    ks = [k for k in ker if t_l0 <= int(k["Start_Timestamp"]) <= t_sync_end]
    k0 = int(ks[0]["Start_Timestamp"])
    k1 = max(int(k["End_Timestamp"]) for k in ks)
    busy = sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks)
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(ks, ks[1:])]
    names = {}
    for k in ks:
        n = k["Kernel_Name"].split("(")[0][:40]
        names.setdefault(n, []).append(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]))
    res = {
        "graph_launches": last - first + 1,
        "kernels": len(ks),
        "region_us (first launch call -> sync return)": round((t_sync_end - t_l0) / 1e3, 2),
        "launch_call_to_first_kernel_us": round((k0 - t_l0) / 1e3, 2),
        "host_launch_calls_us": round((t_l1 - t_l0) / 1e3, 2),
        "gpu_span_us": round((k1 - k0) / 1e3, 2),
        "kernel_busy_us": round(busy / 1e3, 2),
        "sum_gaps_us": round(sum(gaps) / 1e3, 2),
        "max_gap_us": round(max(gaps) / 1e3, 2) if gaps else 0,
        "last_kernel_end_to_sync_return_us": round((t_sync_end - k1) / 1e3, 2),
        "first_step_kernels_us": [round((int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3, 2) for k in ks[:6]],
        "median_kernel_us": {n: round(sorted(v)[len(v) // 2] / 1e3, 2) for n, v in names.items()},
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/k20/trace")
