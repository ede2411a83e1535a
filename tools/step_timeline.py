#!/usr/bin/env python3
"""In-situ timeline of the stream-launched MNIST training step (what the bench times).

Every kernel launcher hands its launch the next slot of the debug buffer (mnist_kernels.hip
``dbg_next``), so capturing two whole steps gives each of their launches its own slot.  The
captured kernel list is then launched straight onto the stream (``GraphedStep``'s
``launch="stream"`` path) for ``--steps`` steps; the stamps left behind are those of the last
two steps.  Per kernel this prints, on the 100 MHz wall clock every CU shares:

  start   first block's first stamp, relative to the first kernel of the pair
  span    first block start -> last block's last stamp (the kernel as its waves see it)
  p50end  median block end (tail imbalance = span - p50end)
  gap     this kernel's first block start - the previous kernel's last block end: the
          dependent-launch boundary as the GPU sees it (dispatch, cache maintenance, ramp)

    python tools/step_timeline.py [--steps 400] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_operator_amd.data.synthetic import make_synthetic_mnist  # noqa: E402
from pytorch_operator_amd.models.mnist import FusedMnistTrainer  # noqa: E402
from pytorch_operator_amd.ops import mnist as K  # noqa: E402
from pytorch_operator_amd.parallel.graphed_step import NativeGraph  # noqa: E402

SLOT_U64 = 1024 * 16  # mnist_kernels.hip kDbgSlotU64
NAMES = ["conv12_fwd", "fc1_fwd", "head", "fc1_bwd", "conv_bwd4", "tail"]
if os.environ.get("PTO_FUSE_HEAD", "1") != "0" and os.environ.get("PTO_W1_TAIL", "1") != "0":
    NAMES = ["conv12_fwd", "fc1_fwd", "fc1_bwd_head", "conv_bwd4", "tail"]
# block ranges of the launches that run several jobs (B = 64): name -> [(first, end, job)]
# (fc1_bwd: the dz2 job takes the first ids, mnist_kernels.hip fc1_bwd_kernel's block layout)
# (round 5 default, w1_tail: fc1_bwd has no dW_fc1 job; the tail's first 400 blocks are the dW_fc1
# tiles + their SGD; PTO_W1_TAIL=0 restores the round-4 layout)
if os.environ.get("PTO_W1_TAIL", "1") != "0" and os.environ.get("PTO_FUSE_HEAD", "1") != "0":
    GROUPS = {"fc1_bwd_head": [(0, 200, "head+dz2"), (200, 216, "stage")],
              "tail": [(0, 400, "dW_fc1+sgd"), (400, 408, "fc2+sgd+stats"), (408, 609, "conv reduce+sgd")]}
elif os.environ.get("PTO_W1_TAIL", "1") != "0":
    GROUPS = {"fc1_bwd": [(0, 200, "dz2"), (200, 204, "fc2+stats"), (204, 220, "stage")],
              "tail": [(0, 400, "dW_fc1+sgd"), (400, 601, "conv reduce+sgd"), (601, 606, "fc2 sgd")]}
else:
    GROUPS = {"fc1_bwd": [(0, 200, "dz2"), (200, 400, "dW_fc1"), (400, 404, "fc2+stats"), (404, 420, "stage")],
              "tail": [(0, 201, "conv reduce+sgd"), (201, 598, "fc sgd")]}


def analyse(dbg: torch.Tensor, nslots: int):
    out = []
    d_all = dbg.view(-1, 16).cpu()
    for k in range(nslots):
        d = d_all[k * 1024:(k + 1) * 1024]
        used = d[:, 0] > 0
        w = d[used][:, :8].double()
        valid = w > 0
        last = (w * valid).max(1).values
        idx = torch.nonzero(used).flatten()
        both = valid[:, 1:] & valid[:, :-1]
        dph = (w[:, 1:] - w[:, :-1]) * both
        phases = (dph.sum(0) / both.sum(0).clamp_min(1) / 100.0).tolist()
        nph = int(both.any(0).sum())
        # effective shader clock per phase: clock64 ticks (stamps 8-15) / wall_clock64 (100 MHz)
        c = d[used][:, 8:].double()
        cv = (c[:, 1:] > 0) & (c[:, :-1] > 0) & both
        dc = (c[:, 1:] - c[:, :-1]) * cv
        dw = (w[:, 1:] - w[:, :-1]) * cv
        ghz = (dc.sum(0) / dw.sum(0).clamp_min(1) / 10.0).tolist()  # ticks per 10 ns -> GHz
        # stamp 7 written by another wave than stamps 0-5 (conv_bwd4: group B's 2b done): us after stamp 1
        aux = None
        if nph < 6 and bool((w[:, 7] > 0).any()):
            ok = (w[:, 7] > 0) & (w[:, 1] > 0)
            aux = float(((w[:, 7] - w[:, 1]) * ok).sum() / ok.sum().clamp_min(1) / 100.0)
        out.append({"aux71": aux, "blocks": int(used.sum()), "start": float(w[:, 0].min()), "end": float(last.max()),
                    "p50end": float(last.median()), "block_end": dict(zip(idx.tolist(), last.tolist())),
                    "phases": phases[:nph], "ghz": ghz[:nph],
                    "block_rows": {"idx": idx, "w": w, "valid": valid}})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--json", default=None)
    ap.add_argument("--reps", type=int, default=5, help="timelines sampled (each after --steps steps)")
    ap.add_argument("--by-mod", action="append", default=[], metavar="KERNEL:N",
                    help="per-block breakdown of KERNEL (second step) grouped by block id %% N: start, "
                         "phase times and end relative to the kernel's first stamp, plus the latest blocks")
    ap.add_argument("--conv1-waves", action="store_true",
                    help="diagnostic build (-DPTO_MNIST_STAMPW): conv12_fwd's per-wave conv1 stamps")
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    ds = make_synthetic_mnist(60000, seed=1, device=dev)
    cur = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cur)
    tr = FusedMnistTrainer(batch_size=64, source=src, lr=0.01, momentum=0.5, device=dev, seed=1)
    for _ in range(3):
        tr.train_step()
    torch.cuda.synchronize()
    dbg = torch.zeros(16 * SLOT_U64, dtype=torch.int64, device=dev)
    K.set_debug_buffer(dbg)

    def two_steps():
        tr.train_step()
        tr.train_step()
    g = NativeGraph(two_steps, dev)
    K.set_debug_buffer(None)  # later launches (none) would not stamp; the captured ones keep dbg
    if not g.stream_ok:
        raise SystemExit("captured step holds non-kernel nodes")
    nk = g.nodes
    samples = []
    for _ in range(args.reps):
        dbg.zero_()
        g.replay_stream(args.steps // 2)
        torch.cuda.synchronize()
        samples.append(analyse(dbg, nk))
        if args.conv1_waves:  # slot 0 = conv12_fwd: stamps 4-7 relative to stamp 1 (conv1 start)
            d = dbg.view(-1, 16).cpu()[:1024].double()
            d = d[d[:, 0] > 0]
            rel = {k: float(((d[:, k] - d[:, 1]) / 100.0).mean()) for k in (4, 5, 7, 2)}
            print("conv1 per-wave (us after conv1 start): wave0 3 tiles done %.2f, wave4 2 tiles %.2f, "
                  "last wave 2 tiles + 4x4x1 group %.2f, barrier %.2f"
                  % (rel[4], rel[7], rel[5], rel[2]), flush=True)
    # per-kernel medians over the samples
    rows = []
    per = nk // 2
    names = NAMES
    for k in range(nk):
        vals = {key: sorted(s[k][key] - s[0]["start"] for s in samples) for key in ("start", "end", "p50end")}
        med = {key: v[len(v) // 2] / 100.0 for key, v in vals.items()}
        gaps = sorted((s[k]["start"] - s[k - 1]["end"]) / 100.0 for s in samples) if k else [float("nan")]
        rows.append({"kernel": names[k % per] if per == len(names) else f"k{k}", "step": k // per,
                     "blocks": samples[0][k]["blocks"], "start_us": round(med["start"], 2),
                     "span_us": round(med["end"] - med["start"], 2),
                     "p50_block_end_us": round(med["p50end"] - med["start"], 2),
                     "gap_from_prev_us": round(gaps[len(gaps) // 2], 2),
                     "phase_means_us": [round(sum(x["phases"][j] for x in (s_[k] for s_ in samples)) / len(samples), 2)
                                        for j in range(len(samples[0][k]["phases"]))],
                     "phase_ghz": [round(sum(x["ghz"][j] for x in (s_[k] for s_ in samples)) / len(samples), 2)
                                   for j in range(len(samples[0][k]["ghz"]))]})
    for r, k in zip(rows, range(nk)):
        if r["kernel"] in GROUPS:
            r["jobs"] = {}
            for lo, hi, job in GROUPS[r["kernel"]]:
                ends = sorted(max((e for b, e in s[k]["block_end"].items() if lo <= b < hi), default=0.0)
                              - s[k]["start"] for s in samples)
                r["jobs"][job] = round(ends[len(ends) // 2] / 100.0, 2)
    period = sorted((s[per]["start"] - s[0]["start"]) / 100.0 for s in samples)
    res = {"step_period_us": round(period[len(period) // 2], 2), "kernels": rows,
           "sum_span_us": round(sum(r["span_us"] for r in rows[per:]), 2),
           "sum_gap_us": round(sum(r["gap_from_prev_us"] for r in rows[1:per + 1]), 2)}
    print(f"step period (kernel 0 of step t -> kernel 0 of step t+1): {res['step_period_us']} us")
    print(f"{'kernel':12s} {'step':>4s} {'blocks':>6s} {'start':>8s} {'span':>7s} {'p50end':>7s} {'gap':>6s}")
    for r in rows:
        print(f"{r['kernel']:12s} {r['step']:4d} {r['blocks']:6d} {r['start_us']:8.2f} {r['span_us']:7.2f} "
              f"{r['p50_block_end_us']:7.2f} {r['gap_from_prev_us']:6.2f}" +
              ("   last block end by job: " + ", ".join(f"{j} {v}" for j, v in r["jobs"].items())
               if r.get("jobs") else ""))
    print(f"one step: sum of spans {res['sum_span_us']} us + sum of gaps {res['sum_gap_us']} us")
    print("mean block phase times (us, stamp k -> k+1): " +
          "; ".join(f"{r['kernel']} {r['phase_means_us']}" for r in rows[per:]))
    aux = [(r["kernel"], round(sum(s_[k]["aux71"] for s_ in samples) / len(samples), 2))
           for r, k in zip(rows[per:], range(per, nk)) if samples[0][k]["aux71"] is not None]
    if aux:
        print("second-group stamp 7 (us after stamp 1; conv_bwd4: 2b done): " +
              "; ".join(f"{n} {v}" for n, v in aux))
    print("effective shader clock per phase (GHz, clock64 / wall_clock64): " +
          "; ".join(f"{r['kernel']} {r['phase_ghz']}" for r in rows[per:]))
    for spec in args.by_mod:
        kname, mod = spec.split(":")
        res.setdefault("by_mod", {})[spec] = by_mod(samples, names, per, kname, int(mod))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


def by_mod(samples, names, per, kname, mod):
    """Mean start / phase times / end of the blocks of KERNEL (second step) grouped by block id % mod,
    over every sample, and the ten latest-ending blocks of the last sample."""
    k = per + names.index(kname)
    acc = {}
    for s in samples:
        br = s[k]["block_rows"]
        t0 = s[k]["start"]
        for row, blk in enumerate(br["idx"].tolist()):
            w, v = br["w"][row], br["valid"][row]
            stamps = [float(w[j]) for j in range(8) if v[j]]
            a = acc.setdefault(blk % mod, {"n": 0, "start": 0.0, "end": 0.0, "ph": [0.0] * 7, "phn": [0] * 7})
            a["n"] += 1
            a["start"] += (float(w[0]) - t0) / 100.0
            a["end"] += (max(stamps) - t0) / 100.0
            for j in range(6):
                if v[j] and v[j + 1]:
                    a["ph"][j] += float(w[j + 1] - w[j]) / 100.0
                    a["phn"][j] += 1
    out = {}
    print(f"{kname} blocks by id % {mod}: start / phases / end (us after the kernel's first stamp)")
    for g in sorted(acc):
        a = acc[g]
        ph = [round(a["ph"][j] / a["phn"][j], 2) for j in range(6) if a["phn"][j]]
        out[g] = {"blocks": a["n"] // len(samples), "start": round(a["start"] / a["n"], 2), "phases": ph,
                  "end": round(a["end"] / a["n"], 2)}
        print(f"  {g}: {out[g]}")
    s = samples[-1]
    ends = sorted(((e - s[k]["start"]) / 100.0, b) for b, e in s[k]["block_end"].items())[-10:]
    print("  latest blocks (end us, block id): " + ", ".join(f"{e:.2f} #{b}" for e, b in ends))
    return out


if __name__ == "__main__":
    main()
