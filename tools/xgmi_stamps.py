#!/usr/bin/env python3
"""Read the xGMI exchange's per-workgroup phase stamps of a rehearsal (``tools/xgmi_check.py
--stamps --out DIR`` writes DIR/rank<r>_stamps.json) and say, for every launch whose bounded wait
timed out, whether the sender workgroup it waited for had not started yet (starvation: it was
never given a CU before the deadline) or had raised its flag in time (a protocol / visibility
bug).

    python tools/xgmi_stamps.py DIR [--json out.json]

Stamps are wall_clock64 ticks (100 MHz), one clock for every process on the GPU, so the ranks'
records of one step line up.  Row layout: [block, step, start, flag1, flag2, end, err, missing]
(missing = q * nblk + j + 1 of the first sender flag still low at a phase-2 timeout).
"""
import argparse
import glob
import json
import os
import sys


def load(d):
    ranks = {}
    for f in sorted(glob.glob(os.path.join(d, "rank*_stamps.json"))):
        r = json.load(open(f))
        ranks[r["rank"]] = r
    return ranks


def analyse(ranks):
    if not ranks:
        return {"error": "no stamp files"}
    nblk = next(iter(ranks.values()))["nblk"]
    tmo = int(next(iter(ranks.values())).get("timeout_s", 5.0) * 1e8)
    by = {}  # (rank, step) -> {block: row}
    for r, rec in ranks.items():
        for row in rec["rows"]:
            by.setdefault((r, row[1]), {})[row[0]] = row
    steps = sorted({s for (_, s) in by})
    out = {"nblk": nblk, "ranks": sorted(ranks), "steps_recorded": steps, "failures": []}
    for s in steps:
        recs = {r: by.get((r, s), {}) for r in ranks}
        bad = [(r, b, row) for r, blocks in recs.items() for b, row in blocks.items() if row[6] or row[7]]
        if not bad:
            continue
        t0 = min(row[2] for blocks in recs.values() for row in blocks.values())
        us = lambda t: round((t - t0) / 100.0, 2) if t else None  # noqa: E731
        fail = {"step": s, "per_rank": {}, "waits": []}
        for r, blocks in recs.items():
            rows = list(blocks.values())
            col = lambda k: [row[k] for row in rows if row[k]]  # noqa: E731
            fail["per_rank"][r] = {
                "blocks_recorded": len(rows),
                "start_us": [us(min(col(2))), us(max(col(2)))] if col(2) else None,
                "flag1_us": [us(min(col(3))), us(max(col(3)))] if col(3) else None,
                "flag2_us": [us(min(col(4))), us(max(col(4)))] if col(4) else None,
                "end_us": [us(min(col(5))), us(max(col(5)))] if col(5) else None,
                "blocks_timed_out": sum(1 for row in rows if row[7]),
            }
        for r, b, row in bad:
            if not row[7]:
                continue
            q, j = divmod(row[7] - 1, nblk)
            deadline = row[2] + tmo
            sender = by.get((q, s), {}).get(j)
            w = {"waiter": [r, b], "waiter_start_us": us(row[2]), "deadline_us": us(deadline),
                 "missing_sender": [q, j]}
            if sender is None:
                w["sender_record"] = None
                w["reading"] = "sender workgroup left no record for this step (never ran it, or ran it degraded)"
            else:
                w["sender_start_us"], w["sender_flag1_us"] = us(sender[2]), us(sender[3])
                if sender[2] > deadline:
                    w["reading"] = "starvation: the sender workgroup started only after the waiter's deadline"
                elif sender[3] and sender[3] <= deadline:
                    w["reading"] = "protocol/visibility: the sender raised flag1 before the deadline, the waiter never saw it"
                else:
                    w["reading"] = "sender started in time but had not raised flag1 by the deadline"
            fail["waits"].append(w)
        fail["waits"] = fail["waits"][:16]
        out["failures"].append(fail)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("dir")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    res = analyse(load(a.dir))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1)[:6000])
    return 0


if __name__ == "__main__":
    sys.exit(main())
