#!/usr/bin/env python3
"""LDS bank-conflict model of conv12_fwd_kernel, fc1_bwd_head_kernel and conv_bwd4_kernel (round 6).

Banking rules (MI355X_MICROARCH.md §LDS): a wave64 LDS instruction is serviced in fixed lane
groups, one cycle per group when conflict-free; within a group each bank serves one distinct dword
per cycle (identical addresses broadcast), so a group costs max over banks of the distinct dwords
on it.  ``SQ_LDS_BANK_CONFLICT`` counts the cycles above one per group -- printed here per access
of the kernels' source, per wave, for the strides given on the command line:

    python tools/lds_banks_fwd.py [--h-rs 514] [--h-ds 516] [--irs 44] ...

(ds_read2_b32 / ds_write2_* are two accesses of the single-width form, as the hardware runs them.)
"""
from __future__ import annotations

import argparse
from collections import defaultdict

GROUPS = {
    "r32": ([list(range(0, 32)), list(range(32, 64))], 32, 1),
    "r64": ([list(range(0, 32)), list(range(32, 64))], 64, 2),
    "r128": ([[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32)),
              [32, 33, 34, 35, 44, 45, 46, 47] + list(range(52, 60)), list(range(36, 44)) + [48, 49, 50, 51] + list(range(60, 64))],
             64, 4),
    "w32": ([list(range(0, 32)), list(range(32, 64))], 32, 1),
    "w64": ([list(range(k, k + 16)) for k in range(0, 64, 16)], 32, 2),
    "w128": ([list(range(k, k + 8)) for k in range(0, 64, 8)], 32, 4),
}


def extra_cycles(kind: str, addr) -> int:
    """Conflict cycles of one wave-instruction: ``addr[lane]`` = first dword (None = inactive)."""
    groups, mod, width = GROUPS[kind]
    extra = 0
    for grp in groups:
        banks = defaultdict(set)
        for ln in grp:
            a = addr[ln]
            if a is None:
                continue
            for d in range(width):
                banks[(a + d) % mod].add(a + d)
        if banks:
            extra += max(len(v) for v in banks.values()) - 1
    return extra


class Tally:
    def __init__(self):
        self.rows = defaultdict(lambda: [0, 0])  # name -> [extra cycles, instructions]

    def add(self, name, kind, addr):
        r = self.rows[name]
        r[0] += extra_cycles(kind, addr)
        r[1] += 1

    def report(self, title, waves):
        print(f"== {title}: conflict cycles per wave (instructions per wave)")
        tot = 0
        for name, (c, n) in sorted(self.rows.items(), key=lambda kv: -kv[1][0]):
            tot += c
            print(f"  {name:34s} {c / waves:7.2f}  ({n / waves:.1f})")
        print(f"  {'total':34s} {tot / waves:7.2f}")
        return tot / waves


def fc1_bwd_head(a) -> float:
    H, HD, NT = a.h_rs, a.h_ds, 512
    r6 = a.layout == "r6"
    # round 6: hs / w2s rows 16-B aligned (H_RS 516) with columns XOR 2 in rows 8-15 (both the
    # logits reads and the ReLU-mask reads conflict-free), float4 stores; dhs plain (--dhs-xor 1:
    # H_DS 520 with the 16-byte chunk index XOR the row -- dz2 reads conflict-free, +VALU, slower)
    hx = (lambda row, col: row * H + (col ^ (2 * (row >> 3)))) if r6 else (lambda row, col: row * H + col)
    dx = (lambda row, col: row * HD + (col ^ (row << 2))) if a.dhs_xor else (lambda row, col: row * HD + col)
    # staging passes: r6 takes rows 0-7 in passes 0-1 and rows 8-15 in passes 2-3 (stage_e)
    se = (lambda q, x: x + q * NT if q < 2 else 1000 + x + (q - 2) * NT) if r6 else (lambda q, x: x + q * NT)
    # --kchunk 1: lane group x of wave wv owns K chunk 4 (x + 4 (wv >> 2)) + (wv & 3) (a wave's chunks 64
    # columns apart: dz2 reads conflict-free; measured slower, not used)
    kc = (lambda wv, x: 4 * (x + 4 * (wv >> 2)) + (wv & 3)) if a.kchunk else (lambda wv, x: 4 * wv + x)
    t = Tally()
    for wv in range(8):
        L = range(64)
        tid = [64 * wv + l for l in L]
        for base, rows, nq in ((0, 2000, 4), (16, 1250, 3)):  # hs (16 rows), w2s (10 rows)
            for q in range(nq):
                ents = [se(q, x) for x in tid]
                lim = min(rows, 1000) if (r6 and q < 2) else rows
                if r6:
                    t.add("hs/w2s stores", "w128", [hx(base + e // 125, 4 * (e % 125)) if e < lim else None
                                                    for e in ents])
                else:
                    for half in (0, 2):
                        t.add("hs/w2s stores", "w64", [hx(base + e // 125, 4 * (e % 125)) + half if e < rows else None
                                                       for e in ents])
        for s in range(16):  # logits operands
            t.add("logits hs reads", "r32", [hx(l & 15, 64 * wv + 4 * s + (l >> 4)) for l in L])
            t.add("logits w2s reads", "r32", [hx(16 + (l & 15), 64 * wv + 4 * s + (l >> 4)) for l in L])
        if wv < 4:  # softmax: d(logits) into dls[16][DLS]
            t.add("dls store", "w32", [(4 * wv + (l >> 4)) * a.dls + (l & 15) for l in L])
        for c in range(10):
            t.add("dh: dls reads", "r32", [(4 * (l >> 4) + (l & 3)) * a.dls + c for l in L])
            for tt in range(4):
                t.add("dh: W2 reads (w2s)", "r32", [hx(16 + c, 16 * kc(wv, tt) + (l & 15)) for l in L])
        for tt in range(4):
            for r in range(4):
                t.add("dh: ReLU mask reads (hs)", "r32", [hx(4 * (l >> 4) + r, 16 * kc(wv, tt) + (l & 15)) for l in L])
                t.add("dhs stores", "w32", [dx(4 * (l >> 4) + r, 16 * kc(wv, tt) + (l & 15)) for l in L])
        for q in range(4):
            t.add("dz2: dhs b128 reads", "r128", [dx(l & 15, 16 * kc(wv, l >> 4) + 4 * q) for l in L])
    return t.report(f"fc1_bwd_head ({a.layout}: H_RS {H}, H_DS {HD}, DLS {a.dls})", 8)


def conv12_fwd(a) -> float:
    IRS, CS, RS, WS = a.irs, a.c2_cs, a.c2_rs, a.c2_ws
    r6 = a.layout == "r6"
    # round 6: w1s rows 26 floats apart (was 25); channel c of in_s at c * C2_CS + 2 (c >> 2) (the
    # conv1 epilogue's 16 channels x 2 columns on 32 banks; conv2's channel pairs keep their
    # 8-bank split); the w2-slice float2 stores of lanes 8-15 of each 16 take the upper pair first;
    # the channel 16-19 group's 16 positions per half-wave are 4 pooled rows x 2 columns
    W1R = 26 if r6 else 25
    cb = (lambda c: c * CS + 2 * (c >> 2)) if r6 else (lambda c: c * CS)
    t = Tally()
    NT = 1024
    for wv in range(16):
        L = range(64)
        tid = [64 * wv + l for l in L]
        t.add("img store", "w32", [(x // 28) * IRS + x % 28 if x < 784 else None for x in tid])
        t.add("w1s store", "w32", [(x // 25) * W1R + x % 25 if x < 500 else None for x in tid])
        for k in range(2):
            for first in (True, False):
                ad = []
                for x in tid:
                    e = x + k * NT
                    half = (2 if ((x >> 3) & 1) else 0) if r6 else 0
                    half = half if first else 2 - half
                    ad.append((e // 125) * WS + 4 * (e % 125) + half if e < 2000 else None)
                t.add("w2 slice stores (b64)", "w64", ad)
        # conv1 weight fragments
        for s_ in range(7):
            t.add("conv1 weight reads (w1s)", "r32", [(l & 15) * W1R + min(4 * s_ + (l >> 4), 24) for l in L])

        def toff(tap):
            return (tap // 5) * IRS + tap % 5

        def tile_reads(t0):
            py, pq = t0 // 3, t0 % 3
            for s_ in range(7):
                ad = []
                for l in L:
                    i, g = l & 15, l >> 4
                    wi, e = i >> 2, i & 3
                    ad.append((2 * py + (e >> 1)) * IRS + 8 * pq + 2 * wi + (e & 1) + toff(min(4 * s_ + g, 24)))
                t.add("conv1 MFMA operand reads (img)", "r32", ad)

        def tile_epi(t0):
            py = t0 // 3
            t.add("conv1 epilogue in_s store", "w32", [cb(l & 15) + py * RS + 4 * (t0 % 3) + (l >> 4) for l in L])

        tiles = [wv, wv + 16] + ([wv + 32] if wv < 4 else [])
        for t0 in tiles:
            tile_reads(t0)
            tile_epi(t0)
        if wv >= 7:
            G = wv - 7

            def pos(l):
                if not r6:
                    p4 = 16 * G + (l >> 2)
                    return p4 // 12, p4 % 12
                b = 2 * G + (l >> 5)
                p = (l >> 2) & 7
                return 4 * (b // 6) + (p >> 1), 2 * (b % 6) + (p & 1)
            for k in range(25):
                ad = []
                for l in L:
                    q = l & 3
                    ph4, pw4 = pos(l)
                    ad.append((2 * ph4 + (q >> 1)) * IRS + 2 * pw4 + (q & 1) + (k // 5) * IRS + k % 5)
                t.add("conv1 group 16-19 reads (img)", "r32", ad)
                t.add("conv1 group 16-19 weight reads", "r32", [(16 + (l & 3)) * W1R + k for l in L])
            t.add("conv1 group epilogue in_s store", "w32",
                  [cb(16 + (l & 3)) + pos(l)[0] * RS + pos(l)[1] for l in L])
        # conv2 implicit GEMM
        pt, kq = wv & 3, wv >> 2
        rng = [(0, 6), (6, 13), (13, 19), (19, 25)][kq]
        for qq in range(*rng):
            cj, kh = qq // 5, qq % 5
            for kw in range(5):
                t.add("conv2 A reads (in_s)", "r32",
                      [cb(4 * cj + (l >> 4)) + (2 * pt + ((l & 15) >> 3) + kh) * RS + ((l & 15) & 7) + kw for l in L])
                t.add("conv2 B reads (w_s)", "r32", [(l & 15) * WS + (l >> 4) * 25 + cj * 100 + kh * 5 + kw for l in L])
        if wv >= 4:  # a1 publication from in_s
            for part in ((0, 2) if r6 else (0,)):
                ad = []
                for x in tid:
                    e = x - 256
                    if 0 <= e < 180:
                        c, rem = e // 36, e % 36
                        ad.append(cb(c) + (rem // 3) * RS + 4 * (rem % 3) + part)
                    else:
                        ad.append(None)
                if any(v is not None for v in ad):
                    t.add("a1 publication reads", "r64" if r6 else "r128", ad)
    return t.report(f"conv12_fwd ({a.layout}: AB_IRS {IRS}, C2_CS {CS}, C2_RS {RS}, C2_WS {WS}, w1s row {W1R})", 16)


def conv_bwd4(a) -> float:
    """conv_bwd4_kernel: every LDS access of one block per (cig, r), averaged over the 16 blocks of a
    4-sample chunk (idx1-dependent phase-4 reads: random pooling argmax)."""
    import random
    rnd = random.Random(7)
    DZS, DZR, WS, DC, A1R, A1C, XR, RED1 = a.g_dzs, 52, 144, 68, 13, 160, a.g_xr, 132
    DZN = DZR * DZS
    A1S = 2 * A1C
    OFF_W = 4 * DZN
    OFF_DCOL = OFF_W + 52 * WS
    OFF_A1 = OFF_DCOL + 128 * DC
    OFF_A1C = OFF_A1 + 4 * A1C + 12 * A1R
    OFF_X = OFF_A1C + 4 * A1S
    OFF_IDX = OFF_X + 28 * XR
    OFF_PK = OFF_IDX + 180
    OFF_PV = OFF_PK + 6 * 256
    OFF_DZ1 = OFF_W
    OFF_RED = OFF_W + 5 * 628
    t = Tally()
    nblk = 0
    for cig in range(4):
        for r in range(4):
            nblk += 1
            jbase = 32 * r - cig
            c0 = max(jbase, 0) // 25
            for wv in range(16):
                tids = [64 * wv + ln for ln in range(64)]
                # ---- phase 1 stores
                for u in range(8):
                    ad = []
                    for tid in tids:
                        if tid < 800:
                            sq, f4 = tid // 200, tid % 200
                            co, ph = f4 >> 2, f4 & 3
                            uu = u if not (a.g_swz and ph & 2) else (u + 4) % 8  # rows swapped for ph 2, 3
                            ad.append(sq * DZN + co * DZS + 16 * ph + (2 * uu if uu < 4 else 8 + 2 * (uu - 4)))
                        else:
                            ad.append(None)
                    if any(x is not None for x in ad):
                        t.add("1 dz2 un-pool float2 stores", "w64", ad)
                ad = [(tid >> 7) * DZN + (50 + ((tid >> 6) & 1)) * DZS + (tid & 63) if tid < 512 else None for tid in tids]
                if any(x is not None for x in ad):
                    t.add("1 dz2 zero rows", "w32", ad)
                t.add("1 w2 slice float4 stores", "w128", [OFF_W + (tid >> 5) * WS + 4 * (tid & 31) for tid in tids])
                ad = [OFF_W + ((tid + 1024) >> 5) * WS + 4 * (tid & 31) if tid < 640 else None for tid in tids]
                if any(x is not None for x in ad):
                    t.add("1 w2 slice float4 stores", "w128", ad)
                for k in range(4):
                    ad = []
                    for tid in tids:
                        e = tid - 736
                        if e >= 0:
                            sm, rem = e // 72, e % 72
                            c = rem // 36
                            p4 = rem - c * 36
                            y = p4 // 3
                            ad.append(OFF_A1C + sm * A1S + c * A1C + y * A1R + 4 * (p4 - 3 * y) + k)
                        else:
                            ad.append(None)
                    if any(x is not None for x in ad):
                        t.add("1 a1 chunk image stores", "w32", ad)
                    ad = []
                    for tid in tids:
                        e = tid - 640
                        if 0 <= e < 180:
                            c, p4 = e // 36, e % 36
                            y = p4 // 3
                            ad.append(OFF_A1 + c * A1C + y * A1R + 4 * (p4 - 3 * y) + k)
                        else:
                            ad.append(None)
                    if any(x is not None for x in ad):
                        t.add("1 own a1 stores", "w32", ad)
                    ad = []
                    for tid in tids:
                        e = tid - 800
                        ad.append(OFF_X + (e // 7) * XR + 4 * (e % 7) + k if 0 <= e < 196 else None)
                    if any(x is not None for x in ad):
                        t.add("1 xn stores", "w32", ad)
                lanes = range(64)
                if wv < 8:
                    # ---- 2a
                    pt, jt0 = wv & 3, (wv >> 2) * 4
                    for sstep in range(13):
                        t.add("2a dz2 operand reads", "r32",
                              [r * DZN + (lane >> 4) * DZS + pt * 16 + (lane & 15) + 4 * sstep * DZS for lane in lanes])
                        for tt in range(4):
                            t.add("2a W2 operand reads", "r32",
                                  [OFF_W + cig + (lane >> 4) * WS + jt0 * 16 + (lane & 15) + 4 * sstep * WS + 16 * tt
                                   for lane in lanes])
                    for tt in range(4):
                        for rr in range(4):
                            t.add("2a dcol stores", "w32",
                                  [OFF_DCOL + ((jt0 + tt) * 16 + (lane >> 4) * 4 + rr) * DC + pt * 16 + (lane & 15)
                                   for lane in lanes])
                    # ---- 3: col2im (items tid, tid + 512)
                    for base_it in (0, 512):
                        its = [tid + base_it for tid in tids]
                        for kh in range(5):
                            for kw in range(5):
                                ad = []
                                for it in its:
                                    if it >= 720:
                                        ad.append(None)
                                        continue
                                    c, p = it // 144, it % 144
                                    y, x = p // 12, p % 12
                                    ad.append(OFF_DCOL + c * 25 * DC + y * 8 + x + kh * (5 * DC - 8) + kw * (DC - 1))
                                if any(v is not None for v in ad):
                                    t.add("3 col2im dcol reads", "r32", ad)
                        ad = []
                        for it in its:
                            if it >= 720:
                                ad.append(None)
                                continue
                            c, p = it // 144, it % 144
                            ad.append(OFF_A1 + c * A1C + (p // 12) * A1R + p % 12)
                        if any(v is not None for v in ad):
                            t.add("3 ReLU-mask a1 reads", "r32", ad)
                    # ---- 4: pooled dW_conv1 items (tid < 300)
                    its = [tid if tid < 300 else None for tid in tids]
                    if any(v is not None for v in its):
                        pidx = {it: [rnd.randrange(4) for _ in range(12)] for it in its if it is not None}
                        for k in range(12):
                            t.add("4 pooled dz1 reads", "r32",
                                  [OFF_DZ1 + (it // 60) * 144 + ((it % 60) // 5) * 12 + k if it is not None else None
                                   for it in its])
                        for px in range(12):
                            for kw in range(5):
                                ad = []
                                for it in its:
                                    if it is None:
                                        ad.append(None)
                                        continue
                                    rem = it % 60
                                    py, kh = rem // 5, rem % 5
                                    pp = pidx[it][px]
                                    ad.append(OFF_X + (2 * py + (pp >> 1) + kh) * XR + 2 * px + (pp & 1) + kw)
                                t.add("4 xn window reads", "r32", ad)
                        for kw in range(5):
                            t.add("4 partial stores", "w32",
                                  [OFF_RED + ((it % 60) // 5) * RED1 + (it // 60) * 25 + (it % 5) * 5 + kw
                                   if it is not None else None for it in its])
                else:
                    # ---- 2b
                    w8 = wv - 8
                    calls = [(w8, 0), (w8, 1)] if w8 < 4 else [(4 + ((w8 - 4) >> 1), (w8 - 4) & 1)]
                    for tp, kh2 in calls:
                        ct, jt = tp >> 1, tp & 1
                        for u in range(32):
                            s_, uu = u >> 4, u & 15
                            ad_a, ad_b = [], []
                            for lane in lanes:
                                i, g = lane & 15, lane >> 4
                                jc = min(max(jbase + jt * 16 + i, 0), 124)
                                ci, tt = jc // 25, jc % 25
                                ad_a.append(OFF_A1C + 2 * kh2 * A1S + (ci - c0) * A1C + (tt // 5) * A1R + tt % 5 + g +
                                            s_ * A1S + (uu >> 1) * A1R + 4 * (uu & 1))
                                ad_b.append(2 * kh2 * DZN + (ct * 16 + i) * DZS + g + s_ * DZN + 4 * uu)
                            t.add("2b a1 im2col operand reads", "r32", ad_a)
                            t.add("2b dz2 operand reads", "r32", ad_b)
                    if w8 >= 4:
                        items = [64 * wv + ln - 768 for ln in lanes]
                        for pos in range(64):
                            ad = []
                            for item in items:
                                sm, jl = item >> 6, item & 31
                                jc = min(max(jbase + jl, 0), 124)
                                ci, tt = jc // 25, jc % 25
                                ad.append(OFF_A1C + sm * A1S + (ci - c0) * A1C + (tt // 5) * A1R + tt % 5 +
                                          (pos >> 3) * A1R + (pos & 7))
                            t.add("2b co 48/49 VALU a1 reads", "r32", ad)
    return t.report(f"conv_bwd4 (G_DZS {DZS}, G_XR {XR}, un-pool store swizzle {a.g_swz})", nblk * 16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="r6", choices=["r5", "r6"])
    ap.add_argument("--h-rs", type=int, default=None)
    ap.add_argument("--h-ds", type=int, default=None)
    ap.add_argument("--dls", type=int, default=17)
    ap.add_argument("--dhs-xor", type=int, default=0, help="1: dhs chunk ^ row (measured slower, not used)")
    ap.add_argument("--kchunk", type=int, default=0, help="1: a wave's K chunks 64 columns apart (measured slower)")
    ap.add_argument("--irs", type=int, default=44)
    ap.add_argument("--c2-cs", type=int, default=200)
    ap.add_argument("--c2-rs", type=int, default=16)
    ap.add_argument("--c2-ws", type=int, default=514)
    ap.add_argument("--g-dzs", type=int, default=82)
    ap.add_argument("--g-xr", type=int, default=29, help="conv_bwd4's xn row stride (round 6: 30)")
    ap.add_argument("--g-swz", type=int, default=0, help="1: conv_bwd4's un-pool float2 stores row-swapped for ph 2, 3")
    ap.add_argument("--only", default="", help="fc1_bwd_head / conv12_fwd / conv_bwd4: one kernel")
    a = ap.parse_args()
    a.h_rs = a.h_rs or (516 if a.layout == "r6" else 514)
    a.h_ds = a.h_ds or (520 if a.dhs_xor else 516)
    for name, fn in (("fc1_bwd_head", fc1_bwd_head), ("conv12_fwd", conv12_fwd), ("conv_bwd4", conv_bwd4)):
        if not a.only or a.only == name:
            fn(a)


if __name__ == "__main__":
    main()
