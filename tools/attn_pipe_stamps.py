"""Per-wave timeline of the software-pipelined dK/dV pass (attention_bwd_pipe.hip) from its
diagnostic s_memtime stamps (tools/build_diag_attn.sh builds the library).

    PTO_HIP_LIB=pytorch_operator_amd/_lib/diag/attn_stamps.so python tools/attn_pipe_stamps.py

Reports the shader clock (s_memtime over s_memrealtime), per-wave cycles per tile in the loop,
the prologue and epilogue, and how the blocks' start times spread over the launch."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_operator_amd.ops import _native  # noqa: E402
from pytorch_operator_amd.ops.attention import flash_attention  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    lib = _native.load()
    lib.pto_attn_set_dkdv_variant(8)
    fn = lib.pto_attn_pipe_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(a.B, a.S, a.Hq, 128, device="cuda", generator=g).bfloat16().requires_grad_()
    k = torch.randn(a.B, a.S, a.Hkv, 128, device="cuda", generator=g).bfloat16().requires_grad_()
    v = torch.randn(a.B, a.S, a.Hkv, 128, device="cuda", generator=g).bfloat16().requires_grad_()
    do = torch.randn(q.shape, device="cuda", generator=g).bfloat16()
    for _ in range(5):
        flash_attention(q, k, v, True).backward(do)
    torch.cuda.synchronize()
    nblk = (a.S // 128) * a.B * a.Hkv
    n = min(nblk, 2048) * 4 * 16
    buf = np.zeros(n, dtype=np.uint64)
    assert fn(buf.ctypes.data, n) == 0
    st = buf.reshape(-1, 4, 16)[: min(nblk, 2048)].astype(np.float64)
    t0, t1, t2, t3, r0, r1, nt = (st[..., i] for i in range(7))
    clock_mhz = float(np.median((t3 - t0) / np.maximum(r1 - r0, 1) * 100.0))
    per_tile = (t2 - t1) / np.maximum(nt, 1)
    start_us = (r0 - r0.min()) / 100.0
    end_us = (r1 - r0.min()) / 100.0
    res = {
        "shape": vars(a), "blocks": int(nblk), "clock_mhz": round(clock_mhz, 1),
        "launch_span_us": round(float(end_us.max()), 1),
        "cycles_per_tile": {p: round(float(np.percentile(per_tile, p)), 1) for p in (10, 50, 90)},
        "cycles_per_tile_wave0_heaviest": round(float(per_tile[np.argmax(nt[:, 0]), 0]), 1),
        "prologue_cycles_p50": round(float(np.median(t1 - t0)), 1),
        "epilogue_cycles_p50": round(float(np.median(t3 - t2)), 1),
        "block_start_us": {p: round(float(np.percentile(start_us[:, 0], p)), 1) for p in (0, 25, 50, 75, 100)},
        "busy_us_sum_over_blocks": round(float(((r1 - r0)[:, 0]).sum() / 100.0), 1),
        "mfma_bound_cycles_per_tile": 32 * 32,
    }
    # tile 9 of every wave that has one: gaps 0-7 / 8-15 / 16-23 / 24-31, the closing wait
    # (vmcnt for the next-but-one tile's DMA) and the barrier
    ok = nt > 10
    ph = st[..., 8:14]
    names = ["gaps0_7", "gaps8_15", "gaps16_23", "gaps24_31+wait", "barrier"]
    d = [ph[..., i + 1] - ph[..., i] for i in range(4)] + [ph[..., 5] - ph[..., 4]]
    res["tile9_phase_cycles_p50"] = {nm: round(float(np.median(x[ok])), 1) for nm, x in zip(names, d)}
    res["tile9_phase_cycles_p90"] = {nm: round(float(np.percentile(x[ok], 90)), 1) for nm, x in zip(names, d)}
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
