#!/usr/bin/env python3
"""Which attention variants are bit-identical to the plain 4-wave kernels (pruning probe, round 5)."""
import json
import math
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from pytorch_operator_amd.ops import _native  # noqa: E402
from pytorch_operator_amd.ops.attention import flash_attention  # noqa: E402

lib = _native.load()
res = {}
for shape in ((2, 512, 8, 2), (1, 384, 4, 4), (3, 128, 2, 1)):
    for causal in (True, False):
        g = torch.Generator(device="cuda").manual_seed(1)
        q, k, v = (torch.randn(shape[0], shape[1], h, 128, device="cuda", generator=g).to(torch.bfloat16)
                   for h in (shape[2], shape[3], shape[3]))
        do = torch.randn(q.shape, device="cuda", generator=g).to(torch.bfloat16)
        outs = {}
        for tag, fv, dqv, dkv in (("plain", 4, 8, 1), ("v4", 4, 8, 4), ("default", 10, 9, 8), ("fwd8", 8, 8, 4)):
            lib.pto_attn_set_variant(fv)
            lib.pto_attn_set_dq_variant(dqv)
            lib.pto_attn_set_dkdv_variant(dkv)
            xs = [x.detach().clone().requires_grad_(True) for x in (q, k, v)]
            o = flash_attention(*xs, causal)
            o.backward(do)
            outs[tag] = [o.detach()] + [x.grad for x in xs]
        key = f"{shape}_{causal}"
        res[key] = {f"{a}_vs_{b}": [bool(torch.equal(x, y)) for x, y in zip(outs[a], outs[b])]
                    for a, b in (("default", "plain"), ("default", "v4"), ("v4", "plain"), ("default", "fwd8"))}
print(json.dumps(res, indent=1))
