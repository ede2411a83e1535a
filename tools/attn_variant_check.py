#!/usr/bin/env python3
"""Compare the rejected attention variants (csrc/kernels/experiments/attention_variants.hip) with
the default passes on a GPU.  Needs an experiment library that links them:

    tools/build_exp.sh ref ""
    PTO_HIP_LIB=$PWD/pytorch_operator_amd/_lib/exp/ref.so python tools/attn_variant_check.py

Prints one JSON object: per variant and shape, whether o / dq / dk / dv equal the default's bits.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops.attention import flash_attention
    lib = _native.load()
    lib.pto_attn_set_variant(9)
    if lib.pto_attn_set_variant(10) != 9:
        print("this library has no experiment variants (build one with tools/build_exp.sh)", file=sys.stderr)
        return 2
    setters = {"fwd": lib.pto_attn_set_variant, "dq": lib.pto_attn_set_dq_variant, "dkdv": lib.pto_attn_set_dkdv_variant}
    defaults = {"fwd": 10, "dq": 9, "dkdv": 8}
    cases = [("fwd", 9), ("dq", 8), ("dkdv", 2), ("dkdv", 3), ("dkdv", 4), ("dkdv", 6), ("dkdv", 7)]
    out = {}
    for shape in ((2, 512, 8, 2), (1, 384, 4, 4)):
        g = torch.Generator(device="cuda").manual_seed(11)
        q, k, v = (torch.randn(shape[0], shape[1], h, 128, device="cuda", generator=g).to(torch.bfloat16)
                   for h in (shape[2], shape[3], shape[3]))
        do = torch.randn(q.shape, device="cuda", generator=g).to(torch.bfloat16)

        def run():
            xs = [x.detach().clone().requires_grad_(True) for x in (q, k, v)]
            o = flash_attention(*xs, True)
            o.backward(do)
            return [o.detach()] + [x.grad for x in xs]
        for kind, d in defaults.items():
            setters[kind](d)
        ref = run()
        for kind, var in cases:
            setters[kind](var)
            got = run()
            setters[kind](defaults[kind])
            out[f"{kind}{var}_{shape}"] = [bool(torch.equal(a, b)) for a, b in zip(got, ref)]
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
