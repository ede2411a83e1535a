"""MasterAdamW (fp32 masters for bf16 matmul weights) vs torch.optim.AdamW -- CPU reference path.

The GPU kernel (csrc/kernels/adamw.hip) is checked against this same reference in
tests/test_llm_gpu.py::test_adamw_kernel_matches_reference.
"""
import torch
import torch.nn as nn

from pytorch_operator_amd.ops.optim import MasterAdamW, to_bf16_matmul_weights


def test_fp32_params_match_torch_adamw():
    torch.manual_seed(0)
    a = nn.Linear(17, 9)
    b = nn.Linear(17, 9)
    b.load_state_dict(a.state_dict())
    oa = MasterAdamW(a.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    ob = torch.optim.AdamW(b.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    for _ in range(5):
        x = torch.randn(4, 17)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).pow(2).sum().backward()
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-6)


def test_bf16_weights_track_fp32_master():
    torch.manual_seed(1)
    m = nn.Sequential(nn.Embedding(10, 8), nn.Linear(8, 8, bias=False))
    ref = nn.Sequential(nn.Embedding(10, 8), nn.Linear(8, 8, bias=False))
    ref.load_state_dict(m.state_dict())
    assert to_bf16_matmul_weights(m) == 64
    assert m[1].weight.dtype == torch.bfloat16 and m[0].weight.dtype == torch.float32
    opt = MasterAdamW(m.parameters(), lr=1e-2, weight_decay=0.0)
    oref = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    for _ in range(3):
        g = torch.randn(8, 8)
        m[1].weight.grad = g.bfloat16()
        ref[1].weight.grad = g.bfloat16().float()  # same (bf16-representable) gradient
        m[0].weight.grad = ref[0].weight.grad = None
        opt.step()
        oref.step()
    master = opt.state[m[1].weight]["master"]
    torch.testing.assert_close(master, ref[1].weight.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(m[1].weight.float(), master.bfloat16().float())
