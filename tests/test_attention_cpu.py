"""CPU side of the flash-attention op: the reference math (the GPU tests' oracle) against
PyTorch SDPA, the shape gate of the HIP path, and the Llama dispatch on CPU tensors."""
import torch

from pytorch_operator_amd.ops import attention as A


def test_reference_matches_sdpa_gqa_causal():
    torch.manual_seed(0)
    q = torch.randn(2, 64, 8, 32, dtype=torch.float64)
    k = torch.randn(2, 64, 2, 32, dtype=torch.float64)
    v = torch.randn(2, 64, 2, 32, dtype=torch.float64)
    for causal in (True, False):
        o, lse = A.attention_reference(q, k, v, causal, return_lse=True)
        ref = A.sdpa_bshd(q, k, v, causal)
        assert torch.allclose(o.double(), ref, atol=1e-5), causal
        assert lse.shape == (2, 8, 64)


def test_hip_gate_rejects_cpu_and_odd_shapes():
    q = torch.zeros(1, 128, 4, 128, dtype=torch.bfloat16)
    assert not A.hip_supported(q, q, q)  # CPU tensors never take the HIP path
    assert torch.equal(A.flash_attention(q, q[:, :, :2], q[:, :, :2]).float(),
                       A.attention_reference(q, q[:, :, :2], q[:, :, :2]).float())


def test_llama_mini_attention_dispatch_on_cpu():
    from pytorch_operator_amd.models.llama import CONFIGS, Llama
    torch.manual_seed(0)
    cfg = CONFIGS["llama-mini"]
    assert cfg.head_dim == A.HEAD_DIM
    m = Llama(cfg)
    tok = torch.randint(0, cfg.vocab_size, (1, 128))
    loss = m(tok, tok)
    loss.backward()
    assert torch.isfinite(loss) and m.layers[0].attention.wqkv.weight.grad is not None
