"""Numerics of the HIP flash attention (csrc/kernels/attention.hip) against an fp32 PyTorch
reference of the same op (forward output, log-sum-exp, and the three input gradients), with
the library SDPA's own bf16 error as the yardstick."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # B, S, Hq, Hkv
    (2, 256, 8, 2),
    (1, 384, 4, 4),
    (1, 512, 8, 1),
]


def _inputs(B, S, Hq, Hkv, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    mk = lambda H: torch.randn(B, S, H, 128, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731
    return mk(Hq), mk(Hkv), mk(Hkv)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("shape", SHAPES)
def test_flash_forward_matches_fp32_reference(shape, causal):
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops.attention import attention_reference, sdpa_bshd
    B, S, Hq, Hkv = shape
    q, k, v = _inputs(*shape)
    ref, lse = attention_reference(q, k, v, causal, return_lse=True)
    ref32 = attention_reference(q.float(), k.float(), v.float(), causal)
    o = torch.empty_like(q)
    lse2 = torch.empty(B, Hq, S, device="cuda")
    _native.check(_native.load().pto_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                              lse2.data_ptr(), B, S, Hq, Hkv, 128, 1 / math.sqrt(128), int(causal),
                                              torch.cuda.current_stream().cuda_stream), "attn_fwd")
    torch.cuda.synchronize()
    err = _rel(o, ref32)
    lib = _rel(sdpa_bshd(q, k, v, causal), ref32)
    assert err < max(2.0 * lib, 4e-3), (err, lib)
    assert float((o.float() - ref32).abs().max()) < 3e-2
    # lse2 is log2 units of the scaled scores
    assert torch.allclose(lse2, lse * math.log2(math.e), atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("shape", SHAPES)
def test_flash_backward_matches_fp32_reference(shape, causal):
    from pytorch_operator_amd.ops.attention import attention_reference, flash_attention, sdpa_bshd
    q, k, v = _inputs(*shape, seed=1)
    g = torch.Generator(device="cuda").manual_seed(7)
    do = torch.randn(q.shape, device="cuda", generator=g).to(torch.bfloat16)

    def grads(fn, *xs):
        xs = [x.detach().clone().requires_grad_(True) for x in xs]
        out = fn(*xs)
        out.backward(do.to(out.dtype))
        return [out.detach()] + [x.grad for x in xs]

    ref = grads(lambda a, b, c: attention_reference(a, b, c, causal).float(), q.float(), k.float(), v.float())
    ours = grads(lambda a, b, c: flash_attention(a, b, c, causal), q, k, v)
    lib = grads(lambda a, b, c: sdpa_bshd(a, b, c, causal), q, k, v)
    for name, a, r, lb in zip(("o", "dq", "dk", "dv"), ours, ref, lib):
        e, el = _rel(a, r), _rel(lb, r)
        assert e < max(2.0 * el, 6e-3), (name, e, el)
        assert torch.isfinite(a.float()).all(), name


@pytest.fixture
def fwd_variant():
    """Select the forward kernel (8-wave default / 4-wave) for one test, then restore."""
    from pytorch_operator_amd.ops import _native
    lib = _native.load()
    old = lib.pto_attn_set_variant(0)  # 0: query only
    yield lambda v: lib.pto_attn_set_variant(v)
    lib.pto_attn_set_variant(old)


def _fwd(q, k, v, causal):
    from pytorch_operator_amd.ops import _native
    B, S, Hq, _ = q.shape
    o = torch.empty_like(q)
    lse2 = torch.empty(B, Hq, S, device="cuda")
    _native.check(_native.load().pto_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                              lse2.data_ptr(), B, S, Hq, k.shape[2], 128, 1 / math.sqrt(128),
                                              int(causal), torch.cuda.current_stream().cuda_stream), "attn_fwd")
    torch.cuda.synchronize()
    return o, lse2


@pytest.mark.parametrize("variant", [4, 10])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_forward_variants_with_growing_scores(fwd_variant, variant, causal):
    """Both forward kernels on scores whose row maximum keeps growing along the keys (large,
    ramped logits): the 8-wave kernel's deferred rescale must fire mid-row, more than once,
    and still give the fp32 reference's output and log-sum-exp."""
    from pytorch_operator_amd.ops.attention import attention_reference
    fwd_variant(variant)
    B, S, Hq, Hkv = 1, 1024, 4, 2
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn(B, S, Hq, 128, device="cuda", generator=g)
    k = torch.randn(B, S, Hkv, 128, device="cuda", generator=g)
    v = torch.randn(B, S, Hkv, 128, device="cuda", generator=g)
    # a shared direction whose weight grows with the key index: for every query the best key
    # moves right tile after tile, by more than the deferral threshold per 64-key tile
    d = torch.randn(128, device="cuda", generator=g)
    d = d / d.norm()
    q = q + 6.0 * d
    k = k + (torch.arange(S, device="cuda", dtype=torch.float32) / 64.0 * 3.0).view(1, S, 1, 1) * d
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    ref32, lse = attention_reference(q.float(), k.float(), v.float(), causal, return_lse=True)
    o, lse2 = _fwd(q, k, v, causal)
    assert torch.isfinite(o.float()).all()
    assert _rel(o, ref32) < 8e-3, _rel(o, ref32)
    assert torch.allclose(lse2, lse * math.log2(math.e), atol=5e-3, rtol=1e-4)


@pytest.mark.parametrize("shape", [(2, 512, 8, 2), (1, 768, 4, 4), (1, 256, 2, 1)])
def test_flash_forward_variants_agree(fwd_variant, shape):
    """The default 8-wave forward (LDS-DMA K/V staging, deferred rescale) vs the plain 4-wave
    forward on the same inputs: bf16 outputs within rounding, the same log-sum-exp."""
    q, k, v = _inputs(*shape, seed=5)
    outs = {}
    for var in (4, 10):
        fwd_variant(var)
        outs[var] = _fwd(q, k, v, True)
    assert _rel(outs[10][0], outs[4][0]) < 4e-3
    assert torch.allclose(outs[10][1], outs[4][1], atol=1e-3, rtol=1e-5)


@pytest.mark.parametrize("dkdv", [1, 8])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_backward_dkdv_variants(dkdv, causal):
    """The dK/dV passes -- plain 4-wave (the reference / fallback) and the default software-
    pipelined pass (1-5 query tiles per head cover its prologue / epilogue) -- with the pipelined
    dQ pass, against the fp32 reference gradients."""
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops.attention import attention_reference, flash_attention, sdpa_bshd
    lib = _native.load()
    old = lib.pto_attn_set_dkdv_variant(dkdv)
    try:
        for shape in ((1, 128, 2, 2), (2, 256, 8, 2), (1, 640, 4, 1), (1, 768, 4, 1), (1, 512, 8, 8)):
            q, k, v = _inputs(*shape, seed=9)
            g = torch.Generator(device="cuda").manual_seed(4)
            do = torch.randn(q.shape, device="cuda", generator=g).to(torch.bfloat16)

            def grads(fn, *xs):
                xs = [x.detach().clone().requires_grad_(True) for x in xs]
                out = fn(*xs)
                out.backward(do.to(out.dtype))
                return [x.grad for x in xs]

            ref = grads(lambda a, b, c: attention_reference(a, b, c, causal).float(), q.float(), k.float(),
                        v.float())
            ours = grads(lambda a, b, c: flash_attention(a, b, c, causal), q, k, v)
            lib_g = grads(lambda a, b, c: sdpa_bshd(a, b, c, causal), q, k, v)
            for name, a, r, lb in zip(("dq", "dk", "dv"), ours, ref, lib_g):
                e, el = _rel(a, r), _rel(lb, r)
                assert e < max(2.0 * el, 6e-3), (shape, name, e, el)
    finally:
        lib.pto_attn_set_dkdv_variant(old)


def test_flash_llama_block_matches_sdpa_path():
    """A D = 128 Llama config through the model's attention dispatch: HIP flash vs library SDPA."""
    from pytorch_operator_amd.models.llama import CONFIGS, Llama
    torch.manual_seed(0)
    m = Llama(CONFIGS["llama-mini"]).cuda()
    tok = torch.randint(0, CONFIGS["llama-mini"].vocab_size, (2, 256), device="cuda")
    out = {}
    for impl in ("hip", "sdpa"):
        for blk in m.layers:
            blk.attention.impl = impl
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):  # the worker's setting
            loss = m(tok, tok)
        loss.backward()
        out[impl] = (float(loss), m.layers[0].attention.wqkv.weight.grad.float().clone())
    assert abs(out["hip"][0] - out["sdpa"][0]) < 2e-2 * abs(out["sdpa"][0])
    assert _rel(out["hip"][1], out["sdpa"][1]) < 5e-2


def test_flash_rejects_unsupported_shape_on_gpu():
    from pytorch_operator_amd.ops.attention import flash_attention
    q = torch.zeros(1, 100, 2, 128, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        flash_attention(q, q, q)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("shape", [(2, 512, 8, 2), (1, 384, 4, 4), (3, 128, 2, 1)])
def test_pipelined_dq_pass_bit_identical(causal, shape):
    """The software-pipelined dQ pass (dQ variant 9, attention_bwd_pipe.hip) runs the plain dQ
    pass's per-element operations in its key order: dQ, and the delta it writes for the dK/dV
    pass, bit-identical to the 4-wave dQ pass (variant 4)."""
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops.attention import flash_attention
    lib = _native.load()
    q, k, v = _inputs(*shape, seed=23)
    g = torch.Generator(device="cuda").manual_seed(6)
    do = torch.randn(q.shape, device="cuda", generator=g).to(torch.bfloat16)
    outs = {}
    old = lib.pto_attn_set_dq_variant(9)
    try:
        for var in (4, 9):
            lib.pto_attn_set_dq_variant(var)
            xs = [x.detach().clone().requires_grad_(True) for x in (q, k, v)]
            flash_attention(*xs, causal).backward(do)
            outs[var] = [x.grad for x in xs]
    finally:
        lib.pto_attn_set_dq_variant(old)
    for a, b in zip(outs[4], outs[9]):
        assert torch.equal(a, b), shape


@pytest.mark.parametrize("causal", [True, False])
def test_pipelined_dkdv_pass_bit_identical(causal):
    """The default dK/dV pass (8: software-pipelined across query tiles, AGPR-pinned accumulators,
    its own translation unit) runs the plain 4-wave pass's per-element operation order: dK and dV
    bit-identical to variant 1.  (The rejected variants 2-7 live in csrc/kernels/experiments/:
    tools/attn_variant_check.py.)"""
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops.attention import flash_attention
    lib = _native.load()
    q, k, v = _inputs(2, 512, 8, 2, seed=21)
    g = torch.Generator(device="cuda").manual_seed(5)
    do = torch.randn(q.shape, device="cuda", generator=g).to(torch.bfloat16)
    outs = {}
    old = lib.pto_attn_set_dkdv_variant(1)
    try:
        for var in (1, 8):
            lib.pto_attn_set_dkdv_variant(var)
            xs = [x.detach().clone().requires_grad_(True) for x in (q, k, v)]
            flash_attention(*xs, causal).backward(do)
            outs[var] = [x.grad for x in xs]
    finally:
        lib.pto_attn_set_dkdv_variant(old)
    for a, b in zip(outs[1], outs[8]):
        assert torch.equal(a, b)


def test_default_library_has_no_rejected_attention_variants():
    """The default build links only the chosen passes and their plain references: asking for a
    rejected variant leaves the selection unchanged."""
    from pytorch_operator_amd.ops import _native
    lib = _native.load()
    for setter, dflt, bad in ((lib.pto_attn_set_variant, 10, (8, 9)), (lib.pto_attn_set_dq_variant, 9, (8,)),
                              (lib.pto_attn_set_dkdv_variant, 8, (2, 3, 4, 6, 7))):
        cur = setter(dflt)
        for v in bad:
            setter(v)
            assert setter(dflt) == dflt, (v, "accepted by the default library")
        setter(cur)
