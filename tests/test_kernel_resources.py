"""Co-residency of the shared-GPU xGMI rehearsal (root cause in
profiles/r5_xgmi_handover.md; round 6: profiles/r6_xgmi_geometry.md).

When ranks share one GPU at the one-GPU-per-rank geometry, a rank's exchange workgroups sit on
the CUs spinning on the peers' flags while a peer still runs its step's kernels.  Each of those
kernels must therefore fit on a CU beside the exchange waves the other ranks can put on a SIMD
(one per 256 exchange workgroups): its waves per SIMD x their VGPR allocation + the exchange
waves' <= 512 VGPRs, <= 8 waves per SIMD, and its LDS beside theirs <= 160 KB.

Round 5 found the fused conv12 forward (4 waves x 104 VGPRs) waiting out the peer's deadline
beside the 112-VGPR exchange.  Round 6: the exchange instantiation with one phase-2 batch per
thread (``xar_kernel``: every chunk at 256 workgroups, 53 float4s at world 8) allocates 96, so at
one exchange wave per SIMD (2 ranks x 256 workgroups) every production kernel of the round-5 DDP
form fits -- fused conv12, conv_bwd4 with its 152 KB of dynamic LDS -- and tools/xgmi_check.py
runs them there.  At two (4 ranks x 128) the split conv1 / conv2 forward and the per-sample conv
backward run.  The fused DDP form's exchange (``xar_kernel_fc``, which also computes the fc
gradient tiles) allocates more; its kernels fit beside one of its waves except conv12, so crowded
rehearsals run the round-5 form when the budget is all they rely on (``--prebarrier 0``).  The
budget is necessary, not sufficient: LDS / VGPR fragmentation around a spinning workgroup still
starved a peer now and then, so crowded rehearsals now run a one-wave rank barrier before each
exchange (profiles/r6_xgmi_geometry.md) and these rows document the static fit.  Reads the AMDGPU
metadata of the built library (tools/isa_dump.py) and one size query, no GPU needed.
"""
import ctypes
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
LIB = ROOT / "pytorch_operator_amd" / "_lib" / "libpto_hip.so"
LDS_CU = 160 * 1024

# the round-5 world > 1 step, production kernels: fused conv1+conv2 forward, split-K fc1, head,
# fc1 backward (pushing dW_fc1), 4-sample-chunk conv backward
PRODUCTION_R5 = ["conv12_fwd_kernel", "fc1_fwd_kernelILi2", "head_kernelILi1", "fc1_bwd_kernel",
                 "conv_bwd4_kernel"]
# the split step tools/xgmi_check.py runs at two exchange waves per SIMD
SPLIT_R5 = ["conv1_fwd_pool_kernel", "conv2_fwd_pool_kernel", "fc1_fwd_kernelILi2", "head_kernelILi1",
            "fc1_bwd_kernel", "conv_bwd_kernel"]
# the fused world > 1 step (round 6): forward, fused head + fc1 backward, conv backward; the
# exchange computes the fc gradients itself
FUSED = ["fc1_fwd_kernelILi2", "fc1_bwd_head_kernel", "conv_bwd4_kernel", "conv_bwd_kernel",
         "conv1_fwd_pool_kernel", "conv2_fwd_pool_kernel"]


@pytest.fixture(scope="module")
def res():
    if not LIB.exists():
        pytest.skip("libpto_hip.so not built")
    import isa_dump
    r = isa_dump.kernel_resources(LIB)
    dyn = {"conv_bwd4_kernel": ctypes.CDLL(str(LIB)).pto_mnist_conv_bwd4_lds()}
    return isa_dump, r, dyn


def _find(r, sub):
    hits = [k for k in r if sub in k]
    assert len(hits) == 1, (sub, hits)
    return r[hits[0]]


def _fits(isa, r, dyn, sub, xname, exchange_waves):
    k, x = _find(r, sub), _find(r, xname)
    wps = -(-k["max_wg"] // 256)  # waves per SIMD of one workgroup
    lds = k["lds"] + dyn.get(sub, 0)
    return (wps * isa.vgpr_alloc(k) + exchange_waves * isa.vgpr_alloc(x) <= 512
            and wps + exchange_waves <= 8 and lds + exchange_waves * x["lds"] <= LDS_CU)


def test_exchange_instantiations(res):
    isa, r, _ = res
    for name in ("xar_kernelENS", "xar_kernel_p2ENS", "xar_kernel_fcENS", "xar_kernel_fc_p2ENS"):
        x = _find(r, name)
        assert x["max_wg"] == 256 and x["spills"] == 0, (name, x)  # one wave per SIMD
    assert isa.vgpr_alloc(_find(r, "xar_kernelENS")) <= 96
    assert isa.vgpr_alloc(_find(r, "xar_kernel_fcENS")) <= 160


def test_production_kernels_fit_beside_one_exchange_wave(res):
    isa, r, dyn = res
    assert dyn["conv_bwd4_kernel"] > 100 * 1024  # the 152 KB plan
    for sub in PRODUCTION_R5:
        assert _fits(isa, r, dyn, sub, "xar_kernelENS", 1), (sub, _find(r, sub))
        assert _find(r, sub)["spills"] == 0, sub


def test_split_kernels_fit_beside_two_exchange_waves(res):
    """W = 4 at 128 workgroups per rank: three peers' exchanges, up to two waves per SIMD."""
    isa, r, dyn = res
    assert -(-3 * 128 // 256) == 2
    for sub in SPLIT_R5:
        assert _fits(isa, r, dyn, sub, "xar_kernelENS", 2), sub
        assert _fits(isa, r, dyn, sub, "xar_kernel_p2ENS", 2), sub  # chunks of 422 float4s at 128
    # the fused conv12 forward does not: why that geometry runs the split forward
    assert not _fits(isa, r, dyn, "conv12_fwd_kernel", "xar_kernelENS", 2)


def test_fused_form_beside_its_exchange(res):
    isa, r, dyn = res
    for sub in FUSED:
        assert _fits(isa, r, dyn, sub, "xar_kernel_fcENS", 1), sub
    # conv12 (4 x 104) does not fit beside the fc exchange: crowded rehearsals run the round-5 form
    assert not _fits(isa, r, dyn, "conv12_fwd_kernel", "xar_kernel_fcENS", 1)
    # nor fc1_bwd_head (2 x 120) beside two of them (W = 4 x 128)
    assert not _fits(isa, r, dyn, "fc1_bwd_head_kernel", "xar_kernel_fcENS", 2)


def test_prebarrier_kernel_holds_next_to_nothing(res):
    """The pre-exchange rank barrier spins beside a peer's step kernels: one wave, no LDS (any LDS
    allocation can split a CU's 160 KB below conv_bwd4's 152 KB range), a few VGPRs."""
    isa, r, _ = res
    k = _find(r, "xar_prebarrier_kernel")
    assert k["lds"] == 0 and k["max_wg"] == 64 and isa.vgpr_alloc(k) <= 16 and k["spills"] == 0, k
