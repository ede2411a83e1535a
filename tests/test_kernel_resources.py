"""Co-residency of the shared-GPU xGMI rehearsal (root cause in
profiles/r5_xgmi_handover.md).

When two ranks share one GPU at the one-GPU-per-rank geometry (256 exchange workgroups each,
tools/xgmi_check.py --nblk 256), a rank's exchange workgroups sit on every CU spinning on the
peer's flags while the peer still runs its step's kernels.  Each of those kernels must therefore
fit on a CU beside one exchange workgroup (one wave per SIMD): its waves per SIMD x their VGPR
allocation + the exchange wave's <= 512 VGPRs, and <= 8 waves per SIMD.  The fused conv12 forward
(4 waves x 104 VGPRs) does not -- its workgroups waited for the peer's exchange to time out, which
the exchange's stamps showed -- so the rehearsal runs the split conv1 / conv2 forward; this test
keeps the kernels it does run within the budget.  Reads the AMDGPU metadata of the built library
(tools/isa_dump.py), no GPU needed.

Round 6 (profiles/r6_xgmi_geometry.md): the fused DDP form's exchange (``xar_kernel_fc``, which
also computes the fc gradient tiles) allocates 152 VGPRs; the round-5 exchange kept its own
instantiation (``xar_kernel``, 112).  With four ranks on one GPU at 128 workgroups each, three
peers' exchanges put up to two exchange waves on a SIMD: the round-5 kernels fit beside two
``xar_kernel`` waves, the fused form's ``fc1_bwd_head`` does not fit beside two ``xar_kernel_fc``
waves -- so crowded rehearsals run the round-5 form (tools/xgmi_check.py ``ddp_form``).
"""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
LIB = ROOT / "pytorch_operator_amd" / "_lib" / "libpto_hip.so"

# the world > 1 step of tools/xgmi_check.py's shared-GPU 256 geometry (fuse_conv12 off,
# conv_chunk 1): conv1 / conv2 forward, split-K fc1, head, fc1 backward, per-sample conv backward
REHEARSAL = ["conv1_fwd_pool_kernel", "conv2_fwd_pool_kernel", "fc1_fwd_kernelILi2", "head_kernelILi1",
             "fc1_bwd_kernel", "conv_bwd_kernel"]


@pytest.fixture(scope="module")
def res():
    if not LIB.exists():
        pytest.skip("libpto_hip.so not built")
    import isa_dump
    return isa_dump, isa_dump.kernel_resources(LIB)


# the fused world > 1 step (round 6) at the same geometry: forward, fused head + fc1 backward,
# per-sample conv backward; the exchange computes the fc gradients itself
FUSED = ["conv1_fwd_pool_kernel", "conv2_fwd_pool_kernel", "fc1_fwd_kernelILi2", "fc1_bwd_head_kernel",
         "conv_bwd_kernel"]


def _find(r, sub):
    hits = [k for k in r if sub in k]
    assert len(hits) == 1, (sub, hits)
    return r[hits[0]]


def test_rehearsal_kernels_fit_beside_a_spinning_exchange_workgroup(res):
    isa, r = res
    xar = _find(r, "xar_kernelENS")
    x = isa.vgpr_alloc(xar)
    assert xar["max_wg"] == 256  # one wave per SIMD
    for sub in REHEARSAL:
        k = _find(r, sub)
        wps = -(-k["max_wg"] // 256)  # waves per SIMD of one workgroup
        assert wps * isa.vgpr_alloc(k) + x <= 512, (sub, k, xar)
        assert wps + 1 <= 8, sub
        assert k["spills"] == 0, sub



def _fits(isa, k, exchange_waves, x):
    wps = -(-k["max_wg"] // 256)
    return wps * isa.vgpr_alloc(k) + exchange_waves * x <= 512 and wps + exchange_waves <= 8


def test_fused_form_kernels_fit_beside_one_fc_exchange_workgroup(res):
    isa, r = res
    xfc = _find(r, "xar_kernel_fcENS")
    assert xfc["max_wg"] == 256 and xfc["spills"] == 0
    x = isa.vgpr_alloc(xfc)
    assert x <= 160, xfc  # keeps fc1_bwd_head (2 waves x 120) beside it
    for sub in FUSED:
        k = _find(r, sub)
        assert _fits(isa, k, 1, x), (sub, k, xfc)
        assert k["spills"] == 0, sub


def test_crowded_geometry_runs_the_round5_form(res):
    """W = 4 at 128 workgroups per rank: up to two peer exchange waves per SIMD."""
    isa, r = res
    x5 = isa.vgpr_alloc(_find(r, "xar_kernelENS"))
    xfc = isa.vgpr_alloc(_find(r, "xar_kernel_fcENS"))
    waves = -(-3 * 128 // 256)
    assert waves == 2
    for sub in REHEARSAL:
        assert _fits(isa, _find(r, sub), waves, x5), sub
    # the fused form would not: its head kernel cannot start beside two fc exchanges
    assert not _fits(isa, _find(r, "fc1_bwd_head_kernel"), waves, xfc)
