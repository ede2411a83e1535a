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

