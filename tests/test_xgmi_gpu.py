"""xGMI peer-memory all-reduce + fused SGD (csrc/kernels/xgmi_allreduce.hip).

2 and 4 ranks on the box's GPU(s) run tools/xgmi_check.py: the kernel must agree with
torch.distributed.all_reduce, the fused-SGD DDP step must match the RCCL/gloo path, and
graph-captured steps must keep the replicas bit-identical.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_ranks(tmp_path, world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tools" / "xgmi_check.py"),
           "--backend", "gloo", "--out", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=str(ROOT)))
    results = [json.loads((tmp_path / f"rank{k}.json").read_text()) for k in range(world)
               if (tmp_path / f"rank{k}.json").exists()]
    assert r.returncode == 0 and len(results) == world, r.stdout[-3000:] + r.stderr[-3000:]
    for res in results:
        assert res["all_ok"], res
