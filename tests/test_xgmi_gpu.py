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


@pytest.mark.parametrize("world,nblk", [(2, 0), (4, 0), (2, 256)])
def test_xgmi_allreduce_ranks(tmp_path, world, nblk):
    """nblk=0 picks 128 workgroups per rank here (ranks share the box's GPU); nblk=256 runs the
    geometry a one-GPU-per-rank job uses, every stage including the autotune hand-over, with the
    step's kernels that fit beside a spinning exchange workgroup (tools/xgmi_check.py,
    tests/test_kernel_resources.py): the production kernels -- fused conv12 forward, conv_bwd4 --
    in the fused DDP form, behind the pre-exchange rank barrier where ranks crowd the CUs."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tools" / "xgmi_check.py"),
           "--backend", "gloo", "--out", str(tmp_path), "--nblk", str(nblk)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=str(ROOT)))
    results = [json.loads((tmp_path / f"rank{k}.json").read_text()) for k in range(world)
               if (tmp_path / f"rank{k}.json").exists()]
    assert r.returncode == 0 and len(results) == world, r.stdout[-3000:] + r.stderr[-3000:]
    for res in results:
        assert res["all_ok"], res
        assert res["nblk"] == nblk or (nblk == 0 and res["nblk"] in (128, 256)), res
        # which production kernels ran beside the spinning exchange (profiles/r6_xgmi_geometry.md)
        # every geometry runs the production step in the fused DDP form; crowded ones (every CU can
        # hold a spinning exchange) behind the pre-exchange rank barrier
        assert res["ddp_form"] == "fused" and res["fuse_conv12"] and res["conv_chunk"] == 4, res
        assert res["prebarrier"] == res["crowded"], res
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / f"xgmi_check_w{world}_nblk{nblk}.json").write_text(json.dumps(results))


def test_xgmi_exchange_stamps_record_every_launch(tmp_path):
    """The exchange's per-workgroup stamp ring (XgmiAllReduce.enable_stamps, the diagnostics behind
    profiles/r5_xgmi_handover.md): a passing 2-rank rehearsal records its launches on both ranks, in
    phase order, and tools/xgmi_stamps.py finds no timed-out wait."""
    import importlib.util
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tools" / "xgmi_check.py"),
           "--backend", "gloo", "--out", str(tmp_path), "--stamps"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=str(ROOT)))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    spec = importlib.util.spec_from_file_location("xgmi_stamps", ROOT / "tools" / "xgmi_stamps.py")
    xs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(xs)
    ranks = xs.load(str(tmp_path / "stamps_main"))
    assert sorted(ranks) == [0, 1]
    for rec in ranks.values():
        assert rec["error"] == 0 and len(rec["rows"]) >= rec["nblk"]
        for blk, step, t0, f1, f2, t1, err, missing in rec["rows"]:
            assert 0 < t0 <= f1 <= f2 <= t1 and err == 0 and missing == 0
    assert xs.analyse(ranks)["failures"] == []


def test_xgmi_stall_makes_every_rank_exit_retryable(tmp_path):
    """A rank that stalls past the exchange's bounded wait must not leave the job running
    rank-local: every rank's worker notices the kernel's error word at its next
    log interval and exits with the retryable code 138 (tf-operator train_util.go:18-53),
    which the operator's ExitCode/OnFailure policies restart from the checkpoint."""
    port = _port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, PYTHONPATH=str(ROOT), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   WORLD_SIZE="2", RANK=str(rank), LOCAL_RANK=str(rank),
                   PTO_FAULT_STALL="1:3:4")  # rank 1 sleeps 4 s before its 4th step block
        cmd = [sys.executable, "-u", "-m", "pytorch_operator_amd.harness.mnist", "--backend", "gloo",
               "--allreduce", "xgmi", "--xgmi-timeout", "0.5", "--dataset-size", "6400",
               "--test-size", "1000", "--log-interval", "10", "--dir", str(tmp_path / f"tb{rank}")]
        procs.append(subprocess.Popen(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    codes = [p.returncode for p in procs]
    assert codes == [138, 138], "\n----\n".join(o[-2500:] for o in outs)
    for o in outs:
        assert '"event": "xgmi_error"' in o and '"path": "xgmi"' in o


def test_physical_gpu_ignores_the_visible_device_list():
    """Ranks decide whether they share a GPU by its PCI ids, not by their cuda index: a process
    that sees the GPU through HIP_VISIBLE_DEVICES (an emulated pod's cuda:0) names the same GPU."""
    import torch

    from pytorch_operator_amd.parallel.xgmi import physical_gpu
    here = physical_gpu(torch.device("cuda", 0))
    assert here[0] == "pci", here
    code = ("import json, torch; from pytorch_operator_amd.parallel.xgmi import physical_gpu; "
            "print(json.dumps(physical_gpu(torch.device('cuda', 0))))")
    env = dict(os.environ, PYTHONPATH=str(ROOT), HIP_VISIBLE_DEVICES="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert tuple(json.loads(r.stdout.strip().splitlines()[-1])) == here
