"""bench.py's launcher decision (CPU): ``python bench.py --gpus N`` with no rank environment
starts the N ranks itself as a child ``torch.distributed.run`` job; a world size that differs
from ``--gpus`` ends the run with exit code 2 before any GPU work.

The real N-rank bench on the GPU box is ``tests/test_bench_gpu.py::test_bench_self_launch``.
"""
import json
import os
import subprocess
import sys
import textwrap
from argparse import Namespace
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=str(ROOT), **kw)
    return env


def test_needs_self_launch_decision():
    assert bench.needs_self_launch(2, {}) is True
    assert bench.needs_self_launch(8, {"PATH": "/bin"}) is True
    assert bench.needs_self_launch(1, {}) is False          # the 1-GPU path is unchanged
    assert bench.needs_self_launch(8, {"WORLD_SIZE": "8"}) is False  # under torchrun / a pod
    assert bench.needs_self_launch(2, {"WORLD_SIZE": "1"}) is False  # mismatch: main() rejects it


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "4", "--steps", "20"], 4, 29511, script="/x/bench.py")
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "4", "--steps", "20"]


def test_check_line():
    ok = {"n_gpus": 4, "world_size": 4, "rccl_nranks": 4}
    assert bench.check_line(ok, 4) is None
    assert bench.check_line(dict(ok, rccl_nranks=None), 4) is None  # gloo: no RCCL communicator
    assert "n_gpus=1" in bench.check_line({"n_gpus": 1, "world_size": 1}, 4)
    assert "RCCL" in bench.check_line(dict(ok, rccl_nranks=1), 4)


@pytest.mark.timeout(120)
def test_world_size_mismatch_exits_2():
    """Launched with WORLD_SIZE=2 but --gpus 1 (or the reverse): exit 2, no line, no torch import."""
    for ws, gpus in (("2", "1"), ("1", "3")):
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", gpus],
                           capture_output=True, text=True, timeout=60, cwd=ROOT,
                           env=_env(WORLD_SIZE=ws, RANK="0", PTO_BENCH_LAUNCHER="test"))
        assert r.returncode == 2, (ws, gpus, r.stdout, r.stderr)
        assert "WORLD_SIZE" in r.stderr and '"metric"' not in r.stdout


@pytest.mark.timeout(300)
def test_rccl_more_ranks_than_gpus_exits_2():
    """--backend nccl asks for 2 ranks; this container has no GPU: refused before launching."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--backend", "nccl"],
                       capture_output=True, text=True, timeout=280, cwd=ROOT, env=_env())
    assert r.returncode == 2, (r.stdout, r.stderr)
    assert "one GPU per rank" in r.stderr and "launching" not in r.stderr


_FAKE = textwrap.dedent('''
    import json, os, sys
    world = int(os.environ["WORLD_SIZE"]); rank = int(os.environ["RANK"])
    gpus = int(sys.argv[sys.argv.index("--gpus") + 1])
    report = int(os.environ.get("FAKE_REPORT", world))
    if rank == 0:
        print("progress line")
        print(json.dumps({"metric": "m", "n_gpus": report, "world_size": report, "rccl_nranks": None,
                          "launcher": os.environ.get("PTO_BENCH_LAUNCHER")}), flush=True)
    sys.exit(int(os.environ.get("FAKE_RC", "0")))
''')


def _launch(tmp_path, capsys, **env):
    script = tmp_path / "fake_bench.py"
    script.write_text(_FAKE)
    old = dict(os.environ)
    os.environ.clear()
    os.environ.update(_env(**env))
    try:
        args = Namespace(gpus=2, backend="gloo")
        rc = bench.self_launch(args, ["--gpus", "2", "--backend", "gloo"], script=str(script))
    finally:
        os.environ.clear()
        os.environ.update(old)
    return rc, capsys.readouterr().out


@pytest.mark.timeout(200)
def test_self_launch_relays_rank0_line(tmp_path, capsys):
    """A real torch.distributed.run child job with 2 ranks: the parent relays rank 0's line
    (launcher recorded) and exits 0; a rank that exits non-zero or reports the wrong world
    makes the parent exit non-zero."""
    rc, out = _launch(tmp_path, capsys)
    assert rc == 0, out
    lines = [json.loads(x) for x in out.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1 and lines[0]["world_size"] == 2, out
    assert lines[0]["launcher"] == "bench.py->torch.distributed.run"
    rc, _ = _launch(tmp_path, capsys, FAKE_REPORT="1")
    assert rc == 2
    rc, _ = _launch(tmp_path, capsys, FAKE_RC="3")
    assert rc != 0
