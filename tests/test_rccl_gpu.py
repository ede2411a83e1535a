"""The RCCL gradient-path step forms under a real RCCL communicator on one GPU.

``FlatGradAllReduce(force=True)`` on a single-rank ``nccl`` process group issues both bucket
all-reduces every step.  ``tools/rccl_w1_check.py`` runs the stream-launched split step, the
one-graph ``graph-comm`` step and eager steps under it, and the start-up race without an xGMI
candidate; at world 1 every form must be bit-identical to the step without collectives.
bench.py's ``--force-collectives`` line and its operator-deployed job carry the race record.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _env():
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.timeout(300)
def test_rccl_forms_bit_identical_at_world1(tmp_path):
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "rccl_w1_check.py"), "--out", str(tmp_path)],
                       capture_output=True, text=True, timeout=280, cwd=ROOT, env=_env())
    f = tmp_path / "rank0.json"
    assert f.exists(), r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(f.read_text())
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / "rccl_w1_check.json").write_text(json.dumps(res, indent=1))
    assert res["rccl_exec"]["split"] and res["rccl_exec"]["launch"] == "stream", res
    assert not res["rccl_graph_exec"]["split"], res
    assert all(v == res["steps"] >= 10 for v in res["cursors"].values()), res
    assert all(v > 0 for v in res["issued"].values()), res
    for k in ("eager", "rccl", "rccl_graph"):
        assert res[f"{k}_vs_split_equal"], (k, res)
    # the default (fused) DDP form is the single-GPU five-launch step's kernels: bit-identical to it;
    # the round-5 form (head launch + fc1_bwd) to the six-kernel step
    assert res["ddp_form"] == "fused" and res["split_vs_fused_equal"], res
    assert res["split_r5_vs_six_equal"], res
    assert res["fused_head_max_rel_diff_vs_six"] < 1e-5, res
    race = res["race"]
    assert race["rccl_ms_per_step"] > 0 and race["rccl_graph_ms_per_step"] > 0, race
    assert race["xgmi_ms_per_step"] is None and "world 1" in race["xgmi_skipped"], race
    assert race["picked"] in ("rccl", "rccl-graph", "rccl-r5") and race["six_kernel_ms_per_step"] > 0, race
    assert race["rccl_r5_ms_per_step"] > 0, race  # the round-5 form raced beside the fused one
    assert r.returncode == 0 and res["all_ok"], res


@pytest.mark.timeout(400)
def test_bench_forced_collectives_world1_through_operator(tmp_path):
    """``bench.py --force-collectives 1 --backend nccl`` at world 1: the race record in the line
    and in the operator-deployed pod's events."""
    out = tmp_path / "bench.json"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--backend", "nccl", "--force-collectives", "1",
           "--steps", "20", "--warmup", "5", "--job-timeout", "200", "--json-out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, cwd=ROOT, env=_env())
    assert r.returncode == 0 and out.exists(), r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads(out.read_text())
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / "bench_w1_forced_rccl.json").write_text(json.dumps(line))
    cfg = line["config"]
    assert line["n_gpus"] == 1 and cfg["forced_collectives"] is True and cfg["backend"] == "rccl", line
    trial = cfg["allreduce_trial"]
    assert trial["rccl_ms_per_step"] > 0 and trial["rccl_graph_ms_per_step"] > 0, trial
    assert trial["xgmi_ms_per_step"] is None, trial
    assert cfg["grad_allreduce"] == trial["picked"], line
    job = line["job"]
    assert job.get("result") == "Succeeded" and job["backend"] == "rccl", job
    jt = job["allreduce_trial"]
    assert jt is not None and jt["rccl_ms_per_step"] > 0 and jt["rccl_graph_ms_per_step"] > 0, job


@pytest.mark.timeout(300)
def test_rccl_tune_candidates_run_under_rccl(tmp_path):
    """tools/rccl_tune.py: every RCCL env candidate initialises a real RCCL communicator and
    all-reduces the two gradient buckets correctly (one rank: the protocol choice itself needs
    >= 2 GPUs, see the tool's docstring)."""
    out = tmp_path / "tune.json"
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "rccl_tune.py"), "--nproc", "1", "--candidates",
                        "default,proto-LL,proto-Simple,algo-Ring", "--iters", "50", "--reps", "3",
                        "--timeout", "120", "--out", str(out)],
                       capture_output=True, text=True, timeout=290, cwd=ROOT, env=_env())
    assert out.exists(), r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / "rccl_tune_w1.json").write_text(json.dumps(res, indent=1))
    assert r.returncode == 0, r.stderr[-3000:]
    for c in res["candidates"]:
        assert "error" not in c, c
        assert c["correct"] and c["backend"] == "nccl" and c["device"] == "cuda" and c["step_us"] > 0
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in res["winner"]["operator_flags"]
