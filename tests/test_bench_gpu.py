"""bench.py at world 2 on the box's one GPU: the driver's multi-GPU command shape
(``torch.distributed.run --nproc-per-node 2 bench.py --gpus 2 ...``), with gloo as the
process-group backend (RCCL wants one GPU per rank) and both ranks sharing cuda:0.

Checks the JSON line's DDP invariants (n_gpus, replicas_in_sync, grad_allreduce_error)
and the PyTorchJob it runs after the timed region: two pods through the real operator and
kubelet emulator (``--job-gpus 0,0`` lets them share the GPU), Succeeded, with the pods'
steady-state step-time percentiles in the line.
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


@pytest.mark.timeout(300)
def test_bench_self_launch(tmp_path):
    """The driver's bare command ``python3 bench.py --gpus 2 ...`` (no torchrun, no WORLD_SIZE):
    bench.py starts the two ranks itself and rank 0's line reports a two-rank run."""
    out = tmp_path / "bench.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(ROOT)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "20",
           "--warmup", "5", "--job-latency", "0", "--json-out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line == json.loads(out.read_text())
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["steps"] == 20, line
    assert line["replicas_in_sync"] is True and line["grad_allreduce_error"] == 0, line
    assert line["launcher"] == "bench.py->torch.distributed.run", line
    assert line["rccl_nranks"] is None and line["config"]["backend"] == "gloo", line
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / "bench_self_launch_w2.json").write_text(json.dumps(line))


@pytest.mark.timeout(200)
def test_bench_rccl_nranks_world1(tmp_path):
    """Forced single-rank RCCL group: the line carries the communicator's own rank count."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(ROOT)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--backend", "nccl", "--force-collectives", "1",
           "--steps", "20", "--warmup", "5", "--job-latency", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric"')][0])
    assert line["world_size"] == 1 and line["rccl_nranks"] == 1, line
    assert line["config"]["backend"] == "rccl", line


@pytest.mark.timeout(400)
@pytest.mark.parametrize("allreduce", ["xgmi", "auto", "auto-slow-xgmi", "auto-xgmi-stall"])
def test_bench_two_ranks_one_gpu(tmp_path, allreduce):
    """``auto-slow-xgmi``: PTO_RACE_DELAY_MS makes the xGMI candidate slow, so the race must
    pick RCCL, and the timed runner must then be the stream-launched RCCL step.
    ``auto-xgmi-stall``: rank 1 sleeps past the exchange's 5 s wait before the fused xGMI form's
    trial, so its exchange fails: that form is dropped, the protocol state is reset and the
    replicas resync from rank 0; the round-5 xGMI form then races from a clean start, and the
    timed steps stay in sync."""
    out = tmp_path / "bench.json"
    env = dict(os.environ, PYTHONPATH=str(ROOT), PTO_XGMI_ANY_BACKEND="1")
    slow_xgmi = stall = False
    if allreduce == "auto-slow-xgmi":
        env["PTO_RACE_DELAY_MS"] = "xgmi:5"
        allreduce = "auto"
        slow_xgmi = True
    elif allreduce == "auto-xgmi-stall":
        env["PTO_RACE_STALL"] = "xgmi:1:6"
        allreduce = "auto"
        stall = True
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--allreduce", allreduce, "--steps", "20", "--warmup", "5",
           "--job-gpus", "0,0", "--job-timeout", "200", "--json-out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, cwd=ROOT, env=env)
    assert r.returncode == 0 and out.exists(), r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == 2 and line["steps"] == 20 and line["warmup"] == 5
    assert line["config"]["parallelism"] == "dp2" and line["config"]["backend"] == "gloo"
    assert line["replicas_in_sync"] is True, line
    assert line["grad_allreduce_error"] == 0, line
    if allreduce == "xgmi":
        assert line["config"]["grad_allreduce"] == "xgmi", line
    else:
        trial = line["config"]["allreduce_trial"]
        assert trial is not None, line
        # every candidate reported: RCCL stream-launched (not the 3-hipGraph form), xGMI timed,
        # the captured one-graph RCCL step skipped on gloo (its collectives are not capturable)
        assert trial["rccl_launch"] == "stream", trial
        if stall:
            # the stall comes after xgmi's check, in its timed trial: xgmi is dropped, every rank's
            # protocol state is reset, and xgmi-r5 then runs from a clean start
            assert trial["xgmi_crosscheck"]["xgmi"]["ok"], trial
            assert trial["xgmi_ms_per_step"] is None and set(trial["xgmi_error"]) == {"xgmi"}, trial
            assert trial["xgmi_resynced_from_rank0"] is True, trial
            assert trial["xgmi_crosscheck"]["xgmi-r5"]["ok"] and trial["xgmi_r5_ms_per_step"] > 0, trial
            assert line["job"]["result"] == "Succeeded", line["job"]
            return
        assert trial["rccl_ms_per_step"] > 0 and trial["xgmi_ms_per_step"] > 0, trial
        assert trial["rccl_graph_ms_per_step"] is None and "gloo" in trial["rccl_graph_skipped"], trial
        assert line["config"]["grad_allreduce"] == trial["picked"], line
        # both DDP forms of each path raced (round 6: fused, and the round-5 form as "-r5")
        assert trial["rccl_r5_ms_per_step"] > 0 and trial["xgmi_r5_ms_per_step"] > 0, trial
        assert trial["ddp_form"] == ("r5" if trial["picked"].endswith("-r5") else "fused"), trial
        # each xGMI form was checked against a step over the other path before it was timed
        cc = trial["xgmi_crosscheck"]
        assert set(cc) == {"xgmi", "xgmi-r5"} and all(v["ok"] for v in cc.values()), cc
        if slow_xgmi:
            assert trial["picked"] in ("rccl", "rccl-r5"), trial
            assert trial["xgmi_ms_per_step"] > trial["rccl_ms_per_step"], trial
            assert "launch=stream" in line["config"]["exec"], line
        # the operator-deployed pods ran the same race
        assert line["job"]["allreduce_trial"] is not None, line["job"]
    assert line["value"] > 0 and line["ms_per_step"] > 0
    job = line["job"]
    assert job.get("result") == "Succeeded" and job.get("replicas") == 2, job
    assert job["node_gpus"] == [0, 0] and job["backend"] == "gloo", job
    sm = job.get("worker_step_ms")
    assert sm and sm["n"] > 0 and 0 < sm["p50"] <= sm["p90"], job
    assert job["worker_capture_seconds"] is not None and job["worker_train_seconds"] > 0, job
    # create -> first step of the two-pod job, and where it went
    assert line["create_to_first_step_s"] is not None and line["create_to_first_step_s"] > 0, line
    bd = job["startup_breakdown"]
    assert bd and bd["job_create_to_process_start_s"] > 0 and bd["first_step_s"] > 0, bd
    (tmp_path / "job.json").write_text(json.dumps(job))
    rec = os.environ.get("PTO_TEST_RECORD_DIR")  # keep the line (profiles/ records the world-2 latency)
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / f"bench_w2_{'slow-xgmi' if slow_xgmi else allreduce}.json").write_text(json.dumps(line))
    print(json.dumps({"world2_shared_gpu": {"create_to_first_step_s": line.get("create_to_first_step_s"),
                                             "startup_breakdown": bd, "allreduce": allreduce}}))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [4, 8])
def test_bench_many_ranks_one_gpu(tmp_path, world):
    """The self-launched bench at world 4 and 8 (the node's rank count) on the box's one GPU,
    racing every candidate with the step cross-check.  One hardware queue per process: with HIP's
    default four, the 16 queues of four processes oversubscribe the GPU's scheduler, which then
    time-slices them and an xGMI step waits milliseconds for a descheduled peer (45.6 vs 0.135 ms
    per step, profiles/r6_w4/).  At world 8 the fused form's exchange workgroups of all eight
    ranks cannot be resident at once, so the race skips that form (profiles/r6_reset/).  On the
    node every rank owns its GPU."""
    out = tmp_path / "bench.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    # two host threads per rank: the box's OMP_NUM_THREADS (16) in each of eight ranks oversubscribes
    # its CPU share, and a descheduled rank can miss its peers' bounded exchange wait
    env.update(PYTHONPATH=str(ROOT), PTO_XGMI_ANY_BACKEND="1", GPU_MAX_HW_QUEUES="1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--backend", "gloo", "--steps", "20",
           "--warmup", "5", "--job-latency", "0", "--json-out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert r.returncode == 0 and out.exists(), r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == world and line["world_size"] == world, line
    assert line["replicas_in_sync"] is True and line["grad_allreduce_error"] == 0, line
    trial = line["config"]["allreduce_trial"]
    note = line["config"]["xgmi_note"] or ""
    if world == 8 and trial is None and "self-test failed" in note:
        # a ninth process with a GPU context on the card (this pytest process, after in-process GPU
        # tests) makes the exchange's start-up self-test see wrong sums at world 8 on one GPU
        # (profiles/r6_w8_selftest/README.md): the safety net must then hold -- RCCL carries the
        # gradients and the replicas stay in sync (asserted above)
        assert line["config"]["grad_allreduce"] == "rccl", line
        print(json.dumps({"w8_xgmi_self_test_failed": note[:300]}))
        return
    assert trial is not None, (note, r.stderr[-3000:])
    cc = trial["xgmi_crosscheck"]
    assert all(v["ok"] for v in cc.values()) and trial["xgmi_r5_ms_per_step"] > 0, trial
    if world == 4:
        assert set(cc) == {"xgmi", "xgmi-r5"} and trial["xgmi_ms_per_step"] > 0, trial
    else:
        assert set(cc) == {"xgmi-r5"} and "resident" in trial["xgmi_skipped"], trial
    assert line["config"]["grad_allreduce"] == trial["picked"], line
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / f"bench_w{world}_one_gpu.json").write_text(json.dumps(line))
