"""The DDP gradient-path race survives a candidate that fails on some ranks only:
every rank agrees on the one-graph RCCL candidate's pre-check before any rank issues its
collectives, a capture failure on one rank drops the candidate on all of them (no hang), the
steps taken before the failure are counted, and the communicator is probed before the race
goes on.  Two gloo ranks on the CPU with a stand-in step runner (no GPU)."""
import multiprocessing as mp
import os
import socket

import pytest
import torch


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scenario, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pytorch_operator_amd.parallel.autotune as at

    class Tr:
        device = torch.device("cpu")
        grad_sync = None
        log = []

    class FakeStep:
        def __init__(self, tr, mode="graph", steps_per_graph=1, launch="graph", **kw):
            self.internal_steps, self.launch = 1, launch
            if mode == "graph-comm":
                tr.log.append("graph-comm built")
                if scenario == "capture_fails" and rank == 1:
                    e = RuntimeError("stream capture failed")
                    e.internal_steps = 2
                    raise e

        def warm(self, n):
            pass

    at.GraphedStep = FakeStep
    at.graph_comm_precheck = lambda tr: "no capture here" if scenario == "precheck_fails" and rank == 1 else None
    tr = Tr()
    try:
        _, pick, rec = at.choose_grad_sync(tr, object(), None, trial_steps=2)
        q.put((rank, pick, rec, list(tr.log)))
    finally:
        dist.destroy_process_group()


def _race(scenario):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, scenario, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        rank, pick, rec, log = q.get(timeout=120)
        out[rank] = (pick, rec, log)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    return out


@pytest.mark.timeout(180)
def test_precheck_disagreement_skips_the_candidate_everywhere_before_its_collectives():
    out = _race("precheck_fails")
    for rank, (pick, rec, log) in out.items():
        assert pick == "rccl" and rec["rccl_graph_ms_per_step"] is None
        assert log == []  # no rank built (entered the warm-up collectives of) the candidate
    assert out[1][1]["rccl_graph_skipped"] == "no capture here"
    assert out[0][1]["rccl_graph_skipped"] == "pre-check failed on another rank"


@pytest.mark.timeout(180)
def test_capture_failure_on_one_rank_drops_the_candidate_on_all():
    out = _race("capture_fails")
    for rank, (pick, rec, log) in out.items():
        assert pick == "rccl" and rec["rccl_graph_ms_per_step"] is None
        assert rec["rccl_graph_skipped"].startswith("capture failed")
        assert rec["xgmi_skipped"].startswith("no xGMI")  # the communicator probe passed
    assert "stream capture failed" in out[1][1]["rccl_graph_skipped"]
    # rccl trial: 1 internal + 2 timed; the failed candidate: 2 (rank 1) / 1 (rank 0) internal
    assert out[1][1]["steps"] == 5 and out[0][1]["steps"] == 4


@pytest.mark.timeout(180)
def test_candidate_runs_when_every_rank_can_capture():
    out = _race("ok")
    for rank, (pick, rec, log) in out.items():
        assert rec["rccl_graph_ms_per_step"] is not None and log == ["graph-comm built"]


def _xc_worker(rank, world, port, scenario, q):
    """The xGMI candidates' step cross-check: a stand-in trainer whose step adds its gradient path's
    update; the xGMI stand-in is right, or off by 1e-3 on one rank (a broken exchange)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pytorch_operator_amd.parallel.autotune as at

    class Sync:
        def __init__(self, scale):
            self.scale = scale

    class Xar:
        err = 0

        def gather_sharded_(self, m):
            pass

        def error(self):
            return self.err

        def reset(self):
            XSync.xar.err = 0

        def fits_shared_gpu(self, fc):
            return not (scenario == "nofit" and fc)

    class XSync(Sync):
        xar = Xar()

    class Tr:
        device = torch.device("cpu")
        grad_sync = None
        ddp_fused = True

        def __init__(self):
            self.flat_params = torch.linspace(-1, 1, 100)
            self.flat_momentum = torch.zeros(100)
            self.cursor = torch.zeros(1, dtype=torch.int32)
            self.staged = 0

        def fused_ok(self):
            return True

        def invalidate_stage(self):
            self.staged += 1

        def train_step(self):
            g = torch.sin(self.flat_params + self.cursor.float()) * self.grad_sync.scale
            self.flat_momentum.mul_(0.5).add_(g)
            self.flat_params.sub_(0.01 * self.flat_momentum)
            self.cursor += 1

    class FakeStep:
        def __init__(self, tr, mode="graph", steps_per_graph=1, launch="graph", **kw):
            self.internal_steps, self.launch, self.tr = 0, launch, tr

        def warm(self, n):
            if scenario == "timeout" and rank == 1 and isinstance(self.tr.grad_sync, XSync):
                self.tr.flat_params.add_(1.0)  # an exchange that stopped half-way
                XSync.xar.err = 4

    at.GraphedStep = FakeStep
    at.graph_comm_precheck = lambda tr: "no capture here"
    tr = Tr()
    bad = scenario == "wrong" and rank == 1
    try:
        _, pick, rec = at.choose_grad_sync(tr, Sync(1.0), XSync(1.001 if bad else 1.0), trial_steps=2)
        q.put((rank, pick, rec, int(tr.cursor.item()), tr.staged, tr.flat_params.tolist()))
    finally:
        dist.destroy_process_group()


def _xc_race(scenario, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_xc_worker, args=(r, world, port, scenario, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        rank, pick, rec, cursor, staged, params = q.get(timeout=120)
        out[rank] = (pick, rec, cursor, staged, params)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    return out


@pytest.mark.timeout(180)
def test_xgmi_candidates_pass_the_step_crosscheck():
    for rank, (pick, rec, cursor, staged, _) in _xc_race("right").items():
        cc = rec["xgmi_crosscheck"]
        assert set(cc) == {"xgmi", "xgmi-r5"} and all(v["ok"] for v in cc.values()), cc
        assert all(v["param_err"] < 1e-6 for v in cc.values()), cc
        assert rec["xgmi_ms_per_step"] is not None and rec["xgmi_r5_ms_per_step"] is not None, rec
        assert rec["steps"] == 2 + 2 + 2 * (1 + 2), rec  # rccl, rccl-r5 trials; per xGMI form 1 checked + 2 timed
        assert staged == 2  # the staged batch dropped after each restore
        assert cursor == 2  # the stand-in runners take no steps: the two checks' net steps


@pytest.mark.timeout(180)
def test_a_wrong_xgmi_step_on_one_rank_drops_the_candidates_everywhere():
    out = _xc_race("wrong")
    # the RCCL trajectory: two steps (one per dropped candidate's check), gradient scale 1
    p, m = torch.linspace(-1, 1, 100), torch.zeros(100)
    for c in range(2):
        m = m.mul(0.5).add(torch.sin(p + c))
        p = p - 0.01 * m
    for rank, (pick, rec, cursor, staged, params) in out.items():
        assert pick.startswith("rccl"), (pick, rec)
        assert rec["xgmi_ms_per_step"] is None and rec["xgmi_skipped"].startswith("cross-check vs RCCL failed")
        assert rec["xgmi_r5_skipped"].startswith("cross-check vs RCCL failed")
        assert not rec["xgmi_crosscheck"]["xgmi"]["ok"]
        # a dropped candidate's step is undone: every rank continues from the RCCL step's state
        assert cursor == 2 and staged == 4
        assert torch.equal(torch.tensor(params), p), rank


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4])
def test_an_exchange_error_on_one_rank_resyncs_every_replica(world):
    out = _xc_race("timeout", world)
    assert len(out) == world
    for rank, (pick, rec, cursor, staged, params) in out.items():
        assert pick.startswith("rccl"), (pick, rec)
        assert rec["xgmi_ms_per_step"] is None and rec["xgmi_r5_ms_per_step"] is None, rec
        assert rec["xgmi_resynced_from_rank0"] is True, rec
        assert params == out[0][4], rank  # the replicas agree again (rank 0's state)


def test_physical_gpu_falls_back_to_the_index_without_a_gpu():
    from pytorch_operator_amd.parallel.xgmi import physical_gpu
    assert physical_gpu(torch.device("cuda", 3)) == ("index", 3)


@pytest.mark.timeout(180)
def test_a_fused_exchange_that_cannot_be_resident_is_skipped():
    """Ranks sharing a GPU whose fused-form exchange workgroups cannot all be resident at once:
    that form is skipped everywhere (it could only time out); the round-5 form still races."""
    for rank, (pick, rec, cursor, staged, params) in _xc_race("nofit").items():
        assert rec["xgmi_ms_per_step"] is None and "resident" in rec["xgmi_skipped"], rec
        assert rec["xgmi_r5_ms_per_step"] is not None and set(rec["xgmi_crosscheck"]) == {"xgmi-r5"}, rec
