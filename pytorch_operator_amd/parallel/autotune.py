"""Pick the fastest DDP gradient path on the actual hardware, at start-up.

The reference synchronises gradients with DDP's bucketed all-reduce
(examples/mnist/mnist.py:135-138).  Here three ways to run the same DDP step race:

``rccl``        two flat-bucket RCCL all-reduces between the three pieces of the step (fc bucket
                overlapping the conv backward), each piece's kernels launched from C++ straight
                onto the stream (``launch="stream"``; ``"graph"`` replays hipGraphs instead);
``rccl-graph``  the whole step with its RCCL collectives captured into ONE hipGraph per step
                (``GraphedStep(mode="graph-comm")``; RCCL only -- gloo collectives are not
                capturable, so with gloo this candidate is reported as skipped);
``xgmi``        the peer-memory exchange kernel fused with SGD (``parallel.xgmi``), one whole
                step per kernel list.  ``xgmi_sync=None`` (no peer exchange: world 1 with forced
                collectives, or a failed self-test) races the two RCCL forms alone.

Each of ``rccl`` / ``rccl-graph`` / ``xgmi`` runs the round-6 fused DDP step (the single-GPU step's
kernels with the gradient tail: 6 launches + one all-reduce over RCCL, 5 launches over xGMI with
the fc gradients computed in the exchange).  ``rccl-r5`` and ``xgmi-r5`` race the round-5 forms
beside them (head launch + fc1_bwd: the fc bucket's all-reduce overlaps the conv backward over
RCCL; dW_fc1 pushed by fc1_bwd over xGMI): which one wins depends on the fabric's all-reduce
latency and on whether ranks share CUs, so it is measured (``PTO_RACE_SKIP`` names candidates to
leave out).

Whether the xGMI kernel beats RCCL for this 1.7 MB gradient is a property of the fabric the job
lands on, so it is measured rather than assumed: every candidate runs ``trial_steps`` real DDP
steps (replicas stay identical), each trial is timed as the MAX over ranks, and every rank adopts
the lowest time (identical numbers on every rank, so an identical choice; an all-reduce checks
it).  The same procedure runs in ``bench.py`` and in the operator-deployed worker
(``harness/mnist.py --allreduce auto``).

Before an xGMI candidate is timed, one step of it is checked against one step over RCCL from the
same state (parameters, momentum, batch cursor): parameters and momentum must agree to fp32
summation-order noise on every rank, or the candidate is dropped (``xgmi_crosscheck`` in the
record).  The start-up self-test exercises the exchange alone; this pins the whole DDP step it
takes part in -- producer pushes, the fc tiles of the fused form, the slab reduction, the sharded
momentum -- at the job's own world size and geometry.

``PTO_RACE_DELAY_MS="<candidate>:<ms>"`` (fault injection for tests) adds ``ms`` per step of host
sleep inside that candidate's timed trial.  ``PTO_RACE_STALL="<candidate>:<rank>:<seconds>"`` makes
that rank sleep before the candidate's timed trial, after its peers have started theirs (an xGMI
candidate's peers then time out in the exchange: the resync path).
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .graphed_step import GraphedStep

CANDIDATES = ("rccl", "rccl-graph", "xgmi", "rccl-r5", "xgmi-r5")


def _skip_listed(name: str) -> bool:
    return name in os.environ.get("PTO_RACE_SKIP", "").split(",")


def _delay_ms(name: str) -> float:
    """The fault-injection delay of candidate ``name``: an entry for ``k`` applies to ``k`` and to its
    round-5 form ``k-r5`` (``xgmi:5`` slows both xGMI candidates, not ``rccl-graph``)."""
    spec = os.environ.get("PTO_RACE_DELAY_MS", "")
    for part in spec.split(","):
        if ":" in part:
            k, v = part.split(":", 1)
            if name in (k.strip(), k.strip() + "-r5"):
                return float(v)
    return 0.0


def _sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _stall(name: str) -> None:
    spec = os.environ.get("PTO_RACE_STALL", "")
    if spec.count(":") == 2:
        k, r, sec = spec.split(":")
        if k.strip() == name and int(r) == dist.get_rank():
            time.sleep(float(sec))


def _timed(runner: GraphedStep, steps: int, device, name: str) -> float:
    _sync(device)
    dist.barrier()
    _stall(name)
    t0 = time.perf_counter()
    runner.warm(steps)
    delay = _delay_ms(name)
    if delay > 0:
        time.sleep(delay * steps / 1e3)
    _sync(device)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def graph_comm_precheck(tr) -> Optional[str]:
    """Why this rank cannot capture the step with its collectives (None: it can).  Local checks
    only -- no collective is issued -- so every rank can agree on the answer before any rank
    enters the candidate's warm-up collectives (a rank raising inside them while the
    others wait in an all-reduce would hang the job)."""
    if dist.get_backend() != "nccl":
        return f"{dist.get_backend()} collectives are not capturable"
    if "rccl-graph" in os.environ.get("PTO_RACE_SKIP", "").split(","):
        return "PTO_RACE_SKIP"
    try:
        ver = torch.cuda.nccl.version()
    except Exception as e:  # noqa: BLE001
        return f"RCCL version unknown: {e!r}"[:120]
    if tuple(ver[:2]) < (2, 9):
        return f"RCCL {ver} predates collective stream capture"
    gs = tr.grad_sync
    if gs is None or not bool(getattr(gs, "active", True)) or getattr(gs, "fused_sgd", False):
        return "the step issues no RCCL collective"
    if os.environ.get("PTO_FAULT_GRAPH_COMM_PRECHECK") == str(dist.get_rank()):
        return "fault injection"  # tests: one rank says no
    return None


def crosscheck_step(tr, rccl_sync, xgmi_sync, dev, rtol: float = 1e-4) -> Dict:
    """One step over xGMI vs one step over RCCL from the same state (the trainer's current form).

    Leaves the trainer one step further (the xGMI step's state, momentum gathered whole).  Returns
    ``{"ok", "param_err", "mom_err"}``; ``ok`` is agreed over ranks.  Errors are max |difference|
    relative to max |reference| (parameters) and max |momentum| (momentum)."""
    # an xGMI step before this one left the momentum sharded (each rank updates the shard it
    # owns): make it whole first, or the RCCL reference steps from stale momentum
    xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
    snap = (tr.flat_params.clone(), tr.flat_momentum.clone(), tr.cursor.clone())
    tr.grad_sync = rccl_sync
    tr.train_step()
    p_ref, m_ref, c_ref = tr.flat_params.clone(), tr.flat_momentum.clone(), tr.cursor.clone()
    tr.flat_params.copy_(snap[0])
    tr.flat_momentum.copy_(snap[1])
    tr.cursor.copy_(snap[2])
    if hasattr(tr, "invalidate_stage"):
        tr.invalidate_stage()  # the staged batch is the NEXT step's: stage again from the cursor
    tr.grad_sync = xgmi_sync
    ok = True
    # every rank's GPU idle before any rank's exchange spins: work a rank still has queued (the
    # host collectives' copies) must not wait for CUs held by a peer's exchange on a shared GPU
    _sync(dev)
    dist.barrier()
    try:
        tr.train_step()
        xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
        _sync(dev)
        pe = float((tr.flat_params - p_ref).abs().max() / p_ref.abs().max().clamp_min(1e-30))
        me = float((tr.flat_momentum - m_ref).abs().max() / m_ref.abs().max().clamp_min(1e-30))
        err = int(xgmi_sync.xar.error())
        ok = pe <= rtol and me <= rtol and not err
    except Exception as e:  # noqa: BLE001 -- a failing candidate is dropped, not fatal
        pe = me = float("inf")
        ok, err = False, -1
        tr.last_crosscheck_error = repr(e)[:200]
    ok = _agree(ok, dev)
    if not ok:
        # the dropped candidate's step may have left anything behind (a timed-out exchange stops
        # half-way): continue from the RCCL step's state, which every rank holds
        tr.flat_params.copy_(p_ref)
        tr.flat_momentum.copy_(m_ref)
        tr.cursor.copy_(c_ref)
        if hasattr(tr, "invalidate_stage"):
            tr.invalidate_stage()
        _sync(dev)
    return {"ok": ok, "param_err": pe, "mom_err": me, "xgmi_error": err}


def _restart_exchange(tr, xgmi_sync, dev) -> None:
    """After an xGMI exchange failed on any rank: zero every rank's protocol state, so the next
    candidate gets a clean start, and restart all replicas from rank 0's parameters and momentum
    (a timed-out exchange falls back to a rank-local SGD step, and the replicas drift apart)."""
    _sync(dev)
    dist.barrier()  # no exchange in flight on any rank
    xgmi_sync.xar.reset()
    xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
    dist.broadcast(tr.flat_params, 0)
    dist.broadcast(tr.flat_momentum, 0)
    _sync(dev)
    dist.barrier()  # every rank's protocol state zeroed before any rank's next exchange


def _agree(flag: bool, dev) -> bool:
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def choose_grad_sync(tr, rccl_sync, xgmi_sync=None, mode: str = "graph", spg: int = 10,
                     trial_steps: int = 60, force: Optional[str] = None,
                     launch: str = "stream") -> Tuple[GraphedStep, str, Dict]:
    """Returns (runner, path, record).  ``path`` is one of ``CANDIDATES``; ``record`` holds
    every candidate's per-step trial time in ms (None when skipped, with the reason), the RCCL
    runner's launch form and ``steps``: the training steps taken here.  ``force`` overrides the
    measured decision (tests cover every hand-over with it).  ``spg``: whole steps per replay of
    a returned graph-replayed xGMI runner.  ``mode="eager"`` races eager launches instead."""
    trial = max(1, int(trial_steps))
    dev = tr.device
    eager = mode == "eager"
    times: Dict[str, Optional[float]] = {}
    runners: Dict[str, GraphedStep] = {}
    skipped: Dict[str, str] = {}
    crosscheck: Dict[str, Dict] = {}
    errors: Dict[str, int] = {}
    resynced = False
    steps = 0
    # the RCCL steps keep momentum for every parameter: make it whole if fused xGMI steps ran
    # before (a no-op when it already is)
    if xgmi_sync is not None:
        xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
    tr.grad_sync = rccl_sync
    fused = bool(getattr(tr, "fused_ok", lambda: False)())  # candidates without -r5: the fused form
    forms = {k: (k.endswith("-r5") or not fused) for k in CANDIDATES}  # True: the round-5 form

    def set_form(name):
        tr.ddp_fused = not forms[name]

    set_form("rccl")
    r = GraphedStep(tr, mode="eager" if eager else "graph", steps_per_graph=1, launch=launch)
    runners["rccl"] = r
    times["rccl"] = _timed(r, trial, dev, "rccl")
    steps += r.internal_steps + trial
    if not fused:
        skipped["rccl-r5"] = "the trainer runs the round-5 form already (ddp_fused off)"
    elif _skip_listed("rccl-r5"):
        skipped["rccl-r5"] = "PTO_RACE_SKIP"
    else:
        set_form("rccl-r5")
        r = GraphedStep(tr, mode="eager" if eager else "graph", steps_per_graph=1, launch=launch)
        runners["rccl-r5"] = r
        times["rccl-r5"] = _timed(r, trial, dev, "rccl-r5")
        steps += r.internal_steps + trial
    set_form("rccl-graph")
    why = "eager race" if eager else graph_comm_precheck(tr)
    # every rank agrees on the pre-check before any rank issues the candidate's collectives
    if not _agree(why is None, dev):
        skipped["rccl-graph"] = why or "pre-check failed on another rank"
    else:
        # past the pre-check, the candidate's eager warm-up steps are the rccl trial's (which just
        # ran on every rank); what can still fail is the capture itself, which issues no
        # collective -- so a failing rank reaches the agreement below like the others
        err = None
        try:
            r = GraphedStep(tr, mode="graph-comm")
        except Exception as e:  # noqa: BLE001 -- the race must survive a failed candidate
            err, r = repr(e)[:200], None
            steps += int(getattr(e, "internal_steps", 0))
        if _agree(err is None, dev):
            runners["rccl-graph"] = r
            times["rccl-graph"] = _timed(r, trial, dev, "rccl-graph")
            steps += r.internal_steps + trial
        else:
            if r is not None:
                steps += r.internal_steps
            skipped["rccl-graph"] = f"capture failed: {err or 'on another rank'}"
            # leave no half-captured work behind, then prove the stream and the communicator
            # still work (one all-reduce every rank issues); if they do not, no further trials
            _sync(dev)
            try:
                probe = torch.ones(1, device=dev)
                dist.all_reduce(probe)
                _sync(dev)
                healthy = int(probe.item()) == dist.get_world_size()
            except Exception:  # noqa: BLE001
                healthy = False
            if not healthy:
                skipped["xgmi"] = "communicator unhealthy after a failed capture"
                xgmi_sync = None
                skipped.setdefault("rccl-graph", "capture failed")
    if xgmi_sync is None:
        skipped.setdefault("xgmi", "no xGMI exchange (world 1 or self-test failed)")
        skipped.setdefault("xgmi-r5", skipped["xgmi"])
    else:
        tr.grad_sync = xgmi_sync
        for name in ("xgmi", "xgmi-r5"):
            if name == "xgmi-r5" and not fused:
                skipped[name] = "the trainer runs the round-5 form already (ddp_fused off)"
                continue
            if name == "xgmi-r5" and _skip_listed(name):
                skipped[name] = "PTO_RACE_SKIP"
                continue
            # ranks sharing one GPU finish an exchange only when all of their exchange workgroups
            # are resident together (the one-GPU rehearsals; one rank per GPU always fits)
            if not _agree(xgmi_sync.xar.fits_shared_gpu(fc=not forms[name]), dev):
                skipped[name] = "its exchange workgroups of every rank sharing the GPU cannot be resident at once"
                continue
            set_form(name)
            if os.environ.get("PTO_RACE_CROSSCHECK", "1") != "0":
                chk = crosscheck_step(tr, rccl_sync, xgmi_sync, dev)
                steps += 1
                crosscheck[name] = {k: (round(v, 9) if isinstance(v, float) else v) for k, v in chk.items()}
                tr.grad_sync = xgmi_sync
                if not chk["ok"]:
                    skipped[name] = (f"cross-check vs RCCL failed (param {chk['param_err']:.2e}, "
                                     f"momentum {chk['mom_err']:.2e}, exchange error {chk['xgmi_error']})")
                    if not _agree(chk["xgmi_error"] == 0, dev):
                        _restart_exchange(tr, xgmi_sync, dev)
                    continue
            r = GraphedStep(tr, mode="eager" if eager else "graph", steps_per_graph=spg, launch=launch)
            runners[name] = r
            t = _timed(r, trial, dev, name)
            steps += r.internal_steps + trial
            # an exchange that timed out mid-trial may have stopped half-way on some ranks only:
            # agree on it, drop the candidate everywhere, restart the protocol and the replicas
            err = int(xgmi_sync.xar.error())
            times[name] = t
            if not _agree(err == 0, dev):
                times[name] = float("inf")
                errors[name] = err
                _restart_exchange(tr, xgmi_sync, dev)
                resynced = True
    if force is not None:
        if force not in runners:
            raise ValueError(f"force={force!r}: candidate not available ({skipped.get(force, 'unknown')})")
        pick = force
    else:
        pick = min(times, key=lambda k: (times[k], CANDIDATES.index(k)))
    # identical MAX-over-ranks numbers give an identical pick everywhere; check it anyway
    idx = torch.tensor([CANDIDATES.index(pick)], dtype=torch.int32, device=dev)
    lo, hi = idx.clone(), idx.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if int(lo.item()) != int(hi.item()):
        pick = "rccl"  # ranks disagree (cannot happen with shared numbers): the safe path
    if not pick.startswith("xgmi"):
        if xgmi_sync is not None:
            xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
        tr.grad_sync = rccl_sync
    else:
        tr.grad_sync = xgmi_sync
    set_form(pick)  # later eager steps of the trainer take the picked form too
    _sync(dev)
    dist.barrier()  # the agreement's copies done on every rank before the picked runner's first step
    record = {f"{k.replace('-', '_')}_ms_per_step": (round(v / trial * 1e3, 4) if v != float("inf") else None)
              for k, v in times.items()}
    for k, why in skipped.items():
        record[f"{k.replace('-', '_')}_ms_per_step"] = None
        record[f"{k.replace('-', '_')}_skipped"] = why
    if crosscheck:
        record["xgmi_crosscheck"] = crosscheck
    if errors:
        record["xgmi_error"] = errors  # this rank's error word per failed candidate (0: a peer's failed)
        record["xgmi_resynced_from_rank0"] = resynced
    record.update({"picked": pick, "rccl_launch": runners["rccl"].launch, "trial_steps": trial,
                   "steps": steps, "ddp_form": "r5" if forms[pick] else "fused"})
    return runners[pick], pick, record
