#!/usr/bin/env python3
"""Job-create-to-first-step latency (BASELINE.md's second headline metric).

Runs a real PyTorchJob through the whole stack -- fake API server -> native C++ operator
-> kubelet emulator -> MNIST DDP worker processes -- and reports, per replica count:

* ``create_to_running_s``   client POST -> the job's Running condition (the reference's
                            only observable: 121 s / 334 s);
* ``create_to_first_step_s`` client POST -> the *last* rank's first optimizer step
                            (``first_step`` JSON line of the worker, wall clock);
* ``create_to_succeeded_s`` client POST -> Succeeded (1 epoch unless --max-steps);
* the worker-reported training throughput.

    python benchmarks/job_latency.py --replicas 1 2 --backend gloo          # CPU
    python benchmarks/job_latency.py --replicas 1 --backend rccl --gpus 0   # MI355X

With ``--gpus`` each replica asks for ``amd.com/gpu: 1``; the kubelet emulator only
schedules as many replicas as listed GPUs.  Times use one host clock (all processes are
local), so no clock skew enters the numbers.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_operator_amd.cluster.local import LocalCluster  # noqa: E402
from kubeflow.pytorchjob.rest import PODS, PYTORCHJOBS  # noqa: E402


def _replica(n, args, gpu):
    c = {"name": "pytorch", "image": "pytorch-operator-amd/worker:latest", "args": args}
    if gpu:
        c["resources"] = {"limits": {"amd.com/gpu": 1}}
    return {"replicas": n, "restartPolicy": "OnFailure", "template": {"spec": {"containers": [c]}}}


def run_one(c: LocalCluster, name: str, replicas: int, args, gpu: bool, timeout: float) -> dict:
    specs = {"Master": _replica(1, args, gpu)}
    if replicas > 1:
        specs["Worker"] = _replica(replicas - 1, args, gpu)
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name},
           "spec": {"cleanPodPolicy": "None", "pytorchReplicaSpecs": specs}}
    t_create = time.time_ns()
    c.rest.create(PYTORCHJOBS, job, "default")
    t_running = t_done = None
    final = None
    while time.time_ns() - t_create < timeout * 1e9:
        st = c.rest.get(PYTORCHJOBS, name, "default").get("status") or {}
        types = [x["type"] for x in st.get("conditions") or []]
        if t_running is None and "Running" in types:
            t_running = time.time_ns()
        if "Succeeded" in types or "Failed" in types:
            t_done = time.time_ns()
            final = types[-1]
            break
        time.sleep(0.02)
    pods = sorted(p["metadata"]["name"] for p in c.rest.list(PODS, "default", f"pytorch-job-name={name}")["items"])
    first, done, paths, startups, trials = [], [], set(), {}, []
    for p in pods:
        for line in c.rest.pod_log(p, "default").splitlines():
            if line.startswith('{"event"'):
                ev = json.loads(line)
                if ev["event"] == "first_step":
                    first.append((ev["unix_ns"], ev.get("rank")))
                elif ev["event"] == "startup":
                    startups[ev.get("rank")] = ev
                elif ev["event"] == "train_done":
                    done.append(ev)
                elif ev["event"] == "grad_allreduce":
                    paths.add(ev.get("path"))
                    if ev.get("trial") and ev.get("rank") == 0:
                        trials.append(ev["trial"])
    s = lambda t: None if t is None else round((t - t_create) / 1e9, 3)  # noqa: E731
    # every rank reports the job-wide aggregate (steps * B * world / t): take rank 0's
    rank0 = [d for d in done if d.get("rank") == 0]
    # where create -> first step goes, for the rank that reached its first step last: the
    # control plane + kubelet (job POST -> worker process start), then the worker's phases
    breakdown = None
    if first:
        t_last, r_last = max(first)
        st = startups.get(r_last)
        if st:
            m = st["marks_unix_ns"]
            breakdown = {"rank": r_last, "job_create_to_process_start_s": s(m.get("process_start")),
                         **st["phases"]}
    return {"replicas": replicas, "result": final,
            "create_to_running_s": s(t_running),
            "create_to_first_step_s": s(max(first)[0]) if len(first) == replicas else None,
            "startup_breakdown": breakdown,
            "create_to_succeeded_s": s(t_done),
            "worker_samples_per_sec": rank0[0].get("samples_per_sec") if rank0 else None,
            # steady state inside the pod: per-step ms of the graphed log blocks (p50/p90/p99),
            # the one-off graph capture kept out of train_seconds
            "worker_step_ms": rank0[0].get("step_ms") if rank0 else None,
            "worker_train_seconds": rank0[0].get("train_seconds") if rank0 else None,
            "worker_capture_seconds": rank0[0].get("capture_seconds") if rank0 else None,
            "grad_allreduce": sorted(x for x in paths if x) or None,
            "allreduce_trial": trials[0] if trials else None,
            "accuracy": rank0[0]["accuracy"] if rank0 else None}


def measure(replicas: int, gpus=None, backend: str = "rccl", timeout: float = 180.0,
            extra_args=(), name: str = "bench-latency",
            operator_args=("--inject-rccl-env", "--xgmi-pod-topology")) -> dict:
    """One job of ``replicas`` pods through the real operator (1 GPU per pod when ``gpus``
    lists node GPU ids) on a kubelet that isolates pods like a real one where the host
    allows it (docs/xgmi_pods.md); the dict of ``run_one`` plus how the pods were placed.
    Used by bench.py after its timed region."""
    args = ["--backend", backend, *extra_args]
    gpu = bool(gpus)
    if not gpu:
        args.append("--no-cuda")
    with LocalCluster(gpus=list(gpus) if gpu else None, operator_args=list(operator_args),
                      isolation="namespaces") as c:
        c.wait_operator_ready()
        r = run_one(c, name, replicas, args, gpu, timeout)
        pod = c.rest.get(PODS, f"{name}-master-0", "default")
        ps = pod.get("spec") or {}
        r["pod_topology"] = {"hostPID": bool(ps.get("hostPID")), "hostIPC": bool(ps.get("hostIPC")),
                             "operator_args": list(operator_args),
                             "kubelet_namespaces": c.kubelet.isolation_active}
        return r


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--replicas", type=int, nargs="+", default=[1, 2])
    p.add_argument("--backend", default="gloo")
    p.add_argument("--gpus", type=int, nargs="*", default=None, help="node GPU ids (enables amd.com/gpu)")
    p.add_argument("--max-steps", type=int, default=0, help="cap steps per epoch (0 = full epoch)")
    p.add_argument("--dataset-size", type=int, default=60000)
    p.add_argument("--timeout", type=float, default=600)
    p.add_argument("--json-out", default=None)
    a = p.parse_args(argv)
    gpu = bool(a.gpus)
    args = ["--backend", a.backend, "--dataset-size", str(a.dataset_size)]
    if not gpu:
        args.append("--no-cuda")
    if a.max_steps:
        args += ["--max-steps", str(a.max_steps)]
    results = []
    with LocalCluster(gpus=a.gpus) as c:
        c.wait_operator_ready()
        for i, n in enumerate(a.replicas):
            r = run_one(c, f"latency-{i}-{n}", n, args, gpu, a.timeout)
            r.update(backend=a.backend, device="mi355x" if gpu else "cpu")
            print(json.dumps(r), flush=True)
            results.append(r)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(results, f, indent=1)
    return 0 if all(r["result"] == "Succeeded" for r in results) else 1


if __name__ == "__main__":
    sys.exit(main())
