"""End to end on a real MI355X: operator binary + local cluster + the HIP MNIST worker.

A PyTorchJob asking for ``amd.com/gpu: 1`` is scheduled by the kubelet emulator onto the
box's GPU (HIP_VISIBLE_DEVICES), the worker trains on the fused gfx950 kernels with
``--backend rccl`` and the job must reach Succeeded with a learned model.
"""
import json
import time

import pytest

from pytorch_operator_amd.cluster.local import LocalCluster
from pytorch_operator_amd.cluster.rest import PYTORCHJOBS

pytestmark = pytest.mark.gpu


def _wait(c, name, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        j = c.rest.get(PYTORCHJOBS, name, "default")
        types = [x["type"] for x in (j.get("status") or {}).get("conditions") or []]
        if "Succeeded" in types or "Failed" in types:
            return j, types
        time.sleep(0.2)
    raise TimeoutError(name)


def test_gpu_mnist_job_hip_kernels(tmp_path):
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "mnist-gpu"},
           "spec": {"cleanPodPolicy": "None", "pytorchReplicaSpecs": {"Master": {
               "replicas": 1, "restartPolicy": "OnFailure",
               "template": {"spec": {"containers": [{
                   "name": "pytorch", "image": "pytorch-operator-amd/worker:latest",
                   "args": ["--backend", "rccl", "--dataset-size", "20000", "--test-size", "2000",
                            "--log-interval", "10"],
                   "resources": {"limits": {"amd.com/gpu": 1}}}]}}}}}}
    with LocalCluster(workdir=str(tmp_path / "c"), gpus=[0]) as c:
        c.wait_operator_ready()
        t0 = time.time()
        c.rest.create(PYTORCHJOBS, job, "default")
        j, types = _wait(c, "mnist-gpu")
        elapsed = time.time() - t0
        log = c.rest.pod_log("mnist-gpu-master-0", "default")
        assert types[-1] == "Succeeded", log[-3000:]
        events = [json.loads(x) for x in log.splitlines() if x.startswith('{"event"')]
        start = next(e for e in events if e["event"] == "start")
        done = next(e for e in events if e["event"] == "train_done")
        assert start["kernels"] == "hip"
        assert done["accuracy"] > 0.9, log[-2000:]
        print(f"job wall {elapsed:.2f}s, train {done['samples_per_sec']} samples/s, acc {done['accuracy']}")
