#!/usr/bin/env python3
"""The reference SDK notebook (sdk/python/examples/kubeflow-pytorchjob-sdk.ipynb) as a script:
create -> get -> watch -> wait -> is_job_succeeded -> get_logs -> delete.

By default it starts a local cluster (fake API server + kubelet emulator + the native
operator); pass --kubeconfig to use a real cluster instead.

    python examples/sdk/pytorchjob_sdk_demo.py [--gpu] [--kubeconfig ~/.kube/config]
"""
import argparse
import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdk", "python")]

from kubeflow.pytorchjob import (PyTorchJobClient, V1Container, V1ObjectMeta, V1PodSpec,  # noqa: E402
                                 V1PodTemplateSpec, V1PyTorchJob, V1PyTorchJobSpec, V1ReplicaSpec,
                                 V1ResourceRequirements)


def build_job(name: str, gpu: bool) -> V1PyTorchJob:
    args = ["--backend", "rccl" if gpu else "gloo", "--dataset-size", "20000"]
    if not gpu:
        args.append("--no-cuda")
    container = V1Container(
        name="pytorch", image="pytorch-operator-amd/worker:latest", args=args,
        resources=V1ResourceRequirements(limits={"amd.com/gpu": 1}) if gpu else None)
    replica = lambda n: V1ReplicaSpec(replicas=n, restart_policy="OnFailure",  # noqa: E731
                                      template=V1PodTemplateSpec(spec=V1PodSpec(containers=[container])))
    specs = {"Master": replica(1)} if gpu else {"Master": replica(1), "Worker": replica(1)}
    return V1PyTorchJob(api_version="kubeflow.org/v1", kind="PyTorchJob",
                        metadata=V1ObjectMeta(name=name, namespace="default"),
                        spec=V1PyTorchJobSpec(clean_pod_policy="None", pytorch_replica_specs=specs))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--gpu", action="store_true", help="request amd.com/gpu (needs an MI355X)")
    a = ap.parse_args(argv)
    with contextlib.ExitStack() as stack:
        kubeconfig = a.kubeconfig
        if kubeconfig is None:
            from pytorch_operator_amd.cluster.local import LocalCluster
            c = stack.enter_context(LocalCluster(gpus=[0] if a.gpu else None))
            c.wait_operator_ready()
            kubeconfig = c.kubeconfig
        client = PyTorchJobClient(config_file=kubeconfig)
        name = "pytorch-dist-mnist-sdk"
        client.create(build_job(name, a.gpu))
        print(client.get(name, namespace="default")["status"] if "status" in client.get(name, namespace="default")
              else "created")
        client.get(name, namespace="default", watch=True, timeout_seconds=600)  # NAME STATE TIME table
        client.wait_for_job(name, namespace="default", polling_interval=1)
        print("succeeded:", client.is_job_succeeded(name, namespace="default"))
        logs = client.get_logs(name, namespace="default")
        print([ln for ln in next(iter(logs.values())).splitlines() if ln.startswith("accuracy=")])
        client.delete(name, namespace="default")
    return 0


if __name__ == "__main__":
    sys.exit(main())
