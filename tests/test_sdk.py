"""The Python SDK (kubeflow.pytorchjob) against the local cluster.

Mirrors the reference SDK tests: model construction/serialisation
(sdk/python/test/test_v1_*.py, which are stubs there) and the SDK e2e flow
(sdk/python/test/test_e2e.py: create -> wait_for_job -> is_job_succeeded -> get_logs ->
delete) with the reference's own model classes and call sequence.
"""
import io

import pytest

from kubeflow.pytorchjob import (ApiClient, Configuration, PyTorchJobClient, V1Container, V1JobCondition,
                                 V1JobStatus, V1ObjectMeta, V1PodSpec, V1PodTemplateSpec, V1PyTorchJob,
                                 V1PyTorchJobList, V1PyTorchJobSpec, V1ReplicaSpec, V1ReplicaStatus,
                                 V1ResourceRequirements, utils)
from kubeflow.pytorchjob.api.py_torch_job_watch import watch
from pytorch_operator_amd.cluster.local import LocalCluster

NS = "default"


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    c = LocalCluster(workdir=str(tmp_path_factory.mktemp("sdk")))
    c.start()
    c.wait_operator_ready()
    yield c
    c.stop()


@pytest.fixture(scope="module")
def client(cluster):
    return PyTorchJobClient(config_file=cluster.kubeconfig)


def mnist_job(name, clean="None", workers=1):
    container = V1Container(name="pytorch", image="gcr.io/kubeflow-ci/pytorch-dist-mnist-test:v1.0",
                            args=["--backend", "gloo", "--dataset-size", "1000", "--test-size", "200",
                                  "--max-steps", "5"])
    spec = lambda n: V1ReplicaSpec(replicas=n, restart_policy="OnFailure",  # noqa: E731
                                   template=V1PodTemplateSpec(spec=V1PodSpec(containers=[container])))
    return V1PyTorchJob(api_version="kubeflow.org/v1", kind="PyTorchJob",
                        metadata=V1ObjectMeta(name=name, namespace=NS),
                        spec=V1PyTorchJobSpec(clean_pod_policy=clean,
                                              pytorch_replica_specs={"Master": spec(1), "Worker": spec(workers)}))


# ---------------------------------------------------------------- models
def test_models_serialise_with_json_keys():
    job = mnist_job("m")
    body = ApiClient().sanitize_for_serialization(job)
    assert body["apiVersion"] == "kubeflow.org/v1"
    assert body["spec"]["cleanPodPolicy"] == "None"
    rs = body["spec"]["pytorchReplicaSpecs"]["Worker"]
    assert rs["restartPolicy"] == "OnFailure" and rs["template"]["spec"]["containers"][0]["name"] == "pytorch"
    assert ApiClient().deserialize(body, V1PyTorchJob) == job
    assert job.to_dict()["spec"]["clean_pod_policy"] == "None"


def test_required_fields_are_enforced():
    with pytest.raises(ValueError):
        V1JobCondition(type="Created")
    with pytest.raises(ValueError):
        V1PyTorchJobSpec()
    with pytest.raises(ValueError):
        V1JobStatus(conditions=[])
    with pytest.raises(ValueError):
        V1PyTorchJobList()
    with pytest.raises(TypeError):
        V1ReplicaStatus(bogus=1)
    st = V1JobStatus(conditions=[V1JobCondition(type="Created", status="True")],
                     replica_statuses={"Master": V1ReplicaStatus(active=1)})
    assert st.replica_statuses["Master"].active == 1
    assert "Created" in repr(st)


def test_deserialize_server_status():
    data = {"conditions": [{"type": "Running", "status": "True", "lastTransitionTime": "2020-01-01T00:00:00Z"}],
            "replicaStatuses": {"Worker": {"active": 2}}, "startTime": "2020-01-01T00:00:00Z"}
    st = ApiClient().deserialize(data, V1JobStatus)
    assert st.conditions[0].type == "Running"
    assert st.replica_statuses["Worker"].active == 2
    assert st.start_time == "2020-01-01T00:00:00Z"


def test_utils_labels_and_selector():
    labels = utils.get_labels("j", master=True, replica_type="Worker", replica_index=0)
    assert labels["job-role"] == "master" and labels["pytorch-replica-type"] == "worker"
    assert labels["pytorch-replica-index"] == "0"
    assert utils.to_selector({"a": "b", "c": "d"}) == "a=b,c=d"
    assert utils.set_pytorchjob_namespace({"metadata": {"namespace": "x"}}) == "x"
    assert utils.set_pytorchjob_namespace(mnist_job("m")) == NS


# ---------------------------------------------------------------- client e2e
def test_sdk_e2e(client):
    """reference sdk/python/test/test_e2e.py, step for step."""
    client.create(mnist_job("pytorchjob-mnist-ci-test"))
    job = client.wait_for_job("pytorchjob-mnist-ci-test", namespace=NS, timeout_seconds=180, polling_interval=0.2)
    assert job["metadata"]["name"] == "pytorchjob-mnist-ci-test"
    assert client.is_job_succeeded("pytorchjob-mnist-ci-test", namespace=NS)
    assert not client.is_job_running("pytorchjob-mnist-ci-test", namespace=NS)
    assert client.get_job_status("pytorchjob-mnist-ci-test", namespace=NS) == "Succeeded"
    logs = client.get_logs("pytorchjob-mnist-ci-test", namespace=NS)
    assert list(logs) == ["pytorchjob-mnist-ci-test-master-0"]
    assert "accuracy=" in logs["pytorchjob-mnist-ci-test-master-0"]
    assert client.get_pod_names("pytorchjob-mnist-ci-test", namespace=NS) == {
        "pytorchjob-mnist-ci-test-master-0", "pytorchjob-mnist-ci-test-worker-0"}
    assert client.get_pod_names("pytorchjob-mnist-ci-test", namespace=NS, replica_type="worker",
                                replica_index=0) == {"pytorchjob-mnist-ci-test-worker-0"}
    client.delete("pytorchjob-mnist-ci-test", namespace=NS)
    with pytest.raises(RuntimeError):
        client.get("pytorchjob-mnist-ci-test", namespace=NS)


def test_get_list_patch_and_errors(client):
    with pytest.raises(RuntimeError):
        client.create({"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "bad"},
                       "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 3}}}}, namespace=NS)
    job = mnist_job("sdk-patch")
    job.spec.pytorch_replica_specs["Master"].template.spec.containers[0].command = ["python", "-c",
                                                                                   "import time; time.sleep(60)"]
    client.create(job)
    lst = client.get(namespace=NS)
    assert "sdk-patch" in [j["metadata"]["name"] for j in lst["items"]]
    out = client.patch("sdk-patch", {"metadata": {"labels": {"team": "mi355x"}}}, namespace=NS)
    assert out["metadata"]["labels"]["team"] == "mi355x"
    client.wait_for_condition("sdk-patch", ["Running"], namespace=NS, timeout_seconds=60, polling_interval=0.2)
    assert client.is_job_running("sdk-patch", namespace=NS)
    with pytest.raises(RuntimeError, match="Timeout waiting"):
        client.wait_for_condition("sdk-patch", ["Succeeded"], namespace=NS, timeout_seconds=0.5,
                                  polling_interval=0.1)
    client.delete("sdk-patch", namespace=NS)
    with pytest.raises(RuntimeError):
        client.delete("sdk-patch", namespace=NS)


def test_watch_prints_table_until_finished(client, cluster):
    client.create(mnist_job("sdk-watch"))
    buf = io.StringIO()
    final = watch(name="sdk-watch", namespace=NS, timeout_seconds=120, api=client.api, out=buf)
    assert final is not None
    lines = buf.getvalue().splitlines()
    assert lines[0].split() == ["NAME", "STATE", "TIME"]
    assert lines[-1].split()[:2] == ["sdk-watch", "Succeeded"]
    client.delete("sdk-watch", namespace=NS)


def test_client_configuration_object(cluster):
    c = PyTorchJobClient(client_configuration=Configuration(host=cluster.api.url))
    assert "items" in c.get(namespace=NS)


def test_generated_schema_is_up_to_date():
    """The reference's verify-codegen step: docs/pytorchjob.schema.json matches the models."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    r = subprocess.run([sys.executable, str(root / "tools" / "gen_schema.py"), "--check"], capture_output=True)
    assert r.returncode == 0, "run `make schema`"


def test_sdk_is_a_standalone_distribution(cluster, tmp_path):
    """``kubeflow-pytorchjob`` (reference sdk/python/setup.py:26-61) installs and runs on its
    own: pip-install it into an empty target, then drive the SDK e2e flow from a process whose
    sys.path holds that target but not this repository (no pytorch_operator_amd)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import shutil
    target = tmp_path / "site"
    src = tmp_path / "sdk_src"  # a copy: pip's build/ directory must not land in the repository
    shutil.copytree(os.path.join(root, "sdk", "python"), src,
                    ignore=shutil.ignore_patterns("build", "*.egg-info", "__pycache__"))
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-build-isolation",
                        "--no-index", "--target", str(target), str(src)],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    dist = [p.name for p in target.iterdir() if p.name.endswith(".dist-info")]
    assert any(d.startswith("kubeflow_pytorchjob-0.1.4") for d in dist), dist
    script = f"""
import sys, json
assert not any(p.rstrip('/').endswith('repo') for p in sys.path), sys.path
try:
    import pytorch_operator_amd
    raise SystemExit("framework importable: the SDK is not standalone")
except ImportError:
    pass
import kubeflow.pytorchjob as kp
assert kp.__file__.startswith({str(target)!r}), kp.__file__
from kubeflow.pytorchjob import (PyTorchJobClient, V1Container, V1ObjectMeta, V1PodSpec,
                                 V1PodTemplateSpec, V1PyTorchJob, V1PyTorchJobSpec, V1ReplicaSpec)
c = V1Container(name="pytorch", image="gcr.io/kubeflow-ci/pytorch-dist-mnist-test:v1.0",
                args=["--backend", "gloo", "--dataset-size", "640", "--test-size", "128", "--max-steps", "3"])
rs = V1ReplicaSpec(replicas=1, restart_policy="OnFailure",
                   template=V1PodTemplateSpec(spec=V1PodSpec(containers=[c])))
job = V1PyTorchJob(api_version="kubeflow.org/v1", kind="PyTorchJob",
                   metadata=V1ObjectMeta(name="standalone-sdk", namespace="default"),
                   spec=V1PyTorchJobSpec(clean_pod_policy="None", pytorch_replica_specs={{"Master": rs}}))
cl = PyTorchJobClient(config_file={cluster.kubeconfig!r})
cl.create(job)
cl.wait_for_job("standalone-sdk", namespace="default", timeout_seconds=180, polling_interval=1)
assert cl.is_job_succeeded("standalone-sdk", namespace="default")
logs = cl.get_logs("standalone-sdk", namespace="default", follow=True)
assert any("accuracy=" in v for v in logs.values()), logs
cl.delete("standalone-sdk", namespace="default")
print("STANDALONE_OK")
"""
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env["PYTHONPATH"] = str(target)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path), env=env)
    assert r.returncode == 0 and "STANDALONE_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_get_logs_follow_streams_until_the_container_ends(client, cluster):
    """get_logs(follow=True) (reference py_torch_job_client.py:385-386) blocks while the pod
    runs and returns the whole log once its container terminates."""
    import threading
    import time
    code = "import time\nfor i in range(6):\n    print('tick', i, flush=True)\n    time.sleep(0.4)\n"
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "follow-logs"},
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "restartPolicy": "Never", "template": {
               "spec": {"containers": [{"name": "pytorch", "image": "x", "command": ["python", "-c", code]}]}}}}}}
    client.create(job, namespace=NS)
    client.wait_for_condition("follow-logs", ["Running", "Succeeded"], namespace=NS, timeout_seconds=60,
                              polling_interval=0.1)
    t0 = time.time()
    out = client.get_logs("follow-logs", namespace=NS, follow=True)
    log = out["follow-logs-master-0"]
    assert "tick 5" in log and time.time() - t0 > 0.5
    client.delete("follow-logs", namespace=NS)


def test_sdk_reference_docs_are_current():
    """sdk/python/docs/*.md (one page per model + PyTorchJobClient, like the reference SDK's
    docs/) are generated from the field tables and signatures; the committed pages must match."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("gen_sdk_docs", os.path.join(root, "tools", "gen_sdk_docs.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    pages = mod.pages()
    assert len(pages) == 9
    for fn, text in pages.items():
        with open(os.path.join(root, "sdk", "python", "docs", fn)) as f:
            assert f.read() == text, f"{fn} is stale: run tools/gen_sdk_docs.py"
