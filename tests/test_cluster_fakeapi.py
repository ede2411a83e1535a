"""The fake API server's Kubernetes semantics (what the operator and SDK rely on)."""
import threading
import time

import pytest

from pytorch_operator_amd.cluster.fake_apiserver import FakeApiServer, label_selector_matches
from kubeflow.pytorchjob.rest import (PODS, PYTORCHJOBS, SERVICES, ApiException, Configuration,
                                               KubeRest)


@pytest.fixture()
def api(tmp_path):
    srv = FakeApiServer(log_dir=str(tmp_path)).start()
    srv.install_crds()
    yield srv, KubeRest(Configuration(host=srv.url))
    srv.stop()


def pod(name, labels=None, owner=None):
    md = {"name": name, "labels": labels or {}}
    if owner:
        md["ownerReferences"] = [{"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "name": owner["metadata"]["name"],
                                  "uid": owner["metadata"]["uid"], "controller": True}]
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md,
            "spec": {"containers": [{"name": "c", "image": "i"}]}}


def job(name, master=1, workers=1):
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name},
            "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": master}, "Worker": {"replicas": workers}}}}


def test_create_get_conflict_and_defaults(api):
    _, r = api
    p = r.create(PODS, pod("a"), "ns1")
    assert p["metadata"]["namespace"] == "ns1" and p["metadata"]["uid"]
    assert p["status"]["phase"] == "Pending"
    assert r.get(PODS, "a", "ns1")["metadata"]["uid"] == p["metadata"]["uid"]
    with pytest.raises(ApiException) as e:
        r.create(PODS, pod("a"), "ns1")
    assert e.value.status == 409
    with pytest.raises(ApiException) as e:
        r.get(PODS, "missing", "ns1")
    assert e.value.status == 404


def test_label_selectors(api):
    _, r = api
    r.create(PODS, pod("a", {"app": "x", "role": "master"}), "d")
    r.create(PODS, pod("b", {"app": "x", "role": "worker"}), "d")
    r.create(PODS, pod("c", {"app": "y"}), "d")
    names = lambda sel: sorted(p["metadata"]["name"] for p in r.list(PODS, "d", sel)["items"])  # noqa: E731
    assert names("app=x") == ["a", "b"]
    assert names("app=x,role!=master") == ["b"]
    assert names("role") == ["a", "b"]
    assert names("!role") == ["c"]
    assert names("role in (master, worker),app==x") == ["a", "b"]
    assert names("app notin (x)") == ["c"]
    assert label_selector_matches("", {"a": "b"})


def test_optimistic_concurrency_and_status_subresource(api):
    _, r = api
    j = r.create(PYTORCHJOBS, job("j"), "d")
    j["status"] = {"conditions": [{"type": "Created", "status": "True"}]}
    j2 = r.replace(PYTORCHJOBS, "j", j, "d")  # PUT on the object ignores .status
    assert "status" not in j2 or not j2["status"]
    assert j2["metadata"]["resourceVersion"] == j["metadata"]["resourceVersion"]  # no-op write
    j["spec"]["cleanPodPolicy"] = "All"
    j3 = r.replace(PYTORCHJOBS, "j", j, "d")
    assert j3["metadata"]["generation"] == 2
    with pytest.raises(ApiException) as e:
        r.replace(PYTORCHJOBS, "j", j, "d")  # j carries the now-stale resourceVersion
    assert e.value.status == 409
    cur = r.get(PYTORCHJOBS, "j", "d")
    cur["status"] = {"conditions": [{"type": "Created", "status": "True"}]}
    s = r.replace_status(PYTORCHJOBS, "j", cur, "d")
    assert s["status"]["conditions"][0]["type"] == "Created"
    stale = dict(cur)
    stale["metadata"] = dict(cur["metadata"], resourceVersion="1")
    with pytest.raises(ApiException) as e:
        r.replace_status(PYTORCHJOBS, "j", stale, "d")
    assert e.value.status == 409


def test_crd_validation_rejects_bad_replicas(api):
    _, r = api
    with pytest.raises(ApiException) as e:
        r.create(PYTORCHJOBS, job("bad", master=2), "d")
    assert e.value.status == 422
    with pytest.raises(ApiException) as e:
        r.create(PYTORCHJOBS, job("bad2", workers=0), "d")
    assert e.value.status == 422


def test_merge_patch_and_json_patch(api):
    _, r = api
    r.create(PODS, pod("a", {"x": "1", "y": "2"}), "d")
    p = r.patch(PODS, "a", {"metadata": {"labels": {"x": None, "z": "3"}}}, "d")
    assert p["metadata"]["labels"] == {"y": "2", "z": "3"}
    p = r.patch(PODS, "a", [{"op": "replace", "path": "/metadata/labels/y", "value": "9"}], "d")
    assert p["metadata"]["labels"]["y"] == "9"
    p = r.patch(PODS, "a", {"status": {"phase": "Running"}}, "d", status=True)
    assert p["status"]["phase"] == "Running"


def test_cascading_delete_through_owner_references(api):
    _, r = api
    j = r.create(PYTORCHJOBS, job("j"), "d")
    r.create(PODS, pod("j-master-0", owner=j), "d")
    r.create(SERVICES, {"metadata": {"name": "j-master-0", "ownerReferences": [
        {"uid": j["metadata"]["uid"], "kind": "PyTorchJob", "name": "j"}]}, "spec": {}}, "d")
    r.create(PODS, pod("unrelated"), "d")
    r.delete(PYTORCHJOBS, "j", "d")
    assert [p["metadata"]["name"] for p in r.list(PODS, "d")["items"]] == ["unrelated"]
    assert r.list(SERVICES, "d")["items"] == []


def test_watch_streams_events_from_resource_version(api):
    _, r = api
    rv = r.list(PODS, "d")["metadata"]["resourceVersion"]
    got = []

    def consume():
        for t, o in r.watch(PODS, "d", rv, timeout_seconds=3):
            got.append((t, o["metadata"]["name"]))
            if len(got) == 3:
                return

    th = threading.Thread(target=consume)
    th.start()
    time.sleep(0.2)
    r.create(PODS, pod("w1"), "d")
    r.patch(PODS, "w1", {"metadata": {"labels": {"a": "b"}}}, "d")
    r.delete(PODS, "w1", "d")
    th.join(10)
    assert got == [("ADDED", "w1"), ("MODIFIED", "w1"), ("DELETED", "w1")]


def test_watch_label_selector_and_namespace_filter(api):
    _, r = api
    rv = r.list(PODS)["metadata"]["resourceVersion"]
    r.create(PODS, pod("x", {"k": "v"}), "a")
    r.create(PODS, pod("y", {"k": "w"}), "a")
    r.create(PODS, pod("z", {"k": "v"}), "b")
    evs = list(r.watch(PODS, "a", rv, label_selector="k=v", timeout_seconds=1))
    assert [o["metadata"]["name"] for _, o in evs] == ["x"]
    evs = list(r.watch(PODS, None, rv, label_selector="k=v", timeout_seconds=1))
    assert sorted(o["metadata"]["name"] for _, o in evs) == ["x", "z"]


def test_watch_too_old_resource_version_is_410(tmp_path):
    srv = FakeApiServer().start()
    srv.store.events = type(srv.store.events)(maxlen=5)
    r = KubeRest(Configuration(host=srv.url))
    try:
        for i in range(20):
            r.create(PODS, pod(f"p{i}"), "d")
        with pytest.raises(ApiException) as e:
            list(r.watch(PODS, "d", "2", timeout_seconds=1))
        assert e.value.status == 410
    finally:
        srv.stop()


def test_pod_logs_endpoint(api, tmp_path):
    srv, r = api
    r.create(PODS, pod("l"), "d")
    (tmp_path / "d_l.log").write_text("line1\nline2\nline3\n")
    assert r.pod_log("l", "d") == "line1\nline2\nline3\n"
    assert r.pod_log("l", "d", tail_lines=1).strip() == "line3"


def test_kubeconfig_roundtrip(api, tmp_path):
    from kubeflow.pytorchjob.rest import load_kube_config
    srv, _ = api
    path = srv.write_kubeconfig(str(tmp_path / "kc.json"), namespace="team")
    cfg = load_kube_config(path)
    assert cfg.host == srv.url and cfg.namespace == "team" and cfg.token == "fake-token"
    assert KubeRest(cfg).list(PYTORCHJOBS, "team")["items"] == []
