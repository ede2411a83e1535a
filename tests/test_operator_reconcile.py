"""Ports of the reference's controller unit tests onto the C++ reconcile core.

Reference: pkg/controller.v1/pytorch/{controller,job,pod,service,status,util}_test.go and
pkg/apis/pytorch/validation/validation_test.go.  The Go tests drive the controller through
fake pod/service controls; here reconcile() is pure and returns the same side effects as data.
"""
import json
import subprocess
import time

import pytest

from pytorch_operator_amd.cluster.local import operator_binary
from opfixtures import (NAMESPACE, TEST_JOB_NAME, condition, env_of, labels, new_job, new_pod,
                        new_pods, new_service, opcore, reconcile)


# ------------------------------------------------------------- TestNormalPath
NORMAL_PATH = {
    # name: (workers, master, worker pods (pend,act,succ,fail), master pods (...), master svcs,
    #        exp pod creations, exp pod deletions, exp svc creations,
    #        exp worker (act,succ,fail), exp master (act,succ,fail), exp condition, exp reason, check start)
    "Local PyTorchJob is created": (0, 1, (0, 0, 0, 0), (0, 0, 0, 0), 0, 1, 0, 1,
                                    (0, 0, 0), (0, 0, 0), None, "", False),
    "Distributed PyTorchJob (4 workers, 1 master) is created": (
        4, 1, (0, 0, 0, 0), (0, 0, 0, 0), 0, 5, 0, 1, (0, 0, 0), (0, 0, 0), None, "", False),
    "Distributed PyTorchJob (4 workers, 1 master) is created, 1 master and 4 workers are pending": (
        4, 1, (4, 0, 0, 0), (1, 0, 0, 0), 1, 0, 0, 0, (0, 0, 0), (0, 0, 0), None, "", False),
    "Distributed PyTorchJob (4 workers, 1 master) is created, 2 workers pending, 1 master 1 worker are running": (
        4, 1, (3, 1, 0, 0), (0, 1, 0, 0), 1, 0, 0, 0, (1, 0, 0), (1, 0, 0), "Running", "PyTorchJobRunning", False),
    "Distributed PyTorchJob (4 workers, 1 master) is created and all replicas are running": (
        4, 1, (0, 4, 0, 0), (0, 1, 0, 0), 1, 0, 0, 0, (4, 0, 0), (1, 0, 0), "Running", "PyTorchJobRunning", True),
    "Distributed PyTorchJob (4 workers, 1 master) is succeeded": (
        4, 1, (0, 0, 4, 0), (0, 0, 1, 0), 1, 0, 0, 0, (0, 4, 0), (0, 1, 0), "Succeeded", "PyTorchJobSucceeded", False),
}


@pytest.mark.parametrize("name", list(NORMAL_PATH))
def test_normal_path(name):
    (workers, master, wp, mp, msvc, exp_create, exp_delete, exp_svc, exp_w, exp_m, cond, reason,
     check_start) = NORMAL_PATH[name]
    job = new_job(workers, master=bool(master))
    pods = new_pods(job, "Worker", *wp) + new_pods(job, "Master", *mp)
    services = [new_service(job, "Master", i) for i in range(msvc)]
    r = reconcile(job, pods, services)
    assert r["error"] == ""
    assert len(r["createPods"]) == exp_create
    assert len(r["deletePods"]) == exp_delete
    assert len(r["createServices"]) == exp_svc
    st = r["status"]
    if workers:
        w = st["replicaStatuses"]["Worker"]
        assert (w.get("active", 0), w.get("succeeded", 0), w.get("failed", 0)) == exp_w
    m = st["replicaStatuses"]["Master"]
    assert (m.get("active", 0), m.get("succeeded", 0), m.get("failed", 0)) == exp_m
    if cond:
        c = condition(st, cond)
        assert c is not None and c["status"] == "True" and c["reason"] == reason
    if check_start:
        assert "startTime" in st
    # controllerRef of every created pod (controller_test.go:283-300)
    for p in r["createPods"]:
        ref = p["metadata"]["ownerReferences"][0]
        assert ref["apiVersion"] == "kubeflow.org/v1" and ref["kind"] == "PyTorchJob"
        assert ref["name"] == TEST_JOB_NAME and ref["controller"] is True
        assert ref["blockOwnerDeletion"] is True


def test_created_pod_and_service_shapes():
    job = new_job(2)
    r = reconcile(job)
    names = sorted(p["metadata"]["name"] for p in r["createPods"])
    assert names == [f"{TEST_JOB_NAME}-master-0", f"{TEST_JOB_NAME}-worker-0", f"{TEST_JOB_NAME}-worker-1"]
    master = [p for p in r["createPods"] if p["metadata"]["name"].endswith("master-0")][0]
    assert master["metadata"]["labels"]["job-role"] == "master"
    assert master["metadata"]["labels"]["group-name"] == "kubeflow.org"
    assert master["metadata"]["labels"]["controller-name"] == "pytorch-operator"
    assert master["spec"]["restartPolicy"] == "OnFailure"
    assert "initContainers" not in master["spec"]
    worker = [p for p in r["createPods"] if p["metadata"]["name"].endswith("worker-1")][0]
    assert "job-role" not in worker["metadata"]["labels"]
    ic = worker["spec"]["initContainers"][0]
    assert ic["name"] == "init-pytorch" and ic["image"] == "alpine:3.10"
    assert f"nslookup {TEST_JOB_NAME}-master-0" in ic["command"][2]
    svc = r["createServices"][0]
    assert svc["metadata"]["name"] == f"{TEST_JOB_NAME}-master-0"
    assert svc["spec"]["clusterIP"] == "None"
    assert svc["spec"]["ports"] == [{"name": "pytorchjob-port", "port": 23456}]
    assert svc["spec"]["selector"]["pytorch-replica-type"] == "master"
    assert r["createPodExpectationKeys"][0] == f"{NAMESPACE}/{TEST_JOB_NAME}/master/pods"


# ------------------------------------------------------------- TestClusterSpec
@pytest.mark.parametrize("workers,rtype,index,exp", [
    (0, "Master", 0, {"WORLD_SIZE": "1", "MASTER_PORT": "23456", "RANK": "0", "MASTER_ADDR": "localhost"}),
    (1, "Master", 0, {"WORLD_SIZE": "2", "MASTER_PORT": "23456", "RANK": "0", "MASTER_ADDR": "localhost"}),
    (1, "Worker", 0, {"WORLD_SIZE": "2", "MASTER_PORT": "23456", "RANK": "1",
                      "MASTER_ADDR": f"{TEST_JOB_NAME}-master-0"}),
    (2, "Master", 0, {"WORLD_SIZE": "3", "MASTER_PORT": "23456", "RANK": "0", "MASTER_ADDR": "localhost"}),
    (2, "Worker", 0, {"WORLD_SIZE": "3", "MASTER_PORT": "23456", "RANK": "1",
                      "MASTER_ADDR": f"{TEST_JOB_NAME}-master-0"}),
    (2, "Worker", 1, {"WORLD_SIZE": "3", "MASTER_PORT": "23456", "RANK": "2",
                      "MASTER_ADDR": f"{TEST_JOB_NAME}-master-0"}),
])
def test_cluster_spec(workers, rtype, index, exp):
    job = new_job(workers)
    pod = json.loads(opcore().build_pod(json.dumps(job), rtype, index))
    env = env_of(pod)
    for k, v in exp.items():
        assert env[k] == v
    assert env["PYTHONUNBUFFERED"] == "0"


def test_master_index_must_be_zero():
    job = new_job(0)
    with pytest.raises(RuntimeError, match="only a single master"):
        opcore().build_pod(json.dumps(job), "Master", 1)


# ------------------------------------------------------------- TestRestartPolicy
@pytest.mark.parametrize("policy,expected", [
    ("ExitCode", "Never"), ("Never", "Never"), ("Always", "Always"), ("OnFailure", "OnFailure")])
def test_restart_policy(policy, expected):
    job = new_job(1)
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["restartPolicy"] = policy
    pod = json.loads(opcore().build_pod(json.dumps(job), "Worker", 0))
    assert pod["spec"]["restartPolicy"] == expected


def test_template_restart_policy_warning_event():
    job = new_job(1)
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["restartPolicy"] = "Always"
    r = reconcile(job)
    reasons = [e["reason"] for e in r["events"]]
    assert "SettedPodTemplateRestartPolicy" in reasons


# ------------------------------------------------------------- TestExitCode
def test_exit_code_retryable_pod_deleted_and_restarting():
    job = new_job(1)
    job["spec"]["pytorchReplicaSpecs"]["Master"]["restartPolicy"] = "ExitCode"
    pods = [new_pod(job, "Master", 0, "Failed", exit_code=130), new_pod(job, "Worker", 0, "Running")]
    r = reconcile(job, pods, [new_service(job, "Master", 0)])
    assert r["deletePods"] == [f"{NAMESPACE}/{TEST_JOB_NAME}-master-0"]
    c = condition(r["status"], "Restarting")
    assert c is not None and c["reason"] == "PyTorchJobRestarting"
    assert any(e["reason"] == "ExitedWithCode" and "exited with code 130" in e["message"]
               for e in r["events"])
    assert r["metrics"]["restarted"] == 1


def test_exit_code_permanent_fails_job():
    job = new_job(1)
    job["spec"]["pytorchReplicaSpecs"]["Master"]["restartPolicy"] = "ExitCode"
    pods = [new_pod(job, "Master", 0, "Failed", exit_code=1), new_pod(job, "Worker", 0, "Running")]
    r = reconcile(job, pods, [new_service(job, "Master", 0)])
    assert r["deletePods"] == []
    assert condition(r["status"], "Failed")["reason"] == "PyTorchJobFailed"


@pytest.mark.parametrize("code,retry", [(1, False), (2, False), (126, False), (127, False),
                                        (128, False), (139, False), (130, True), (137, True),
                                        (143, True), (138, True), (3, False), (0, False)])
def test_retryable_exit_codes(code, retry):
    assert opcore().is_retryable_exit_code(code) is retry


# ------------------------------------------------------------- TestStatus
STATUS_CASES = [
    # description, workers, (fW, sW, aW), (fM, sM, aM), restart, expected type
    ("Master is succeeded", 1, (0, 1, 0), (0, 1, 0), False, "Succeeded"),
    ("Master is running", 1, (0, 0, 0), (0, 0, 1), False, "Running"),
    ("Master is failed", 1, (0, 0, 0), (1, 0, 0), False, "Failed"),
    ("Master is running, workers are failed", 4, (4, 0, 0), (0, 0, 1), False, "Running"),
    ("Master is running, workers are succeeded", 4, (0, 4, 0), (0, 0, 1), False, "Running"),
    ("Master is running, a worker is failed", 4, (1, 0, 3), (0, 0, 1), False, "Failed"),
    ("Master is failed, workers are succeeded", 4, (0, 4, 0), (1, 0, 0), False, "Failed"),
    ("Master is succeeded, workers are failed", 4, (4, 0, 0), (0, 1, 0), False, "Succeeded"),
    ("Master is failed and restarting", 4, (4, 0, 0), (1, 0, 0), True, "Restarting"),
]


@pytest.mark.parametrize("case", STATUS_CASES, ids=[c[0] for c in STATUS_CASES])
def test_status(case):
    _, workers, w, m, restart, expected = case
    job = new_job(workers)

    def rs(t):
        f, s, a = t
        return {k: v for k, v in (("failed", f), ("succeeded", s), ("active", a)) if v}
    job["status"] = {"conditions": [], "replicaStatuses": {"Master": rs(m), "Worker": rs(w)}}
    now = int(time.time() * 1000)
    out = json.loads(opcore().update_status_single(json.dumps(job), "Master", 1, restart, now))
    assert out["error"] == ""
    job["status"] = out["status"]
    out = json.loads(opcore().update_status_single(json.dumps(job), "Worker", workers, restart, now))
    st = out["status"]
    assert any(c["type"] == expected for c in st["conditions"])
    # filterOutConditionTest: Running is never True once terminal
    terminal = any(c["type"] in ("Succeeded", "Failed") and c["status"] == "True" for c in st["conditions"])
    if terminal:
        assert not any(c["type"] == "Running" and c["status"] == "True" for c in st["conditions"])


def test_failed_worker_sets_failed_condition():  # TestFailed
    job = new_job(3)
    job["status"] = {"conditions": [], "replicaStatuses": {"Worker": {"failed": 1}}}
    out = json.loads(opcore().update_status_single(json.dumps(job), "Worker", 3, False, 0))
    assert condition(out["status"], "Failed") is not None


def test_running_and_restarting_are_exclusive():
    job = new_job(1)
    job["status"] = {"conditions": [], "replicaStatuses": {"Master": {"active": 1}, "Worker": {"failed": 1}}}
    out = json.loads(opcore().update_status_single(json.dumps(job), "Master", 1, False, 0))
    job["status"] = out["status"]
    assert condition(job["status"], "Running")["status"] == "True"
    out = json.loads(opcore().update_status_single(json.dumps(job), "Worker", 1, True, 0))
    assert condition(out["status"], "Running") is None
    assert condition(out["status"], "Restarting")["status"] == "True"


# ------------------------------------------------------------- job_test.go
@pytest.mark.parametrize("policy,exp_pod_deletes,exp_svc_deletes", [
    ("All", 5, 1), ("None", 0, 0), ("Running", 0, 0)])
def test_delete_pods_and_services(policy, exp_pod_deletes, exp_svc_deletes):
    job = new_job(4, cleanPodPolicy=policy)
    job["status"] = {"conditions": [{"type": "Succeeded", "status": "True", "reason": "PyTorchJobSucceeded",
                                     "lastUpdateTime": "2020-01-01T00:00:00Z",
                                     "lastTransitionTime": "2020-01-01T00:00:00Z"}],
                     "replicaStatuses": {}, "completionTime": "2020-01-01T00:00:00Z"}
    pods = new_pods(job, "Worker", 0, 4) + new_pods(job, "Master", 0, 1)
    r = reconcile(job, pods, [new_service(job, "Master", 0)])
    assert len(r["deletePods"]) == exp_pod_deletes
    assert len(r["deleteServices"]) == exp_svc_deletes


def _finished(job, completion_ms):
    from opfixtures import opcore as oc
    t = oc().format_time(completion_ms)
    job["status"] = {"conditions": [{"type": "Succeeded", "status": "True", "reason": "PyTorchJobSucceeded",
                                     "lastUpdateTime": t, "lastTransitionTime": t}],
                     "replicaStatuses": {}, "completionTime": t}
    return job


@pytest.mark.parametrize("ttl,age_s,expect_delete", [(None, 10, False), (0, 1, True), (2, 3, True),
                                                     (100, 3, False)])
def test_cleanup_pytorchjob_ttl(ttl, age_s, expect_delete):
    extra = {} if ttl is None else {"ttlSecondsAfterFinished": ttl}
    now = int(time.time() * 1000)
    job = _finished(new_job(1, **extra), now - age_s * 1000)
    r = reconcile(job, [], [], now_ms=now)
    assert r["deleteJob"] is expect_delete
    if ttl is not None and not expect_delete:
        assert r["requeueAfter"] and 0 < r["requeueAfter"][0] <= ttl


def test_active_deadline_seconds():
    now = int(time.time() * 1000)
    job = new_job(4, activeDeadlineSeconds=2, cleanPodPolicy="All")
    job["status"] = {"conditions": [], "replicaStatuses": {},
                     "startTime": opcore().format_time(now - 3000)}
    pods = new_pods(job, "Worker", 0, 4) + new_pods(job, "Master", 0, 1)
    r = reconcile(job, pods, [new_service(job, "Master", 0)], now_ms=now)
    assert len(r["deletePods"]) == 5 and len(r["deleteServices"]) == 1
    c = condition(r["status"], "Failed")
    assert c["message"] == f"PyTorchJob {TEST_JOB_NAME} has failed because it was active longer than specified deadline"


def test_active_deadline_requeue_when_start_time_set():
    job = new_job(1, activeDeadlineSeconds=60)
    r = reconcile(job)
    assert "startTime" in r["status"]
    assert 60.0 in r["requeueAfter"]


def test_backoff_for_on_failure():
    job = new_job(4, backoffLimit=4, cleanPodPolicy="All")
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["restartPolicy"] = "OnFailure"
    pods = new_pods(job, "Worker", 0, 4, restart_count=1) + new_pods(job, "Master", 0, 1, restart_count=0)
    r = reconcile(job, pods, [new_service(job, "Master", 0)])
    assert len(r["deletePods"]) == 5 and len(r["deleteServices"]) == 1
    assert condition(r["status"], "Failed")["message"].endswith("reached the specified backoff limit")


def test_backoff_limit_zero_any_restart_fails():
    job = new_job(1, backoffLimit=0)
    pods = [new_pod(job, "Master", 0, "Running"), new_pod(job, "Worker", 0, "Running", restart_count=1)]
    assert opcore().past_backoff_limit(json.dumps(job), json.dumps(pods)) is True


def test_backoff_new_failure_with_requeues():
    job = new_job(2, backoffLimit=1)
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["restartPolicy"] = "Never"
    job["spec"]["pytorchReplicaSpecs"]["Master"]["restartPolicy"] = "Never"
    pods = [new_pod(job, "Master", 0, "Running"), new_pod(job, "Worker", 0, "Running"),
            new_pod(job, "Worker", 1, "Failed")]
    r = reconcile(job, pods, [new_service(job, "Master", 0)], requeues=1)
    assert condition(r["status"], "Failed")["message"].endswith("reached the specified backoff limit")
    r0 = reconcile(job, pods, [new_service(job, "Master", 0)], requeues=0)
    assert "backoff" not in (condition(r0["status"], "Failed") or {}).get("message", "")


def test_copy_labels_and_annotations():
    job = new_job(1)
    tmpl = job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]
    tmpl["metadata"] = {"labels": {"label1": "1"}, "annotations": {"annotation1": "1"}}
    r = reconcile(job)
    w = [p for p in r["createPods"] if "worker" in p["metadata"]["name"]][0]
    assert w["metadata"]["labels"]["label1"] == "1"
    assert w["metadata"]["annotations"]["annotation1"] == "1"


def test_succeeded_moves_active_to_succeeded():
    job = new_job(1)
    job["status"] = {"conditions": [{"type": "Succeeded", "status": "True", "reason": "x",
                                     "lastUpdateTime": "2020-01-01T00:00:00Z",
                                     "lastTransitionTime": "2020-01-01T00:00:00Z"}],
                     "replicaStatuses": {"Worker": {"active": 1}, "Master": {"succeeded": 1}}}
    r = reconcile(job)
    assert r["status"]["replicaStatuses"]["Worker"] == {"succeeded": 1}
    assert r["statusChanged"] is True


# ------------------------------------------------------------- job added / update
def test_add_job_sets_created_condition():
    job = new_job(1)
    out = json.loads(opcore().on_job_added(json.dumps(job), 0))
    assert out["valid"] and out["metrics"]["created"] == 1
    c = condition(out["status"], "Created")
    assert c["reason"] == "PyTorchJobCreated" and c["message"] == f"PyTorchJob {TEST_JOB_NAME} is created."


def test_add_invalid_job_fails_with_invalid_spec():
    job = new_job(1)
    del job["spec"]["pytorchReplicaSpecs"]["Master"]
    out = json.loads(opcore().on_job_added(json.dumps(job), 0))
    assert not out["valid"]
    c = condition(out["status"], "Failed")
    assert c["reason"] == "InvalidPyTorchJobSpec"
    assert "Master ReplicaSpec must be present" in c["message"]


def test_deadline_requeue_on_update():
    old = new_job(1, activeDeadlineSeconds=100)
    cur = new_job(1, activeDeadlineSeconds=10)
    now = int(time.time() * 1000)
    cur["status"] = {"startTime": opcore().format_time(now - 4000)}
    d = opcore().deadline_requeue_on_update(json.dumps(old), json.dumps(cur), now)
    assert 5.0 <= d <= 6.5
    assert opcore().deadline_requeue_on_update(json.dumps(cur), json.dumps(cur), now) < 0


# ------------------------------------------------------------- gang scheduling
def test_gang_scheduling_podgroup_and_scheduler_name():
    job = new_job(2)
    cfg = {"enableGangScheduling": True, "gangSchedulerName": "volcano"}
    r = reconcile(job, config=cfg)
    pg = r["createPodGroup"]
    assert pg["spec"]["minMember"] == 3 and pg["metadata"]["name"] == TEST_JOB_NAME
    for p in r["createPods"]:
        assert p["spec"]["schedulerName"] == "volcano"
        assert p["metadata"]["annotations"]["scheduling.k8s.io/group-name"] == TEST_JOB_NAME
    r2 = reconcile(job, config=cfg, podgroup_exists=True)
    assert r2["createPodGroup"] is None


def test_gang_scheduling_volcano_podgroup_api():
    """--gang-podgroup-api volcano: the PodGroup is scheduling.volcano.sh/v1beta1 (what Volcano
    >= 1.0 reads) with minMember = all replicas and the default queue; pods carry the same
    group-name annotation and scheduler name; kube-batch v1alpha1 stays the default."""
    job = new_job(3)
    r = reconcile(job, config={"enableGangScheduling": True, "gangPodgroupApi": "volcano"})
    pg = r["createPodGroup"]
    assert pg["apiVersion"] == "scheduling.volcano.sh/v1beta1" and pg["kind"] == "PodGroup"
    assert pg["spec"] == {"minMember": 4, "queue": "default"}
    assert pg["metadata"]["ownerReferences"][0]["kind"] == "PyTorchJob"
    for p in r["createPods"]:
        assert p["spec"]["schedulerName"] == "volcano"
        assert p["metadata"]["annotations"]["scheduling.k8s.io/group-name"] == TEST_JOB_NAME
    dflt = reconcile(job, config={"enableGangScheduling": True})["createPodGroup"]
    assert dflt["apiVersion"] == "scheduling.incubator.k8s.io/v1alpha1" and "queue" not in dflt["spec"]


def test_gang_scheduling_other_scheduler_warns():
    job = new_job(1)
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["schedulerName"] = "other"
    r = reconcile(job, config={"enableGangScheduling": True})
    assert any(e["reason"] == "SettedPodTemplateSchedulerName" for e in r["events"])


# ------------------------------------------------------------- util_test.go
def test_gen_owner_reference_and_labels():
    job = new_job(1)
    ref = json.loads(opcore().gen_owner_reference(json.dumps(job)))
    assert ref == {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "name": TEST_JOB_NAME,
                   "uid": job["metadata"]["uid"], "controller": True, "blockOwnerDeletion": True}
    assert labels("a/b") == {"group-name": "kubeflow.org", "job-name": "a-b",
                             "pytorch-job-name": "a-b", "controller-name": "pytorch-operator"}


def test_get_init_container_custom_template():
    tmpl = "- name: init\n  image: {{.InitContainerImage}}\n  command: ['echo', '{{.MasterAddr}}']\n"
    out = json.loads(opcore().init_containers("m-0", json.dumps(
        {"initContainerTemplate": tmpl, "initContainerImage": "busybox"})))
    assert out == [{"name": "init", "image": "busybox", "command": ["echo", "m-0"]}]


def test_rccl_env_injection_extension():
    job = new_job(1)
    pod = json.loads(opcore().build_pod(json.dumps(job), "Worker", 0, json.dumps({"injectRcclEnv": True})))
    env = env_of(pod)
    assert env["LOCAL_RANK"] == "0" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # device-memory kernel arguments pinned in the pod (bench.py pins the same; +8.3 us/step
    # with host-memory kernargs, profiles/r5_env/ab.txt)
    assert env["HIP_FORCE_DEV_KERNARG"] == "1"
    assert "NCCL_MIN_NCHANNELS" not in env  # unmeasured tuning is not injected by default
    pod = json.loads(opcore().build_pod(json.dumps(job), "Worker", 0))
    assert "LOCAL_RANK" not in env_of(pod)
    # --rccl-env replaces the set; a value the template already sets wins
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]["env"] = [
        {"name": "NCCL_PROTO", "value": "Simple"}]
    cfg = {"injectRcclEnv": True, "rcclEnv": {"NCCL_PROTO": "LL128", "NCCL_ALGO": "Ring"}}
    env = env_of(json.loads(opcore().build_pod(json.dumps(job), "Worker", 0, json.dumps(cfg))))
    assert env["NCCL_PROTO"] == "Simple" and env["NCCL_ALGO"] == "Ring"
    assert "HSA_ENABLE_IPC_MODE_LEGACY" not in env
    assert env["HIP_FORCE_DEV_KERNARG"] == "1"  # not part of the replaceable RCCL set
    # a template that chooses host-memory kernel arguments keeps its choice
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]["env"] = [
        {"name": "HIP_FORCE_DEV_KERNARG", "value": "0"}]
    env = env_of(json.loads(opcore().build_pod(json.dumps(job), "Worker", 0, json.dumps(cfg))))
    assert env["HIP_FORCE_DEV_KERNARG"] == "0"


def _gpu_job(n_workers):
    job = new_job(n_workers)
    for rs in job["spec"]["pytorchReplicaSpecs"].values():
        rs["template"]["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": 1}}
    return job


def test_xgmi_pod_topology_fields():
    """--xgmi-pod-topology (docs/xgmi_pods.md): what one-GPU pods on one node need for
    peer memory over xGMI -- host PID namespace (dmabuf IPC import opens the exporter's
    /proc/<pid>/fd/<fd>), host IPC namespace + /dev/shm (RCCL SHM transport), RCCL's host
    identity from the node name, and all pods of the job on one node."""
    job = _gpu_job(7)
    cfg = json.dumps({"injectRcclEnv": True, "xgmiPodTopology": True})
    for rt, idx in (("Master", 0), ("Worker", 6)):
        pod = json.loads(opcore().build_pod(json.dumps(job), rt, idx, cfg))
        spec = pod["spec"]
        assert spec["hostPID"] is True and spec["hostIPC"] is True
        term = spec["affinity"]["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][0]
        assert term["topologyKey"] == "kubernetes.io/hostname"
        assert term["labelSelector"]["matchLabels"] == {"job-name": job["metadata"]["name"]}
        c = [c for c in spec["containers"] if c["name"] == "pytorch"][0]
        hid = [e for e in c["env"] if e["name"] == "NCCL_HOSTID"]
        assert hid == [{"name": "NCCL_HOSTID", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}}]
        env = env_of(pod)
        assert env["LOCAL_RANK"] == "0" and env["WORLD_SIZE"] == "8"
    # CPU pods (no amd.com/gpu) and the flag off: untouched
    pod = json.loads(opcore().build_pod(json.dumps(new_job(1)), "Worker", 0, cfg))
    assert "hostPID" not in pod["spec"] and "affinity" not in pod["spec"]
    pod = json.loads(opcore().build_pod(json.dumps(_gpu_job(1)), "Worker", 0))
    assert "hostPID" not in pod["spec"]
    # a template that decides for itself keeps its choice
    job = _gpu_job(1)
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["hostPID"] = False
    pod = json.loads(opcore().build_pod(json.dumps(job), "Worker", 0, cfg))
    assert pod["spec"]["hostPID"] is False and pod["spec"]["hostIPC"] is True


def test_operator_flags_for_xgmi_topology():
    bin_ = operator_binary()
    r = subprocess.run([bin_, "--rccl-env", "NOVALUE", "--version"], capture_output=True, text=True)
    assert r.returncode != 0 and "KEY=VALUE" in (r.stderr + r.stdout)
    r = subprocess.run([bin_, "--xgmi-pod-topology", "--rccl-env", "NCCL_PROTO=LL128", "--version"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


# ------------------------------------------------------------- defaults / validation
def test_defaults():
    raw = {"metadata": {"name": "x"}, "spec": {"pytorchReplicaSpecs": {
        "master": {"template": {"spec": {"containers": [{"name": "pytorch", "image": "i"}]}}},
        "WORKER": {"replicas": 3, "template": {"spec": {"containers": [
            {"name": "side", "image": "s"}, {"name": "pytorch", "image": "i"}]}}}}}}
    d = json.loads(opcore().set_defaults(json.dumps(raw)))
    specs = d["spec"]["pytorchReplicaSpecs"]
    assert set(specs) == {"Master", "Worker"}
    assert d["spec"]["cleanPodPolicy"] == "None"
    assert specs["Master"]["replicas"] == 1 and specs["Master"]["restartPolicy"] == "OnFailure"
    assert specs["Master"]["template"]["spec"]["containers"][0]["ports"] == [
        {"name": "pytorchjob-port", "containerPort": 23456}]
    assert "ports" not in specs["Worker"]["template"]["spec"]["containers"][1]  # only Master gets the port


def _c(name="pytorch", image="img"):
    return {"name": name, "image": image}


@pytest.mark.parametrize("spec,msg", [
    ({"pytorchReplicaSpecs": None}, "PyTorchJobSpec is not valid"),
    ({"pytorchReplicaSpecs": {"Worker": {"template": {"spec": {"containers": []}}}}},
     "containers definition expected in Worker"),
    ({"pytorchReplicaSpecs": {"Worker": {"template": {"spec": {"containers": [_c(image="")]}}}}},
     "Image is undefined in the container of Worker"),
    ({"pytorchReplicaSpecs": {"Worker": {"template": {"spec": {"containers": [_c(name="")]}}}}},
     "There is no container named pytorch in Worker"),
    ({"pytorchReplicaSpecs": {"Master": {"replicas": 2, "template": {"spec": {"containers": [_c()]}}}}},
     "There must be only 1 master replica"),
    ({"pytorchReplicaSpecs": {"Worker": {"replicas": 1, "template": {"spec": {"containers": [_c()]}}}}},
     "Master ReplicaSpec must be present"),
    ({"pytorchReplicaSpecs": {"Chief": {"template": {"spec": {"containers": [_c()]}}}}},
     "PyTorchReplicaType is Chief but must be one of [Master Worker]"),
])
def test_validate_invalid_specs(spec, msg):
    err = opcore().validate_spec(json.dumps(spec))
    assert msg in err


def test_validate_valid_spec():
    spec = {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "template": {"spec": {"containers": [_c()]}}},
                                    "Worker": {"replicas": 3, "template": {"spec": {"containers": [_c()]}}}}}
    assert opcore().validate_spec(json.dumps(spec)) == ""


# ------------------------------------------------------------- primitives
def test_expectations_semantics():
    e = opcore().Expectations(ttl_s=0.2)
    assert e.satisfied("k")
    e.expect_creations("k", 2)
    assert not e.satisfied("k")
    e.creation_observed("k")
    assert not e.satisfied("k")
    e.creation_observed("k")
    assert e.satisfied("k")
    e.expect_creations("k", 1)
    time.sleep(0.25)
    assert e.satisfied("k")  # expired


def test_workqueue_dedup_and_processing():
    q = opcore().WorkQueue()
    q.add("a")
    q.add("a")
    assert q.len() == 1
    assert q.get(0.1) == "a"
    q.add("a")           # re-added while processing: parked until done()
    assert q.get(0.05) is None
    q.done("a")
    assert q.get(0.1) == "a"
    q.done("a")


def test_workqueue_rate_limit_backoff():
    q = opcore().WorkQueue(base_delay_s=0.01)
    assert q.num_requeues("x") == 0
    d1, d2, d3 = q.when("x"), q.when("x"), q.when("x")
    assert d1 == pytest.approx(0.01) and d2 == pytest.approx(0.02) and d3 == pytest.approx(0.04)
    assert q.num_requeues("x") == 3
    q.forget("x")
    assert q.num_requeues("x") == 0
    t = time.time()
    q.add_after("y", 0.05)
    assert q.get(1.0) == "y"
    assert time.time() - t >= 0.045


def test_json_and_yaml_roundtrip():
    s = '{"a":[1,2.5,"x\\u00e9\\n"],"b":{"c":null,"d":true}}'
    assert json.loads(opcore().json_roundtrip(s)) == json.loads(s)
    y = "a: 1\nb:\n  - x\n  - {k: v}\nc: 'q''s'\nd: [1, \"two\"]\n"
    assert json.loads(opcore().yaml_to_json(y)) == {"a": 1, "b": ["x", {"k": "v"}], "c": "q's", "d": [1, "two"]}
    assert opcore().parse_time("2019-11-07T09:21:44Z") == 1573118504000
    assert opcore().format_time(1573118504000) == "2019-11-07T09:21:44Z"
