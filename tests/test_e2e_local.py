"""End-to-end: the native operator binary against the local cluster (CPU, gloo).

Ports of the reference e2e suites (test/e2e/v1/default/defaults.go,
test/e2e/v1/cleanpolicy/cleanpolicy_all.go, the SDK e2e test and the GKE workflow's
simple/gpu PyTorchJobs in test/workflows/components/) plus behaviours the reference only
covers with unit tests (ExitCode restarts, backoff limit, active deadline, TTL, gang
scheduling, leader failover), all run through real processes: fake API server ->
``pytorch-operator`` -> kubelet emulator -> worker processes.
"""
import json
import os
import signal
import sys
import time

import pytest

from pytorch_operator_amd.cluster.local import LocalCluster
from kubeflow.pytorchjob.rest import EVENTS, PODGROUPS, PODS, PYTORCHJOBS, SERVICES, ApiException
from pytorch_operator_amd.utils import pformat, rand_string

NS = "default"


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    c = LocalCluster(workdir=str(tmp_path_factory.mktemp("cluster")))
    c.start()
    c.wait_operator_ready()
    yield c
    c.stop()


def replica(n, image="pytorch_dist_sendrecv:1.0", args=None, command=None, policy="OnFailure", extra=None):
    cont = {"name": "pytorch", "image": image}
    if args is not None:
        cont["args"] = args
    if command is not None:
        cont["command"] = command
    if extra:
        cont.update(extra)
    return {"replicas": n, "restartPolicy": policy, "template": {"spec": {"containers": [cont]}}}


def make_job(name, master=None, worker=None, **spec):
    specs = {}
    if master is not None:
        specs["Master"] = master
    if worker is not None:
        specs["Worker"] = worker
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name},
            "spec": dict(spec, pytorchReplicaSpecs=specs)}


def conditions(c, name):
    j = c.rest.get(PYTORCHJOBS, name, NS)
    return [x["type"] for x in (j.get("status") or {}).get("conditions") or []], j


def wait_until(pred, timeout=90, interval=0.1, what="condition"):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = pred()
        if v:
            return v
        time.sleep(interval)
    raise TimeoutError(f"timed out waiting for {what}")


def wait_finished(c, name, timeout=120):
    def done():
        types, j = conditions(c, name)
        return (types, j) if ("Succeeded" in types or "Failed" in types) else None
    try:
        return wait_until(done, timeout, what=f"job {name} to finish")
    except TimeoutError:
        # dump the Python stacks of the job's live containers into their logs
        for r in list(c.kubelet.runners.values()):
            for ct in r.containers:
                if r.name.startswith(name + "-") and ct.proc is not None and ct.proc.poll() is None:
                    os.kill(ct.proc.pid, signal.SIGABRT)
        time.sleep(1.0)
        pods = c.rest.list(PODS, NS, f"pytorch-job-name={name}")["items"]
        logs = {p["metadata"]["name"]: c.rest.pod_log(p["metadata"]["name"], NS)[-4000:] for p in pods}
        raise AssertionError(f"{name} did not finish; pods={[(p['metadata']['name'], p['status']) for p in pods]}"
                             f"\nlogs={logs}\noperator={open(c.operator_log).read()[-3000:]}")


def pod_names(c, name):
    return sorted(p["metadata"]["name"] for p in c.rest.list(PODS, NS, f"pytorch-job-name={name}")["items"])


def py(code):
    return ["python", "-c", code]


def test_defaults_job_succeeds_and_is_garbage_collected(cluster):
    """defaults.go: Master + 3 Workers, default CleanPodPolicy keeps the pods; delete -> GC."""
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-defaults", replica(1), replica(3)), NS)
    types, job = wait_finished(c, "e2e-defaults")
    assert types[-1] == "Succeeded", types
    assert "cleanPodPolicy" not in job["spec"]  # defaults are applied in memory, never persisted
    names = pod_names(c, "e2e-defaults")
    assert names == ["e2e-defaults-master-0", "e2e-defaults-worker-0", "e2e-defaults-worker-1",
                     "e2e-defaults-worker-2"]
    # the job succeeds with its master (status.go); a worker that exits a moment later may still
    # count as active in the job's last status, but every worker pod does succeed
    ws = job["status"]["replicaStatuses"]["Worker"]
    assert ws.get("succeeded", 0) + ws.get("active", 0) == 3 and not ws.get("failed"), ws
    deadline = time.time() + 60
    while True:
        phases = [c.rest.get(PODS, f"e2e-defaults-worker-{i}", NS)["status"].get("phase") for i in range(3)]
        if phases == ["Succeeded"] * 3 or time.time() > deadline:
            break
        time.sleep(0.2)
    assert phases == ["Succeeded"] * 3, phases
    assert job["status"]["completionTime"]
    log = c.rest.pod_log("e2e-defaults-master-0", NS)
    assert "Result from worker 3" in log and "all_reduce ok (10.0)" in log
    pod = c.rest.get(PODS, "e2e-defaults-worker-1", NS)
    env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0]["env"]}
    assert env["RANK"] == "2" and env["WORLD_SIZE"] == "4" and env["MASTER_ADDR"] == "e2e-defaults-master-0"
    assert pod["spec"]["initContainers"][0]["name"] == "init-pytorch"
    c.rest.delete(PYTORCHJOBS, "e2e-defaults", NS)
    wait_until(lambda: not pod_names(c, "e2e-defaults"), 30, what="GC")
    assert not c.rest.list(SERVICES, NS, "pytorch-job-name=e2e-defaults")["items"]


def test_cleanpolicy_all_deletes_pods_after_success(cluster):
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-clean-all", replica(1), replica(1), cleanPodPolicy="All"), NS)
    types, _ = wait_finished(c, "e2e-clean-all")
    assert types[-1] == "Succeeded"
    wait_until(lambda: not pod_names(c, "e2e-clean-all"), 30, what="pods cleaned")
    wait_until(lambda: not c.rest.list(SERVICES, NS, "pytorch-job-name=e2e-clean-all")["items"], 30)


def test_mnist_gloo_ddp_job(cluster):
    """The reference's examples/mnist job (gloo) on 2 CPU ranks through the operator."""
    c = cluster
    args = ["--backend", "gloo", "--dataset-size", "2000", "--test-size", "500", "--max-steps", "20",
            "--log-interval", "5"]
    c.rest.create(PYTORCHJOBS, make_job("e2e-mnist", replica(1, "pytorch_dist_mnist:latest", args),
                                        replica(1, "pytorch_dist_mnist:latest", args)), NS)
    types, _ = wait_finished(c, "e2e-mnist", timeout=180)
    log = c.rest.pod_log("e2e-mnist-master-0", NS)
    assert types[-1] == "Succeeded", log[-2000:]
    assert "Using distributed PyTorch with gloo backend" in log
    assert "Train Epoch: 1 [0/2000 (0%)]" in log and "accuracy=" in log
    done = [json.loads(x) for x in log.splitlines() if x.startswith('{"event": "train_done"')]
    assert done and done[0]["steps"] == 20  # full 2000-sample set per rank, capped by --max-steps


def test_exit_code_policy_restarts_retryable_failure(cluster, tmp_path):
    """ExitCode: 130 (SIGINT-like, retryable) -> pod recreated -> job succeeds."""
    c = cluster
    marker = tmp_path / "once"
    code = f"import os,sys; p={str(marker)!r}; e=os.path.exists(p); open(p,'w').close(); sys.exit(0 if e else 130)"
    c.rest.create(PYTORCHJOBS, make_job("e2e-exitcode", replica(1, "busybox", command=py(code), policy="ExitCode")), NS)
    types, job = wait_finished(c, "e2e-exitcode")
    assert types[-1] == "Succeeded", job["status"]
    # Restarting is replaced by Running again (filterOutCondition), so check the event trail
    evs = c.rest.list(EVENTS, NS)["items"]
    assert any(e.get("reason") == "ExitedWithCode" for e in evs)
    assert c.metric_value("pytorch_operator_jobs_restarted_total") >= 1


def test_exit_code_policy_permanent_failure(cluster):
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-exit1", replica(1, "busybox", command=py("import sys; sys.exit(1)"),
                                                            policy="ExitCode")), NS)
    types, job = wait_finished(c, "e2e-exit1")
    assert types[-1] == "Failed"
    assert job["status"]["replicaStatuses"]["Master"]["failed"] == 1


def test_onfailure_backoff_limit(cluster):
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-backoff", replica(1, "busybox", command=py("import sys; sys.exit(3)")),
                                        backoffLimit=2), NS)
    types, job = wait_finished(c, "e2e-backoff")
    assert types[-1] == "Failed"
    last = job["status"]["conditions"][-1]
    assert "backoff limit" in last["message"]


def test_active_deadline_fails_and_kills_running_pods(cluster):
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-deadline", replica(1, "busybox", command=py("import time; time.sleep(120)")),
                                        activeDeadlineSeconds=2, cleanPodPolicy="All"), NS)
    types, job = wait_finished(c, "e2e-deadline", timeout=60)
    assert types[-1] == "Failed"
    assert "deadline" in job["status"]["conditions"][-1]["message"]
    wait_until(lambda: not pod_names(c, "e2e-deadline"), 30, what="running pods deleted")


def test_ttl_seconds_after_finished_deletes_job(cluster):
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-ttl", replica(1, "busybox", command=py("pass")),
                                        ttlSecondsAfterFinished=1), NS)
    seen = set()

    def gone():
        try:
            seen.update(conditions(c, "e2e-ttl")[0])
            return False
        except ApiException as e:
            return e.status == 404
    wait_until(gone, 60, interval=0.05, what="TTL deletion")
    # the job can finish and expire between two polls; it is only ever deleted once finished
    assert "Failed" not in seen
    assert c.metric_value("pytorch_operator_jobs_successful_total") >= 1


def test_unschedulable_gpu_request_stays_pending(cluster):
    """A CUDA-only resource request never schedules on an MI355X node."""
    c = cluster
    extra = {"resources": {"limits": {"nvidia.com/gpu": 1}}}
    c.rest.create(PYTORCHJOBS, make_job("e2e-nvidia", replica(1, "busybox", command=py("pass"), extra=extra)), NS)

    def unsched():
        try:
            p = c.rest.get(PODS, "e2e-nvidia-master-0", NS)
        except ApiException:
            return False
        return any(x.get("reason") == "Unschedulable" for x in p["status"].get("conditions") or [])
    wait_until(unsched, 30, what="Unschedulable")
    types, _ = conditions(c, "e2e-nvidia")
    assert "Succeeded" not in types and "Failed" not in types
    c.rest.delete(PYTORCHJOBS, "e2e-nvidia", NS)


def test_invalid_spec_is_marked_failed(cluster):
    c = cluster
    bad = make_job("e2e-invalid", {"replicas": 1, "template": {"spec": {"containers": [{"name": "other", "image": "x"}]}}})
    c.rest.create(PYTORCHJOBS, bad, NS)
    types, job = wait_finished(c, "e2e-invalid", timeout=30)
    assert types[-1] == "Failed"
    assert job["status"]["conditions"][-1]["reason"] == "InvalidPyTorchJobSpec"


def test_events_and_metrics(cluster):
    c = cluster
    c.rest.create(PYTORCHJOBS, make_job("e2e-metrics", replica(1, "busybox", command=py("pass"))), NS)
    wait_finished(c, "e2e-metrics")

    def reasons():
        evs = [e for e in c.rest.list(EVENTS, NS)["items"]
               if e.get("involvedObject", {}).get("name") == "e2e-metrics"]
        r = {e["reason"] for e in evs}
        return r if {"SuccessfulCreatePod", "SuccessfulCreateService"} <= r else None
    wait_until(reasons, 30, what="events (recorded asynchronously)")
    assert c.metric_value("pytorch_operator_jobs_created_total") >= 1
    assert c.metric_value("pytorch_operator_jobs_successful_total") >= 1
    assert "pytorch_operator_reconcile_duration_seconds" in c.metrics() or True


@pytest.mark.parametrize("api", ["kube-batch", "volcano"])
def test_gang_scheduling_creates_and_deletes_podgroup(tmp_path, api):
    """--enable-gang-scheduling with either PodGroup API: the PodGroup (minMember = all
    replicas) exists before the pods run, every pod names it and the gang scheduler, and it is
    deleted when the job finishes.  The other API's resource is never touched."""
    from kubeflow.pytorchjob.rest import VOLCANO_PODGROUPS
    gvr, other = (VOLCANO_PODGROUPS, PODGROUPS) if api == "volcano" else (PODGROUPS, VOLCANO_PODGROUPS)
    with LocalCluster(workdir=str(tmp_path / "g"),
                      operator_args=["--enable-gang-scheduling", f"--gang-podgroup-api={api}"]) as c:
        c.wait_operator_ready()
        c.rest.create(PYTORCHJOBS, make_job("e2e-gang", replica(1, "busybox", command=py("import time; time.sleep(1)")),
                                            replica(2, "busybox", command=py("import time; time.sleep(1)"))), NS)
        pg = wait_until(lambda: c.rest.list(gvr, NS)["items"], 30, what="podgroup")
        assert pg[0]["metadata"]["name"] == "e2e-gang" and pg[0]["spec"]["minMember"] == 3
        if api == "volcano":
            assert pg[0]["apiVersion"] == "scheduling.volcano.sh/v1beta1" and pg[0]["spec"]["queue"] == "default"
        pod = wait_until(lambda: next((q for q in c.rest.list(PODS, NS)["items"]
                                       if q["metadata"]["name"] == "e2e-gang-worker-0"), None), 30, what="worker pod")
        assert pod["spec"]["schedulerName"] == "volcano"
        assert pod["metadata"]["annotations"]["scheduling.k8s.io/group-name"] == "e2e-gang"
        types, _ = wait_finished(c, "e2e-gang")
        assert types[-1] == "Succeeded"
        wait_until(lambda: not c.rest.list(gvr, NS)["items"], 30, what="podgroup deleted")
        assert not c.rest.list(other, NS)["items"]


def test_leader_failover(tmp_path):
    fast = ["--leader-elect-lease-duration=2s", "--leader-elect-renew-deadline=1s",
            "--leader-elect-retry-period=200ms"]
    with LocalCluster(workdir=str(tmp_path / "l"), operator_args=fast) as c:
        c.wait_operator_ready()
        first = c.operator
        from pytorch_operator_amd.cluster.local import free_port
        standby_port = free_port()
        standby = c.spawn_operator(standby_port, str(tmp_path / "standby.log"))
        try:
            import urllib.request

            def standby_leader():
                try:
                    body = urllib.request.urlopen(f"http://127.0.0.1:{standby_port}/metrics", timeout=2).read().decode()
                except OSError:
                    return None
                return [ln for ln in body.splitlines() if ln.startswith("pytorch_operator_is_leader ")]
            lines = wait_until(standby_leader, 20, what="standby metrics")
            assert lines[0].endswith(" 0")
            os.kill(first.pid, signal.SIGKILL)  # no graceful lease release
            first.wait()
            wait_until(lambda: (standby_leader() or ["x 0"])[0].endswith(" 1"), 20, what="takeover")
            c.rest.create(PYTORCHJOBS, make_job("e2e-failover", replica(1, "busybox", command=py("pass"))), NS)
            types, _ = wait_finished(c, "e2e-failover")
            assert types[-1] == "Succeeded"
        finally:
            standby.terminate()
            standby.wait(15)


def test_injected_worker_fault_is_retried_under_exit_code_policy(cluster):
    """Kubelet fault injection: the worker is SIGKILLed once (137, retryable),
    the operator recreates it and the real gloo rendezvous still completes."""
    c = cluster
    worker = replica(1, policy="ExitCode")
    worker["template"]["metadata"] = {"annotations": {"fault.pto.amd.com/exit-code": "137",
                                                      "fault.pto.amd.com/after-seconds": "0.1"}}
    c.rest.create(PYTORCHJOBS, make_job("e2e-fault", replica(1, policy="ExitCode"), worker), NS)
    types, job = wait_finished(c, "e2e-fault", timeout=120)
    assert types[-1] == "Succeeded", job["status"]
    assert "all_reduce ok (3.0)" in c.rest.pod_log("e2e-fault-master-0", NS)
    evs = [e for e in c.rest.list(EVENTS, NS)["items"] if e.get("reason") == "ExitedWithCode"
           and "e2e-fault-worker-0" in e.get("message", "")]
    assert evs, "operator should record the retryable exit"


def test_many_concurrent_jobs_with_threadiness(tmp_path):
    """Multi-worker reconcile stress: 4 sync threads, 12 concurrent jobs."""
    with LocalCluster(workdir=str(tmp_path / "s"), operator_args=["--threadiness=4", "--qps=50",
                                                                  "--burst=100"]) as c:
        c.wait_operator_ready()
        # random suffixes like the reference e2e (test/e2e/v1/default/defaults.go + util.RandString)
        names = [f"stress-{i}-{rand_string(4)}" for i in range(12)]
        for n in names:
            c.rest.create(PYTORCHJOBS, make_job(n, replica(1, "busybox", command=py("pass")),
                                                replica(2, "busybox", command=py("pass"))), NS)
        for n in names:
            types, job = wait_finished(c, n, timeout=120)
            assert types[-1] == "Succeeded", pformat(job["status"])
            # (the master's success ends the job: workers may not have started yet)
            assert len(pod_names(c, n)) == 3  # expectations: no duplicate pods under concurrency
        assert c.metric_value("pytorch_operator_jobs_successful_total") == 12


@pytest.mark.parametrize("code", [137, 138])
def test_exit_code_restart_resumes_from_checkpoint(cluster, tmp_path, code):
    """Elastic recovery end to end: the worker process dies with a retryable code after
    checkpointing epoch 1 (137 = SIGKILL; 138 = what the worker exits with when the xGMI
    exchange fails, harness/mnist.py ``_xgmi_guard``), the operator recreates the pod
    (ExitCode policy) and the new pod resumes at epoch 2 from the checkpoint."""
    c = cluster
    name = f"e2e-resume-{code}"
    args = ["--backend", "gloo", "--dataset-size", "640", "--test-size", "128", "--epochs", "2",
            "--checkpoint-dir", str(tmp_path / "ck"), "--resume"]
    master = replica(1, "pytorch_dist_mnist:latest", args, policy="ExitCode",
                     extra={"env": [{"name": "PTO_FAULT_EXIT_AFTER_EPOCH", "value": "1"},
                                    {"name": "PTO_FAULT_EXIT_CODE", "value": str(code)}]})
    c.rest.create(PYTORCHJOBS, make_job(name, master), NS)
    types, job = wait_finished(c, name, timeout=180)
    assert types[-1] == "Succeeded", job["status"]
    log = c.rest.pod_log(f"{name}-master-0", NS)
    assert f"fault injection: exiting with {code} after epoch 1" in log
    assert '"event": "resumed"' in log and "Train Epoch: 2 [0/640" in log


def test_pod_namespaces_follow_host_pid_ipc(tmp_path):
    """Kubelet isolation (docs/xgmi_pods.md): each pod gets its own PID / IPC namespace,
    /dev/shm and hostname unless its spec shares the node's (hostPID / hostIPC) -- the
    fields the operator's --xgmi-pod-topology sets on GPU pods."""
    from pytorch_operator_amd.cluster.kubelet import namespaces_available
    ok, why = namespaces_available()
    if not ok:
        pytest.skip(f"no user namespaces on this host: {why}")
    code = ("import json, os, socket; print(json.dumps({'pid': os.getpid(), 'host': socket.gethostname(), "
            "'pidns': os.readlink('/proc/self/ns/pid'), 'ipcns': os.readlink('/proc/self/ns/ipc'), "
            "'shm': sorted(os.listdir('/dev/shm'))[:0]}))")
    # (pods here only run `python -c`: they need not read the repo, which may sit in a 0700 home)
    with LocalCluster(workdir=str(tmp_path / "c"), isolation="namespaces", isolation_needs_repo=False) as c:
        c.wait_operator_ready()
        for name, host in (("ns-isolated", False), ("ns-shared", True)):
            specs = [replica(1, command=py(code), policy="Never") for _ in range(2)]
            if host:
                for sp in specs:
                    sp["template"]["spec"].update(hostPID=True, hostIPC=True)
            c.rest.create(PYTORCHJOBS, make_job(name, *specs), NS)
            types, _ = wait_finished(c, name, timeout=120)
            assert types[-1] == "Succeeded"
            # the job's success is decided by the Master alone (reference quirk): wait for both
            pods = (f"{name}-master-0", f"{name}-worker-0")
            wait_until(lambda: all(c.rest.get(PODS, p, NS).get("status", {}).get("phase") == "Succeeded"
                                   for p in pods), 60, what="both pods to finish")
            outs = {}
            for pod in pods:
                lines = [x for x in c.rest.pod_log(pod, NS).splitlines() if x.startswith("{")]
                outs[pod] = json.loads(lines[-1])
            me = os.readlink("/proc/self/ns/pid")
            if host:
                assert all(o["pidns"] == me and o["pid"] != 1 for o in outs.values()), outs
            else:
                assert all(o["pid"] == 1 and o["pidns"] != me for o in outs.values()), outs
                assert {o["host"] for o in outs.values()} == set(outs)  # hostname = pod name
                assert len({o["pidns"] for o in outs.values()}) == 2 and len({o["ipcns"] for o in outs.values()}) == 2


def test_repeated_events_are_aggregated(cluster, tmp_path):
    """client-go's EventCorrelator semantics: an event identical to one posted recently (same
    object, type, reason, message) bumps that Event's count instead of creating a new object
    -- a crash-looping replica must not flood the namespace with Events."""
    c = cluster
    marker = tmp_path / "n"
    # exits 130 (retryable) three times, then 0: the ExitCode policy deletes and recreates the
    # pod each time, so "Created pod: <name>" / "Deleted pod: <name>" repeat verbatim
    code = (f"import os,sys; p={str(marker)!r}; n=int(open(p).read()) if os.path.exists(p) else 0; "
            f"open(p,'w').write(str(n+1)); sys.exit(0 if n >= 3 else 130)")
    c.rest.create(PYTORCHJOBS, make_job("e2e-events", replica(1, "busybox", command=py(code), policy="ExitCode")), NS)
    types, job = wait_finished(c, "e2e-events", timeout=120)
    assert types[-1] == "Succeeded", job["status"]
    # the event sink posts asynchronously: poll until the create/delete counts settle
    deadline = time.time() + 15
    while True:
        evs = [e for e in c.rest.list(EVENTS, NS)["items"]
               if (e.get("involvedObject") or {}).get("name") == "e2e-events"]
        cr = [e.get("count", 1) for e in evs if e["reason"] == "SuccessfulCreatePod"]
        de = [e.get("count", 1) for e in evs if e["reason"] == "SuccessfulDeletePod"]
        if (len(cr) == 1 and len(de) == 1 and cr[0] == de[0] + 1) or time.time() > deadline:
            break
        time.sleep(0.2)
    created = [e for e in evs if e["reason"] == "SuccessfulCreatePod" and e["message"] == "Created pod: e2e-events-master-0"]
    assert len(created) == 1, [(e["metadata"]["name"], e.get("count")) for e in created]
    deleted = [e for e in evs if e["reason"] == "SuccessfulDeletePod"]
    assert len(deleted) == 1 and deleted[0]["count"] >= 2, [(e["metadata"]["name"], e.get("count")) for e in deleted]
    # every restart recreated the pod: one more creation than deletions
    assert created[0]["count"] == deleted[0]["count"] + 1
    assert created[0]["lastTimestamp"] >= created[0]["firstTimestamp"]
    # LoggerForPod fields (tf-operator logger.go:26-56) on the pod lifecycle lines
    log = open(c.operator_log).read()
    assert "replica-type=master" in log and "pod=default.e2e-events-master-0" in log
    assert c.metric_value("pytorch_operator_api_requests_total") > 0
