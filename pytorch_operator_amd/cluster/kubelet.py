"""A single-node kubelet emulator: runs PyTorchJob pods as local processes.

Together with ``fake_apiserver`` this replaces the reference's GKE test cluster
(test/workflows, py/kubeflow/pytorchjob_tests) so the C++ operator can be exercised
end to end in CI: the operator creates pods/services, this emulator "schedules" and
runs them, and reports status back exactly the way the operator reads it.

What it emulates
----------------
* scheduling: binds a pod to this node when its extended resources fit.  ``amd.com/gpu``
  limits allocate device ids from ``gpus`` and export ``HIP_VISIBLE_DEVICES`` (the AMD
  device plugin contract); requests for a resource this node does not have (e.g.
  ``nvidia.com/gpu``) leave the pod Pending with ``PodScheduled=False/Unschedulable``;
* images: an image is resolved to an entrypoint through ``image_map`` (substring match,
  e.g. ``pytorch_dist_mnist`` -> ``python -m pytorch_operator_amd.harness.mnist``);
  explicit ``command``/``args`` run as given (``python`` means this interpreter);
  an unknown image without a command waits in ``ErrImagePull``;
* init containers: the operator's default init container (``until nslookup <master>``)
  is resolved against the API server's Services (cluster DNS); any other init container
  runs like a main container and must exit 0;
* pod networking: every pod shares the host (podIP 127.0.0.1).  A ``MASTER_ADDR`` naming a
  Service is rewritten to 127.0.0.1 and its ``MASTER_PORT`` to a per-Service free local
  port, so concurrent jobs do not collide on 23456;
* restart policies: ``Always`` / ``OnFailure`` restart the container in place
  (``restartCount``, ``lastState.terminated``), ``Never`` ends the pod Succeeded/Failed
  with ``state.terminated.exitCode`` -- the field the ExitCode restart policy reads
  (reference pkg/controller.v1/pytorch/pod.go:116-135);
* deletion: SIGTERM to the container's process group, SIGKILL after the grace period;
* fault injection (the SURVEY 5.3 injector): pod annotations
  ``fault.pto.amd.com/exit-code`` (exit code to report), ``fault.pto.amd.com/after-seconds``
  (delay after container start, default 0) and ``fault.pto.amd.com/times`` (how many runs of
  that pod *name* to hit, default 1; counted across pod recreations) kill the container and
  report the given code -- e.g. 137 to exercise the ExitCode restart policy with a real job;
* logs: stdout/stderr of every container go to ``<log_dir>/<ns>_<pod>.log``, served by the
  fake API server's ``pods/{name}/log`` endpoint;
* namespaces (``isolation="namespaces"``): like a real kubelet, a pod gets its own PID and
  IPC namespaces, a private ``/dev/shm`` and its own hostname unless its spec sets
  ``hostPID`` / ``hostIPC`` (``unshare`` in a user namespace, before anything in the pod
  touches the GPU).  A pod with both ``hostPID`` and ``hostIPC`` runs in the node's
  namespaces (its UTS namespace too: isolating only the hostname would need a separate user
  namespace, which a real kubelet does not create).  This is what makes the operator's
  ``--xgmi-pod-topology`` observable on one node: without it, xGMI peer-memory IPC between
  pods fails exactly as on a cluster (docs/xgmi_pods.md).
"""
from __future__ import annotations

import copy
import os
import re
import shlex
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

from kubeflow.pytorchjob.rest import PODS, SERVICES, ApiException, KubeRest

REPO_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))


def default_image_map(python: str = sys.executable) -> Dict[str, List[str]]:
    mnist = [python, "-m", "pytorch_operator_amd.harness.mnist"]
    smoke = [python, "-m", "pytorch_operator_amd.harness.dist_sendrecv"]
    return {
        "pytorch_dist_mnist": mnist, "pytorch-dist-mnist": mnist, "mnist": mnist,
        "pytorch_dist_sendrecv": smoke, "smoke-dist": smoke, "dist-sendrecv": smoke,
        "pytorch-operator-amd/worker": [python, "-m", "pytorch_operator_amd.harness.mnist"],
    }


SCRIPT_MAP = {
    "/opt/mnist/src/mnist.py": ["-m", "pytorch_operator_amd.harness.mnist"],
    "/opt/mlkube/dist_sendrecv.py": ["-m", "pytorch_operator_amd.harness.dist_sendrecv"],
}


_POD_SCOPED_ENV = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                   "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE",
                   "KUBECONFIG", "PYTHONPATH"}
# a launcher's (torchrun) per-process state must never leak into a pod: e.g. an inherited
# TORCHELASTIC_USE_AGENT_STORE makes the pod's env:// rendezvous a client of a store nobody hosts
_POD_SCOPED_PREFIXES = ("TORCHELASTIC_", "TORCH_ELASTIC_")


def _node_env() -> Dict[str, str]:
    return {k: v for k, v in os.environ.items()
            if k not in _POD_SCOPED_ENV and not k.startswith(_POD_SCOPED_PREFIXES)}


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


def _ephemeral_range():
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo, hi = (int(x) for x in f.read().split())
        return lo, hi
    except (OSError, ValueError):
        return 32768, 60999


def _free_port(taken=()) -> int:
    """A free port *below* the kernel's ephemeral range.

    Rendezvous ports are connected to before anyone listens (workers race the master's
    TCPStore); a port inside the ephemeral range can then be handed out as the client's own
    source port, and the TCP simultaneous-open rule connects the socket to itself -- a
    silent hang in init_process_group.  Ports below the range never collide that way.
    """
    import random
    lo, _ = _ephemeral_range()
    base = max(1024, lo - 12000)
    for _ in range(1000):
        port = random.randrange(base, lo)
        if port in taken:
            continue
        with socket.socket() as s:
            try:
                s.bind(("0.0.0.0", port))
            except OSError:
                continue
            return port
    raise RuntimeError("no free rendezvous port")


def namespaces_available(readable: Optional[str] = None) -> tuple:
    """(ok, error): can this node give a pod its own user/PID/IPC/UTS/mount namespaces (and,
    with ``readable``, can a process in them still read that path -- a checkout under
    another user's 0700 home is not readable from a user namespace)?"""
    import shutil
    if not shutil.which("unshare"):
        return False, "unshare not found"
    probe = "echo $$" + (f" && test -r '{readable}'" if readable else "")
    try:
        r = subprocess.run(["unshare", "--user", "--map-root-user", "--fork", "--kill-child", "--mount", "--uts",
                            "--pid", "--mount-proc", "--ipc", "sh", "-c", probe],
                           capture_output=True, text=True, timeout=10)
    except (OSError, subprocess.TimeoutExpired) as e:
        return False, repr(e)
    if r.returncode != 0 or r.stdout.strip() != "1":
        why = (r.stderr or r.stdout).strip()[-300:]
        return False, why or f"{readable} is not readable inside a user namespace"
    return True, ""


class _Container:
    def __init__(self, spec: dict):
        self.spec = spec
        self.name = spec.get("name", "c")
        self.proc: Optional[subprocess.Popen] = None
        self.restart_count = 0
        self.state: dict = {"waiting": {"reason": "ContainerCreating"}}
        self.last_state: dict = {}
        self.done = False
        self.exit_code: Optional[int] = None


class PodRunner(threading.Thread):
    def __init__(self, kubelet: "LocalKubelet", pod: dict):
        super().__init__(daemon=True, name="pod-" + pod["metadata"]["name"])
        self.k = kubelet
        self.pod = pod
        self.ns = pod["metadata"].get("namespace", "default")
        self.name = pod["metadata"]["name"]
        self.uid = pod["metadata"]["uid"]
        self.stopping = threading.Event()
        self.gpus: List[int] = []
        self.log_path = os.path.join(self.k.log_dir, f"{self.ns}_{self.name}.log")
        self.workdir = os.path.join(self.k.log_dir, "pods", f"{self.ns}_{self.name}_{self.uid[:8]}", "work")
        self.containers = [_Container(c) for c in pod["spec"].get("containers") or []]
        self.init_status: List[dict] = []
        self.phase = "Pending"
        self.start_time = None

    # ---------------------------------------------------------------- status
    def _push(self, phase: Optional[str] = None, conditions: Optional[list] = None, reason=None, message=None):
        if phase:
            self.phase = phase
        st = {"phase": self.phase, "hostIP": "127.0.0.1", "podIP": "127.0.0.1"}
        if self.start_time:
            st["startTime"] = self.start_time
        st["containerStatuses"] = [{
            "name": c.name, "image": c.spec.get("image", ""), "restartCount": c.restart_count,
            "ready": "running" in c.state, "started": "running" in c.state,
            "state": c.state, "lastState": c.last_state} for c in self.containers]
        if self.init_status:
            st["initContainerStatuses"] = self.init_status
        if conditions is not None:
            st["conditions"] = conditions
        if reason:
            st["reason"] = reason
        if message:
            st["message"] = message
        try:
            self.k.rest.patch(PODS, self.name, {"status": st}, self.ns, status=True)
        except ApiException as e:
            if e.status == 404:
                self.stopping.set()
            elif e.status != 409:
                raise

    def _alive(self) -> bool:
        return not self.stopping.is_set() and not self.k.stopped.is_set()

    # ---------------------------------------------------------------- run
    def run(self):
        try:
            self._run()
        except Exception as e:  # noqa: BLE001 -- a broken pod must not kill the node
            self.k._log(f"pod {self.ns}/{self.name}: runtime error {e!r}")
        finally:
            self.k._release(self)

    def _run(self):
        os.makedirs(self.workdir, exist_ok=True)
        # 1. scheduling
        while self._alive():
            ok, why = self.k._admit(self)
            if ok:
                break
            self._push("Pending", [{"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                                    "message": why, "lastTransitionTime": _now()}])
            self.stopping.wait(1.0)
        if not self._alive():
            return
        try:
            self.k.rest.patch(PODS, self.name, {"spec": {"nodeName": self.k.node_name}}, self.ns)
        except ApiException:
            return
        self.start_time = _now()
        cond = [{"type": "PodScheduled", "status": "True", "lastTransitionTime": _now()}]
        self._push("Pending", cond)
        # 2. init containers
        for ic in self.pod["spec"].get("initContainers") or []:
            code = self._run_init(ic)
            if code is None:
                return
            self.init_status.append({"name": ic.get("name"), "ready": code == 0, "restartCount": 0,
                                     "state": {"terminated": {"exitCode": code, "reason":
                                               "Completed" if code == 0 else "Error", "finishedAt": _now()}}})
            if code != 0:
                self._push("Failed", cond, reason="InitContainerFailed")
                return
        # 3. main containers
        policy = self.pod["spec"].get("restartPolicy", "Always")
        threads = [threading.Thread(target=self._run_container, args=(c, policy), daemon=True)
                   for c in self.containers]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if not self._alive():
            return
        codes = [c.exit_code for c in self.containers]
        phase = "Succeeded" if all(c == 0 for c in codes) else "Failed"
        self._push(phase, cond + [{"type": "Ready", "status": "False", "reason": "PodCompleted"}])

    def _run_init(self, spec: dict) -> Optional[int]:
        text = " ".join(spec.get("command") or []) + " " + " ".join(spec.get("args") or [])
        m = re.search(r"nslookup\s+([A-Za-z0-9.-]+)", text)
        if m:  # cluster DNS: the name resolves once a Service of that name exists
            host = m.group(1).split(".")[0]
            while self._alive():
                try:
                    self.k.rest.get(SERVICES, host, self.ns)
                    return 0
                except ApiException as e:
                    if e.status != 404:
                        raise
                self.stopping.wait(self.k.dns_poll_s)
            return None
        c = _Container(spec)
        self._run_container(c, "Never", init=True)
        return c.exit_code if self._alive() else None

    def _argv(self, spec: dict) -> Optional[List[str]]:
        cmd = list(spec.get("command") or [])
        args = [str(a) for a in spec.get("args") or []]
        if not cmd:
            image = spec.get("image", "")
            base = image.split("@")[0].rsplit(":", 1)[0] if ":" in image.split("/")[-1] else image
            for key, entry in self.k.image_map.items():
                if key in base:
                    return list(entry) + args
            return None
        if cmd[0] in ("python", "python3") or cmd[0].endswith("/python") or cmd[0].endswith("/python3"):
            cmd[0] = self.k.python
            if len(cmd) > 1 and cmd[1] in SCRIPT_MAP:
                cmd = [cmd[0]] + SCRIPT_MAP[cmd[1]] + cmd[2:]
        return cmd + args

    def _isolate(self, argv: List[str]) -> List[str]:
        """Wrap ``argv`` in the namespaces this pod does not share with the node."""
        if not self.k.isolation_active:
            return argv
        ps = self.pod.get("spec") or {}
        host_pid, host_ipc = bool(ps.get("hostPID")), bool(ps.get("hostIPC"))
        if host_pid and host_ipc:
            return argv
        wrap = ["unshare", "--user", "--map-root-user", "--fork", "--kill-child", "--mount", "--uts"]
        if not host_pid:
            wrap += ["--pid", "--mount-proc"]
        setup = 'hostname "$0" 2>/dev/null; '
        if not host_ipc:
            wrap.append("--ipc")
            setup += "mount -t tmpfs -o size=64m tmpfs /dev/shm 2>/dev/null; "
        return wrap + ["sh", "-c", setup + 'exec "$@"', self.name] + argv

    def _env(self, spec: dict) -> Dict[str, str]:
        # the node's environment minus anything a container must get from its pod spec
        base = _node_env()
        base["PYTHONPATH"] = os.pathsep.join([self.k.repo_root] + [p for p in
                                            os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
        base["HOSTNAME"] = self.name
        base["PYTHONUNBUFFERED"] = "1"
        base.setdefault("PYTHONFAULTHANDLER", "1")  # SIGABRT/SIGSEGV dump Python stacks into the pod log
        base.setdefault("OMP_NUM_THREADS", "1")
        md = self.pod["metadata"]
        for e in spec.get("env") or []:
            if "value" in e:
                base[e["name"]] = str(e["value"])
            elif "valueFrom" in e:
                fp = ((e["valueFrom"].get("fieldRef") or {}).get("fieldPath") or "")
                val = {"metadata.name": md.get("name"), "metadata.namespace": self.ns,
                       "status.podIP": "127.0.0.1", "spec.nodeName": self.k.node_name,
                       "metadata.uid": md.get("uid")}.get(fp)
                if val is not None:
                    base[e["name"]] = val
        addr = base.get("MASTER_ADDR")
        if addr:
            # the master itself gets MASTER_ADDR=localhost (pod.go:246-251): its Service
            # carries the pod's name, so map it to the same per-Service port as the workers
            svc = self.name if addr in ("localhost", "127.0.0.1") else addr.split(".")[0]
            port = self.k._service_port(self.ns, svc, base.get("MASTER_PORT"),
                                        known=addr in ("localhost", "127.0.0.1"))
            if port is not None:
                base["MASTER_ADDR"] = "127.0.0.1"
                base["MASTER_PORT"] = str(port)
        if self.gpus:
            # node-relative ids -> the node's own visible set (never widen visibility)
            node = [d for d in os.environ.get("HIP_VISIBLE_DEVICES", "").split(",") if d.strip()]
            ids = [node[g] if node else str(g) for g in self.gpus]
            base["HIP_VISIBLE_DEVICES"] = ",".join(ids)
        elif self.k.hide_gpus_without_request:
            base["HIP_VISIBLE_DEVICES"] = ""
        base.update(self.k.extra_env)
        return base

    def _run_container(self, c: _Container, policy: str, init: bool = False):
        argv = self._argv(c.spec)
        if argv is not None:
            argv = self._isolate(argv)
        if argv is None:
            c.state = {"waiting": {"reason": "ErrImagePull",
                                   "message": f"image {c.spec.get('image')!r} not known to this node"}}
            if not init:
                self._push("Pending")
            while self._alive():
                self.stopping.wait(1.0)
            return
        backoff = 0.2
        while self._alive():
            with open(self.log_path, "ab") as log:
                log.write(f"==> {' '.join(shlex.quote(a) for a in argv)}\n".encode())
                log.flush()
                try:
                    c.proc = subprocess.Popen(argv, env=self._env(c.spec), cwd=self.workdir, stdout=log,
                                              stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                              start_new_session=True)
                except OSError as e:
                    log.write(f"failed to start: {e}\n".encode())
                    c.exit_code = 127
                    c.state = {"terminated": {"exitCode": 127, "reason": "ContainerCannotRun",
                                              "message": str(e), "finishedAt": _now()}}
                    if not init:
                        self._push()
                    return
            started = _now()
            c.state = {"running": {"startedAt": started}}
            if not init:
                self._push("Running", [{"type": "PodScheduled", "status": "True"},
                                       {"type": "Ready", "status": "True", "lastTransitionTime": started}])
            injected = None if init else self.k._fault_for(self)
            if injected is not None:
                code_fault, after = injected
                timer = threading.Timer(after, self._inject, args=(c.proc,))
                timer.daemon = True
                timer.start()
            code = c.proc.wait()
            if code < 0:  # killed by signal -> 128+N like a container runtime
                code = 128 - code
            if injected is not None:
                timer.cancel()
                if code == 128 + signal.SIGKILL and self._alive():
                    code = code_fault
            if not self._alive():
                return
            term = {"exitCode": code, "reason": "Completed" if code == 0 else "Error",
                    "startedAt": started, "finishedAt": _now()}
            restart = policy == "Always" or (policy == "OnFailure" and code != 0)
            if restart and not init:
                c.restart_count += 1
                c.last_state = {"terminated": term}
                c.state = {"waiting": {"reason": "CrashLoopBackOff" if code else "Completed"}}
                self._push()
                self.stopping.wait(backoff)
                backoff = min(backoff * 2, 10.0)
                continue
            c.exit_code = code
            c.state = {"terminated": term}
            return

    @staticmethod
    def _inject(proc: subprocess.Popen):
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass

    def kill(self, grace_s: float = 2.0):
        self.stopping.set()
        procs = [c.proc for c in self.containers if c.proc is not None and c.proc.poll() is None]
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
        deadline = time.time() + grace_s
        for p in procs:
            try:
                p.wait(max(0.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                p.wait()


class LocalKubelet:
    """Watch pods on the API server and run them locally.  ``start()`` / ``stop()``."""

    def __init__(self, rest: KubeRest, log_dir: str, node_name: str = "mi355x-node-0",
                 namespace: Optional[str] = None, gpus: Optional[List[int]] = None,
                 image_map: Optional[Dict[str, List[str]]] = None, python: str = sys.executable,
                 repo_root: str = REPO_ROOT, extra_env: Optional[Dict[str, str]] = None,
                 hide_gpus_without_request: bool = True, dns_poll_s: float = 0.1, verbose: bool = False,
                 isolation: str = "none", isolation_needs_repo: bool = True):
        self.rest = rest
        self.log_dir = os.path.abspath(log_dir)
        os.makedirs(self.log_dir, exist_ok=True)
        self.node_name = node_name
        self.namespace = namespace
        self.free_gpus = list(gpus or [])
        self.python = python
        self.image_map = image_map if image_map is not None else default_image_map(python)
        self.repo_root = repo_root
        self.extra_env = dict(extra_env or {})
        self.hide_gpus_without_request = hide_gpus_without_request
        self.dns_poll_s = dns_poll_s
        self.verbose = verbose
        self.runners: Dict[str, PodRunner] = {}
        self.ports: Dict[tuple, int] = {}
        self.faults_done: Dict[tuple, int] = {}
        self.lock = threading.RLock()
        self.stopped = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True, name="kubelet")
        self.finished_pods: List[str] = []
        if isolation not in ("none", "namespaces"):
            raise ValueError(f"unknown isolation {isolation!r}")
        self.isolation = isolation
        self.isolation_active = False
        self.isolation_error = ""
        if isolation == "namespaces":
            probe = os.path.join(repo_root, "pytorch_operator_amd", "__init__.py") if isolation_needs_repo else None
            self.isolation_active, self.isolation_error = namespaces_available(probe)
            if not self.isolation_active:
                self._log(f"pod namespaces unavailable ({self.isolation_error}); pods share the node's")

    def _log(self, msg: str):
        if self.verbose:
            print(f"[kubelet] {msg}", file=sys.stderr, flush=True)

    # ---------------------------------------------------------------- resources
    def _admit(self, r: PodRunner):
        want = 0
        for c in r.pod["spec"].get("containers") or []:
            res = c.get("resources") or {}
            lim = dict(res.get("requests") or {}, **(res.get("limits") or {}))
            for k, v in lim.items():
                if k in ("cpu", "memory", "ephemeral-storage"):
                    continue
                if k == "amd.com/gpu":
                    want += int(v)
                else:
                    return False, f"0/1 nodes are available: 1 Insufficient {k}."
        with self.lock:
            if want > len(self.free_gpus):
                return False, "0/1 nodes are available: 1 Insufficient amd.com/gpu."
            r.gpus = self.free_gpus[:want]
            self.free_gpus = self.free_gpus[want:]
        return True, ""

    def _release(self, r: PodRunner):
        with self.lock:
            self.free_gpus = sorted(self.free_gpus + r.gpus)
            r.gpus = []
            self.finished_pods.append(f"{r.ns}/{r.name}")

    def _fault_for(self, r: PodRunner):
        """(exit_code, after_s) when this run of the pod should be killed, else None."""
        ann = r.pod["metadata"].get("annotations") or {}
        if "fault.pto.amd.com/exit-code" not in ann:
            return None
        key = (r.ns, r.name)
        with self.lock:
            n = self.faults_done.get(key, 0)
            if n >= int(ann.get("fault.pto.amd.com/times", "1")):
                return None
            self.faults_done[key] = n + 1
        return int(ann["fault.pto.amd.com/exit-code"]), float(ann.get("fault.pto.amd.com/after-seconds", "0"))

    def _service_port(self, ns: str, svc: str, port: Optional[str], known: bool = False) -> Optional[int]:
        """Host port standing in for ``svc:port``.  ``known``: the caller is the pod behind
        the Service (the master, which may start before its Service is created)."""
        with self.lock:
            key = (ns, svc, port)
            if key in self.ports:
                return self.ports[key]
        if not known:
            try:
                self.rest.get(SERVICES, svc, ns)
            except ApiException:
                return None
        with self.lock:
            if key not in self.ports:
                self.ports[key] = _free_port(set(self.ports.values()))
            return self.ports[key]

    # ---------------------------------------------------------------- watch loop
    def _mine(self, pod: dict) -> bool:
        node = pod.get("spec", {}).get("nodeName")
        return not node or node == self.node_name

    def _on_pod(self, etype: str, pod: dict):
        uid = pod["metadata"]["uid"]
        with self.lock:
            r = self.runners.get(uid)
        if etype == "DELETED" or pod["metadata"].get("deletionTimestamp"):
            if r is not None:
                self._log(f"kill {pod['metadata']['name']}")
                r.kill()
                with self.lock:
                    self.runners.pop(uid, None)
            return
        if r is None and self._mine(pod) and pod.get("status", {}).get("phase", "Pending") == "Pending" \
                and not pod.get("spec", {}).get("nodeName"):
            r = PodRunner(self, copy.deepcopy(pod))
            with self.lock:
                self.runners[uid] = r
            self._log(f"start {pod['metadata']['name']}")
            r.start()

    def _loop(self):
        while not self.stopped.is_set():
            try:
                lst = self.rest.list(PODS, self.namespace)
                live = set()
                for p in lst.get("items", []):
                    live.add(p["metadata"]["uid"])
                    self._on_pod("ADDED", p)
                with self.lock:
                    gone = [u for u in self.runners if u not in live]
                for u in gone:
                    r = self.runners.pop(u, None)
                    if r:
                        r.kill()
                rv = lst.get("metadata", {}).get("resourceVersion", "")
                while not self.stopped.is_set():
                    for etype, obj in self.rest.watch(PODS, self.namespace, rv, timeout_seconds=5):
                        rv = obj.get("metadata", {}).get("resourceVersion", rv)
                        self._on_pod(etype, obj)
                        if self.stopped.is_set():
                            break
            except ApiException as e:
                self._log(f"watch error {e.status}; relisting")
                time.sleep(0.1)
            except OSError as e:
                if self.stopped.is_set():
                    return
                self._log(f"connection error {e}; retrying")
                time.sleep(0.5)

    def start(self) -> "LocalKubelet":
        self.thread.start()
        return self

    def stop(self):
        self.stopped.set()
        with self.lock:
            rs = list(self.runners.values())
            self.runners.clear()
        for r in rs:
            r.kill()
        self.thread.join(timeout=10)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
