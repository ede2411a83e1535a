"""LocalCluster: fake API server + kubelet emulator + the native operator binary.

A one-node "cluster" for e2e tests and local development (the role GKE plays in the
reference's test/workflows).  Usage::

    with LocalCluster(gpus=[0]) as c:
        c.rest.create(PYTORCHJOBS, job, "default")
        ...

or from a shell: ``python -m pytorch_operator_amd.cluster up --gpus 0``.
"""
from __future__ import annotations

import os
import socket
import subprocess
import tempfile
import time
import urllib.request
from typing import Dict, List, Optional

from .fake_apiserver import FakeApiServer
from .kubelet import LocalKubelet
from kubeflow.pytorchjob.rest import Configuration, KubeRest

_LIB = os.path.join(os.path.dirname(__file__), "..", "_lib")


def operator_binary() -> str:
    p = os.path.abspath(os.path.join(_LIB, "pytorch-operator"))
    if not os.path.exists(p):
        from .. import native_build
        native_build.build_operator()
    return p


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class LocalCluster:
    def __init__(self, workdir: Optional[str] = None, gpus: Optional[List[int]] = None,
                 operator_args: Optional[List[str]] = None, start_operator: bool = True,
                 operator_env: Optional[Dict[str, str]] = None, kubelet_env: Optional[Dict[str, str]] = None,
                 verbose: bool = False, isolation: str = "none", isolation_needs_repo: bool = True):
        self._tmp = None
        if workdir is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="pto-cluster-")
            workdir = self._tmp.name
        self.workdir = workdir
        os.makedirs(workdir, exist_ok=True)
        self.log_dir = os.path.join(workdir, "pods")
        self.api = FakeApiServer(log_dir=self.log_dir)
        self.gpus = gpus
        self.operator_args = list(operator_args or [])
        self.start_operator = start_operator
        self.operator_env = dict(operator_env or {})
        self.kubelet_env = kubelet_env
        self.verbose = verbose
        self.isolation = isolation
        self.isolation_needs_repo = isolation_needs_repo
        self.operator: Optional[subprocess.Popen] = None
        self.monitoring_port = free_port()
        self.operator_log = os.path.join(workdir, "operator.log")
        self.kubelet: Optional[LocalKubelet] = None
        self.rest: Optional[KubeRest] = None
        self.kubeconfig = os.path.join(workdir, "kubeconfig.json")

    def start(self) -> "LocalCluster":
        self.api.start()
        self.api.install_crds()
        self.api.write_kubeconfig(self.kubeconfig)
        self.rest = KubeRest(Configuration(host=self.api.url, token="fake-token"))
        self.kubelet = LocalKubelet(self.rest, self.log_dir, gpus=self.gpus, extra_env=self.kubelet_env,
                                    verbose=self.verbose, isolation=self.isolation,
                                    isolation_needs_repo=self.isolation_needs_repo).start()
        if self.start_operator:
            self.start_operator_process()
        return self

    def spawn_operator(self, monitoring_port: int, log_path: str,
                       extra_args: Optional[List[str]] = None) -> subprocess.Popen:
        """Start one operator replica (several may run: leader election picks one)."""
        args = [operator_binary(), "--kubeconfig", self.kubeconfig,
                f"--monitoring-port={monitoring_port}", "--json-log-format=false",
                *self.operator_args, *(extra_args or [])]
        env = dict(os.environ, KUBEFLOW_NAMESPACE="kubeflow", **self.operator_env)
        env.pop("KUBECONFIG", None)
        with open(log_path, "ab") as log:
            return subprocess.Popen(args, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)

    def start_operator_process(self, extra_args: Optional[List[str]] = None) -> subprocess.Popen:
        self.operator = self.spawn_operator(self.monitoring_port, self.operator_log, extra_args)
        return self.operator

    def stop_operator(self, timeout: float = 15.0):
        if self.operator and self.operator.poll() is None:
            self.operator.terminate()
            try:
                self.operator.wait(timeout)
            except subprocess.TimeoutExpired:
                self.operator.kill()
                self.operator.wait()

    def metrics(self) -> str:
        with urllib.request.urlopen(f"http://127.0.0.1:{self.monitoring_port}/metrics", timeout=5) as r:
            return r.read().decode()

    def metric_value(self, name: str) -> float:
        total = 0.0
        for line in self.metrics().splitlines():
            if line.startswith(name + " ") or line.startswith(name + "{"):
                total += float(line.rsplit(" ", 1)[1])
        return total

    def wait_operator_ready(self, timeout: float = 30.0):
        t0 = time.time()
        while time.time() - t0 < timeout:
            try:
                if self.metric_value("pytorch_operator_is_leader") >= 1:
                    return
            except OSError:
                pass
            if self.operator and self.operator.poll() is not None:
                raise RuntimeError(f"operator exited with {self.operator.returncode}: "
                                   + open(self.operator_log).read()[-2000:])
            time.sleep(0.05)
        raise TimeoutError("operator did not become leader")

    def stop(self):
        self.stop_operator()
        if self.kubelet:
            self.kubelet.stop()
        self.api.stop()
        if self._tmp:
            self._tmp.cleanup()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
