"""Client configuration: API server address, credentials and TLS settings.

Stdlib-only counterpart of ``kubernetes.client.Configuration`` plus the kubeconfig /
in-cluster loaders the reference SDK gets from ``kubernetes.config``
(sdk/python/kubeflow/pytorchjob/api/py_torch_job_client.py:44-50 of the reference).
Supported kubeconfig fields: ``server``, ``certificate-authority[-data]``,
``insecure-skip-tls-verify``, ``tls-server-name``, ``token``, ``tokenFile``,
``client-certificate[-data]``, ``client-key[-data]`` and ``exec`` credential plugins
(client.authentication.k8s.io ExecCredential: token or client certificate).
"""
from __future__ import annotations

import base64
import json
import os
import subprocess
import tempfile
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional


@dataclass
class ExecPlugin:
    """A kubeconfig ``users[].user.exec`` credential plugin."""
    command: str
    args: List[str] = field(default_factory=list)
    env: Dict[str, str] = field(default_factory=dict)
    api_version: str = "client.authentication.k8s.io/v1"


@dataclass
class Configuration:
    host: str = "http://127.0.0.1:8001"
    token: Optional[str] = None
    verify_ssl: bool = True
    ssl_ca_cert: Optional[str] = None
    cert_file: Optional[str] = None
    key_file: Optional[str] = None
    tls_server_name: Optional[str] = None  # name checked against the server certificate
    namespace: str = "default"
    extra_headers: Dict[str, str] = field(default_factory=dict)
    exec_plugin: Optional[ExecPlugin] = None
    _exec_expiry: float = 0.0
    _exec_files: Optional[tuple] = None  # (cert, key) paths of the plugin's last client certificate

    def _has_exec_credential(self) -> bool:
        return bool(self.token) or self._exec_files is not None

    def refresh_credentials(self, force: bool = False) -> None:
        """Run the exec credential plugin when there is one and its credential (a token or a
        client certificate) is missing or expired."""
        if self.exec_plugin is None or (not force and self._has_exec_credential() and
                                        time.time() < self._exec_expiry):
            return
        cred = run_exec_plugin(self.exec_plugin)
        st = cred.get("status") or {}
        if st.get("token"):
            self.token = st["token"]
        if st.get("clientCertificateData") and st.get("clientKeyData"):
            # one pair of files per Configuration inside a private (0700) directory, rewritten on
            # refresh and removed at exit (the key is a secret: never leave one temp file per
            # request behind, and never write it where another local user can pre-create names)
            if self._exec_files is None:
                d = tempfile.mkdtemp(prefix="pytorchjob-exec-")  # mode 0700
                self._exec_files = (os.path.join(d, "client.crt"), os.path.join(d, "client.key"))
                import atexit
                atexit.register(_remove_files, self._exec_files, d)
            _write_private(self._exec_files[0], st["clientCertificateData"])
            _write_private(self._exec_files[1], st["clientKeyData"])
            self.cert_file, self.key_file = self._exec_files
        exp = st.get("expirationTimestamp")
        self._exec_expiry = _parse_rfc3339(exp) - 10 if exp else float("inf")


def run_exec_plugin(plugin: ExecPlugin, timeout: float = 60.0) -> dict:
    """Run ``plugin`` the way client-go does (KUBERNETES_EXEC_INFO in the environment) and
    return its ExecCredential."""
    env = dict(os.environ, **plugin.env)
    env["KUBERNETES_EXEC_INFO"] = json.dumps({"apiVersion": plugin.api_version, "kind": "ExecCredential",
                                              "spec": {"interactive": False}})
    r = subprocess.run([plugin.command, *plugin.args], env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"exec credential plugin {plugin.command!r} failed ({r.returncode}): {r.stderr[-500:]}")
    cred = json.loads(r.stdout)
    if cred.get("kind") != "ExecCredential":
        raise RuntimeError(f"exec credential plugin {plugin.command!r} did not return an ExecCredential")
    return cred


def _parse_rfc3339(s: str) -> float:
    import calendar
    s = s.rstrip("Z").split(".")[0]
    return float(calendar.timegm(time.strptime(s, "%Y-%m-%dT%H:%M:%S")))


def _write_private(path: str, text: str) -> None:
    """Atomically replace ``path`` (in a private directory) with a new 0600 file: the temp file
    is created with O_EXCL by mkstemp in the same directory, never at a guessable name."""
    fd, tmp = tempfile.mkstemp(dir=os.path.dirname(path), prefix=".tmp-")
    try:
        with os.fdopen(fd, "w") as f:
            f.write(text)
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


def _remove_files(paths, directory: Optional[str] = None) -> None:
    for p in paths:
        try:
            os.unlink(p)
        except OSError:
            pass
    if directory:
        try:
            os.rmdir(directory)
        except OSError:
            pass


def _materialise(data_b64: Optional[str]) -> Optional[str]:
    if not data_b64:
        return None
    f = tempfile.NamedTemporaryFile(delete=False, suffix=".pem")
    f.write(base64.b64decode(data_b64))
    f.close()
    return f.name


def load_kube_config(config_file: Optional[str] = None, context: Optional[str] = None) -> Configuration:
    """kubeconfig (YAML or JSON) -> Configuration (current or named context)."""
    import yaml
    path = config_file or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
    with open(path) as f:
        doc = yaml.safe_load(f)
    ctx_name = context or doc.get("current-context")
    by = lambda key, name: next((e for e in doc.get(key) or [] if e.get("name") == name), None)  # noqa: E731
    ctx = (by("contexts", ctx_name) or {}).get("context", {})
    cl = (by("clusters", ctx.get("cluster")) or (doc.get("clusters") or [{}])[0]).get("cluster", {})
    us = (by("users", ctx.get("user")) or {}).get("user", {})
    cfg = Configuration(host=cl.get("server", ""), namespace=ctx.get("namespace") or "default")
    cfg.verify_ssl = not cl.get("insecure-skip-tls-verify", False)
    cfg.ssl_ca_cert = cl.get("certificate-authority") or _materialise(cl.get("certificate-authority-data"))
    cfg.tls_server_name = cl.get("tls-server-name") or None
    cfg.token = us.get("token")
    if us.get("tokenFile"):
        with open(us["tokenFile"]) as f:
            cfg.token = f.read().strip()
    cfg.cert_file = us.get("client-certificate") or _materialise(us.get("client-certificate-data"))
    cfg.key_file = us.get("client-key") or _materialise(us.get("client-key-data"))
    ex = us.get("exec")
    if ex:
        cfg.exec_plugin = ExecPlugin(command=ex["command"], args=list(ex.get("args") or []),
                                     env={e["name"]: str(e["value"]) for e in ex.get("env") or []},
                                     api_version=ex.get("apiVersion", "client.authentication.k8s.io/v1"))
        cfg.refresh_credentials(force=True)
    if us.get("auth-provider"):
        raise RuntimeError("kubeconfig auth-provider plugins are removed in current Kubernetes clients; "
                           "use an exec credential plugin")
    return cfg


def load_incluster_config() -> Configuration:
    host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
    if not host or not port:
        raise RuntimeError("not running inside a cluster")
    sa = "/var/run/secrets/kubernetes.io/serviceaccount"
    with open(f"{sa}/token") as f:
        token = f.read().strip()
    ns = "default"
    if os.path.exists(f"{sa}/namespace"):
        with open(f"{sa}/namespace") as f:
            ns = f.read().strip()
    if ":" in host and not host.startswith("["):
        host = f"[{host}]"  # IPv6 service address
    return Configuration(host=f"https://{host}:{port}", token=token, ssl_ca_cert=f"{sa}/ca.crt", namespace=ns)
