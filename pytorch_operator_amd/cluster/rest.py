"""A small Kubernetes REST client (stdlib only).

The official ``kubernetes`` Python client is not installed in this image, so the SDK
(``sdk/python/kubeflow/pytorchjob``), the kubelet emulator and the e2e tests share this
client.  It speaks the same API the C++ operator does (csrc/operator/src/kube.cpp):
typed paths per group/version/resource, JSON bodies, merge-patch, watch streams of
newline-delimited JSON events, bearer-token/kubeconfig/in-cluster configuration.
"""
from __future__ import annotations

import json
import os
import ssl
import base64
import tempfile
import http.client
from dataclasses import dataclass, field
from typing import Dict, Iterator, Optional, Tuple
from urllib.parse import urlencode, urlparse


class ApiException(Exception):
    """Mirrors ``kubernetes.client.rest.ApiException`` (status, reason, body)."""

    def __init__(self, status: int = 0, reason: str = "", body: str = ""):
        self.status, self.reason, self.body = status, reason, body
        super().__init__(f"({status})\nReason: {reason}\nHTTP response body: {body}")


@dataclass(frozen=True)
class GVR:
    group: str
    version: str
    plural: str
    namespaced: bool = True

    def path(self, namespace: Optional[str] = None, name: Optional[str] = None,
             sub: Optional[str] = None) -> str:
        p = f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"
        if self.namespaced and namespace:
            p += f"/namespaces/{namespace}"
        p += f"/{self.plural}"
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return p


PODS = GVR("", "v1", "pods")
SERVICES = GVR("", "v1", "services")
EVENTS = GVR("", "v1", "events")
NAMESPACES = GVR("", "v1", "namespaces", namespaced=False)
LEASES = GVR("coordination.k8s.io", "v1", "leases")
PYTORCHJOBS = GVR("kubeflow.org", "v1", "pytorchjobs")
PODGROUPS = GVR("scheduling.incubator.k8s.io", "v1alpha1", "podgroups")
CRDS = GVR("apiextensions.k8s.io", "v1", "customresourcedefinitions", namespaced=False)


@dataclass
class Configuration:
    host: str = "http://127.0.0.1:8001"
    token: Optional[str] = None
    verify_ssl: bool = True
    ssl_ca_cert: Optional[str] = None
    cert_file: Optional[str] = None
    key_file: Optional[str] = None
    namespace: str = "default"
    extra_headers: Dict[str, str] = field(default_factory=dict)


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
    cfg.token = us.get("token")
    if us.get("tokenFile"):
        with open(us["tokenFile"]) as f:
            cfg.token = f.read().strip()
    cfg.cert_file = us.get("client-certificate") or _materialise(us.get("client-certificate-data"))
    cfg.key_file = us.get("client-key") or _materialise(us.get("client-key-data"))
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
    return Configuration(host=f"https://{host}:{port}", token=token, ssl_ca_cert=f"{sa}/ca.crt", namespace=ns)


class KubeRest:
    def __init__(self, config: Optional[Configuration] = None, timeout: float = 30.0):
        self.config = config or Configuration()
        self.timeout = timeout
        u = urlparse(self.config.host)
        self._scheme, self._host = u.scheme or "http", u.hostname or "127.0.0.1"
        self._port = u.port or (443 if self._scheme == "https" else 80)
        self._base = (u.path or "").rstrip("/")

    # ------------------------------------------------------------------ transport
    def _conn(self, timeout: Optional[float]):
        if self._scheme == "https":
            ctx = ssl.create_default_context(cafile=self.config.ssl_ca_cert)
            if not self.config.verify_ssl:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if self.config.cert_file:
                ctx.load_cert_chain(self.config.cert_file, self.config.key_file)
            return http.client.HTTPSConnection(self._host, self._port, timeout=timeout, context=ctx)
        return http.client.HTTPConnection(self._host, self._port, timeout=timeout)

    def _headers(self, ctype: Optional[str]) -> Dict[str, str]:
        h = {"Accept": "application/json", "User-Agent": "pytorchjob-sdk-amd/0.1"}
        if ctype:
            h["Content-Type"] = ctype
        if self.config.token:
            h["Authorization"] = f"Bearer {self.config.token}"
        h.update(self.config.extra_headers)
        return h

    def request(self, method: str, path: str, body=None, query: Optional[dict] = None,
                content_type: str = "application/json", raw: bool = False):
        url = self._base + path + ("?" + urlencode(query) if query else "")
        data = None if body is None else json.dumps(body).encode()
        conn = self._conn(self.timeout)
        try:
            conn.request(method, url, body=data, headers=self._headers(content_type if data else None))
            resp = conn.getresponse()
            payload = resp.read()
        finally:
            conn.close()
        if resp.status >= 300:
            raise ApiException(resp.status, resp.reason, payload.decode(errors="replace"))
        if raw:
            return payload.decode(errors="replace")
        return json.loads(payload) if payload else {}

    # ------------------------------------------------------------------ verbs
    def get(self, gvr: GVR, name: str, namespace: Optional[str] = None) -> dict:
        return self.request("GET", gvr.path(namespace, name))

    def list(self, gvr: GVR, namespace: Optional[str] = None, label_selector: str = "",
             field_selector: str = "") -> dict:
        q = {}
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        return self.request("GET", gvr.path(namespace), query=q or None)

    def create(self, gvr: GVR, body: dict, namespace: Optional[str] = None) -> dict:
        return self.request("POST", gvr.path(namespace), body)

    def replace(self, gvr: GVR, name: str, body: dict, namespace: Optional[str] = None) -> dict:
        return self.request("PUT", gvr.path(namespace, name), body)

    def replace_status(self, gvr: GVR, name: str, body: dict, namespace: Optional[str] = None) -> dict:
        return self.request("PUT", gvr.path(namespace, name, "status"), body)

    def patch(self, gvr: GVR, name: str, body, namespace: Optional[str] = None,
              status: bool = False) -> dict:
        ctype = "application/json-patch+json" if isinstance(body, list) else "application/merge-patch+json"
        return self.request("PATCH", gvr.path(namespace, name, "status" if status else None), body,
                            content_type=ctype)

    def delete(self, gvr: GVR, name: str, namespace: Optional[str] = None,
               propagation: str = "Background") -> dict:
        return self.request("DELETE", gvr.path(namespace, name),
                            {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": propagation})

    def pod_log(self, name: str, namespace: Optional[str] = None, container: Optional[str] = None,
                tail_lines: Optional[int] = None) -> str:
        q = {}
        if container:
            q["container"] = container
        if tail_lines:
            q["tailLines"] = str(tail_lines)
        return self.request("GET", PODS.path(namespace, name, "log"), query=q or None, raw=True)

    def watch(self, gvr: GVR, namespace: Optional[str] = None, resource_version: str = "",
              label_selector: str = "", timeout_seconds: int = 60,
              field_selector: str = "") -> Iterator[Tuple[str, dict]]:
        """Yield (type, object) until the server closes the stream or timeout_seconds."""
        q = {"watch": "true", "timeoutSeconds": str(int(timeout_seconds))}
        if resource_version:
            q["resourceVersion"] = resource_version
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        conn = self._conn(timeout_seconds + 30)
        try:
            conn.request("GET", self._base + gvr.path(namespace) + "?" + urlencode(q),
                         headers=self._headers(None))
            resp = conn.getresponse()
            if resp.status >= 300:
                raise ApiException(resp.status, resp.reason, resp.read().decode(errors="replace"))
            while True:
                line = resp.readline()
                if not line:
                    return
                line = line.strip()
                if not line:
                    continue
                ev = json.loads(line)
                if ev.get("type") == "ERROR":
                    st = ev.get("object") or {}
                    raise ApiException(int(st.get("code", 500)), st.get("reason", ""), json.dumps(st))
                yield ev.get("type"), ev.get("object")
        finally:
            conn.close()
