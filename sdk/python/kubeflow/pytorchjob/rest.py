"""REST transport for the PyTorchJob SDK (stdlib only: no ``kubernetes`` package needed).

Plays the role ``kubernetes.client`` (CustomObjectsApi / CoreV1Api) plays for the reference
SDK (sdk/python/kubeflow/pytorchjob/api/py_torch_job_client.py:17-20 of the reference):
typed paths per group/version/resource, JSON bodies, merge/JSON patch, watch streams of
newline-delimited JSON events, pod logs (optionally followed to the end of the container),
bearer-token / client-certificate / exec-plugin auth and verified TLS (CA bundle + host
name or ``tls-server-name``).  The MI355X operator's local test cluster
(``pytorch_operator_amd.cluster``) uses this same module.
"""
from __future__ import annotations

import http.client
import json
import socket
import ssl
from dataclasses import dataclass
from typing import Callable, Dict, Iterator, Optional, Tuple
from urllib.parse import urlencode, urlparse

from .configuration import Configuration, load_incluster_config, load_kube_config  # noqa: F401


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
VOLCANO_PODGROUPS = GVR("scheduling.volcano.sh", "v1beta1", "podgroups")
CRDS = GVR("apiextensions.k8s.io", "v1", "customresourcedefinitions", namespaced=False)


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
            return _HTTPSConnection(self._host, self._port, timeout=timeout, context=ctx,
                                    server_name=self.config.tls_server_name)
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
                content_type: str = "application/json", raw: bool = False,
                on_chunk: Optional[Callable[[bytes], None]] = None):
        url = self._base + path + ("?" + urlencode(query) if query else "")
        data = None if body is None else json.dumps(body).encode()
        self.config.refresh_credentials()
        for attempt in (0, 1):
            conn = self._conn(self.timeout)
            try:
                conn.request(method, url, body=data, headers=self._headers(content_type if data else None))
                resp = conn.getresponse()
                if on_chunk is not None and resp.status < 300:
                    parts = []
                    while True:
                        chunk = resp.read1(65536)
                        if not chunk:
                            break
                        parts.append(chunk)
                        on_chunk(chunk)
                    payload = b"".join(parts)
                else:
                    payload = resp.read()
            finally:
                conn.close()
            if resp.status == 401 and attempt == 0 and self.config.exec_plugin is not None:
                self.config.refresh_credentials(force=True)  # expired plugin credential
                continue
            break
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
                tail_lines: Optional[int] = None, follow: bool = False,
                on_chunk: Optional[Callable[[bytes], None]] = None) -> str:
        """The pod's log.  ``follow``: stream it until the container terminates (the server
        closes the response), passing each piece to ``on_chunk`` as it arrives."""
        q = {}
        if container:
            q["container"] = container
        if tail_lines:
            q["tailLines"] = str(tail_lines)
        if follow:
            q["follow"] = "true"
        return self.request("GET", PODS.path(namespace, name, "log"), query=q or None, raw=True,
                            on_chunk=on_chunk if follow else None)

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
        self.config.refresh_credentials()
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


class _HTTPSConnection(http.client.HTTPSConnection):
    """HTTPS with the certificate checked against ``server_name`` (kubeconfig
    ``tls-server-name``) when the URL's host is not the name on the certificate."""

    def __init__(self, host, port, timeout, context, server_name: Optional[str] = None):
        super().__init__(host, port, timeout=timeout, context=context)
        self._server_name = server_name
        self._ctx = context

    def connect(self):
        if not self._server_name:
            return super().connect()
        sock = socket.create_connection((self.host, self.port), self.timeout, self.source_address)
        self.sock = self._ctx.wrap_socket(sock, server_hostname=self._server_name)
