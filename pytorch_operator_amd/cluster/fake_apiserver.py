"""An in-process Kubernetes API server emulator for tests and local runs.

The reference is only ever exercised against a real GKE cluster (test/workflows,
scripts/create-cluster.sh); this image has no kubectl/kind/docker, so the operator's
informers, clients and leader election are tested against this server instead.  It is
faithful on the semantics the operator depends on:

* REST paths for core/v1 (pods, services, events, endpoints, namespaces), coordination.k8s.io/v1
  leases, kubeflow.org/v1 pytorchjobs (with a ``/status`` subresource),
  scheduling.incubator.k8s.io/v1alpha1 + scheduling.volcano.sh/v1beta1 podgroups and
  apiextensions.k8s.io/v1 customresourcedefinitions;
* a global monotonically increasing ``resourceVersion``; optimistic concurrency on PUT
  (stale resourceVersion -> 409 Conflict); create of an existing name -> 409;
* LIST with ``labelSelector`` (=, ==, !=, exists, !exists, in/notin) and ``fieldSelector``
  on metadata.name/namespace; WATCH streams (chunked, one JSON event per line) from any
  retained resourceVersion, ``410 Gone`` (as an ERROR event) when the version is compacted,
  ``timeoutSeconds``;
* status subresource: PUT on the object ignores .status, PUT /status only changes .status;
* JSON merge patch (also accepted for strategic-merge content types);
* background cascading deletion through ownerReferences (the GC the operator relies on
  when a finished PyTorchJob is deleted, reference e2e test/e2e/v1/default/defaults.go:168-188);
* pod logs at ``/api/v1/namespaces/{ns}/pods/{name}/log`` (served from files written by
  the kubelet emulator);
* the CRD's openAPI validation of replica counts (manifests/crd.yaml:21-38).
"""
from __future__ import annotations

import copy
import json
import re
import threading
import time
import uuid
from collections import deque
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlparse

# (group, version, plural) -> (kind, namespaced, has_status_subresource)
RESOURCES = {
    ("", "v1", "pods"): ("Pod", True, True),
    ("", "v1", "services"): ("Service", True, True),
    ("", "v1", "events"): ("Event", True, False),
    ("", "v1", "endpoints"): ("Endpoints", True, False),
    ("", "v1", "configmaps"): ("ConfigMap", True, False),
    ("", "v1", "namespaces"): ("Namespace", False, True),
    ("coordination.k8s.io", "v1", "leases"): ("Lease", True, False),
    ("kubeflow.org", "v1", "pytorchjobs"): ("PyTorchJob", True, True),
    ("scheduling.incubator.k8s.io", "v1alpha1", "podgroups"): ("PodGroup", True, True),
    ("scheduling.volcano.sh", "v1beta1", "podgroups"): ("PodGroup", True, True),
    ("apiextensions.k8s.io", "v1", "customresourcedefinitions"): ("CustomResourceDefinition", False, True),
}
CRD_RESOURCES = {("kubeflow.org", "v1", "pytorchjobs")}


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


class ApiException(Exception):
    def __init__(self, code: int, reason: str, message: str):
        super().__init__(message)
        self.code, self.reason, self.message = code, reason, message

    def status(self) -> dict:
        return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                "message": self.message, "reason": self.reason, "code": self.code}


# ----------------------------------------------------------------- selectors
_SEL_RE = re.compile(r"^\s*(!?)([A-Za-z0-9_./-]+)\s*(?:(==|!=|=)\s*([A-Za-z0-9_.-]*)|\s+(in|notin)\s*\(([^)]*)\))?\s*$")


def _split_selector(sel: str) -> List[str]:
    parts, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return parts


def label_selector_matches(sel: str, labels: Optional[dict]) -> bool:
    labels = labels or {}
    for term in _split_selector(sel or ""):
        m = _SEL_RE.match(term)
        if not m:
            raise ApiException(400, "BadRequest", f"unable to parse requirement: {term}")
        neg, key, op, val, setop, setvals = m.groups()
        if op:
            if op in ("=", "=="):
                if labels.get(key) != val:
                    return False
            elif labels.get(key) == val:
                return False
        elif setop:
            vals = {v.strip() for v in setvals.split(",") if v.strip()}
            if setop == "in" and labels.get(key) not in vals:
                return False
            if setop == "notin" and key in labels and labels[key] in vals:
                return False
        elif neg:
            if key in labels:
                return False
        elif key not in labels:
            return False
    return True


def field_selector_matches(sel: str, obj: dict) -> bool:
    for term in filter(None, (sel or "").split(",")):
        if "!=" in term:
            k, v = term.split("!=", 1)
            want, neg = v, True
        else:
            k, v = term.split("=", 1)
            want, neg = v.lstrip("="), False
        cur = obj
        for part in k.strip().split("."):
            cur = cur.get(part) if isinstance(cur, dict) else None
        if (str(cur) == want) == neg:
            return False
    return True


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


# ----------------------------------------------------------------- store
class Store:
    """Objects + an event log for watches.  Thread-safe."""

    def __init__(self, retain_events: int = 20000):
        self.lock = threading.RLock()
        self.cond = threading.Condition(self.lock)
        self.objects: Dict[Tuple, dict] = {}  # (gvr, ns, name) -> obj
        self.rv = 1
        self.events: deque = deque(maxlen=retain_events)  # (rv, gvr, type, obj)
        self.oldest_rv = 1
        self.log_dir: Optional[str] = None
        self.request_count = 0

    def _bump(self) -> str:
        self.rv += 1
        return str(self.rv)

    def _emit(self, gvr, etype, obj):
        if len(self.events) == self.events.maxlen:
            self.oldest_rv = self.events[0][0] + 1
        self.events.append((int(obj["metadata"]["resourceVersion"]), gvr, etype, copy.deepcopy(obj)))
        self.cond.notify_all()

    # -- validation (manifests/crd.yaml openAPIV3Schema)
    @staticmethod
    def _validate(gvr, obj):
        if gvr in CRD_RESOURCES:
            specs = (obj.get("spec") or {}).get("pytorchReplicaSpecs") or {}
            m = specs.get("Master") or {}
            if "replicas" in m and not (1 <= int(m["replicas"]) <= 1):
                raise ApiException(422, "Invalid", "spec.pytorchReplicaSpecs.Master.replicas in body "
                                                   "should be less than or equal to 1")
            w = specs.get("Worker") or {}
            if "replicas" in w and int(w["replicas"]) < 1:
                raise ApiException(422, "Invalid", "spec.pytorchReplicaSpecs.Worker.replicas in body "
                                                   "should be greater than or equal to 1")

    def create(self, gvr, ns, obj) -> dict:
        kind, namespaced, _ = RESOURCES[gvr]
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if not md.get("name"):
            if md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise ApiException(422, "Invalid", "metadata.name: Required value")
        if namespaced:
            if md.get("namespace") and ns and md["namespace"] != ns:
                raise ApiException(400, "BadRequest", "the namespace of the object does not match")
            md["namespace"] = ns or md.get("namespace") or "default"
        else:
            md.pop("namespace", None)
            ns = ""
        self._validate(gvr, obj)
        with self.lock:
            key = (gvr, md.get("namespace", ""), md["name"])
            if key in self.objects:
                raise ApiException(409, "AlreadyExists", f'{gvr[2]} "{md["name"]}" already exists')
            obj.setdefault("kind", kind)
            obj.setdefault("apiVersion", f"{gvr[0]}/{gvr[1]}" if gvr[0] else gvr[1])
            md["uid"] = str(uuid.uuid4())
            md["creationTimestamp"] = _now()
            md["generation"] = 1
            md["resourceVersion"] = self._bump()
            if gvr == ("", "v1", "pods"):
                obj.setdefault("status", {}).setdefault("phase", "Pending")
            self.objects[key] = obj
            self._emit(gvr, "ADDED", obj)
            return copy.deepcopy(obj)

    def get(self, gvr, ns, name) -> dict:
        with self.lock:
            o = self.objects.get((gvr, ns or "", name))
            if o is None:
                raise ApiException(404, "NotFound", f'{gvr[2]} "{name}" not found')
            return copy.deepcopy(o)

    def list(self, gvr, ns, label_sel="", field_sel="") -> Tuple[List[dict], str]:
        with self.lock:
            items = [copy.deepcopy(o) for (g, n, _), o in sorted(self.objects.items(), key=lambda kv: kv[0][1:])
                     if g == gvr and (not ns or n == ns)
                     and label_selector_matches(label_sel, o["metadata"].get("labels"))
                     and field_selector_matches(field_sel, o)]
            return items, str(self.rv)

    def update(self, gvr, ns, name, obj, subresource="") -> dict:
        _, _, has_status = RESOURCES[gvr]
        with self.lock:
            key = (gvr, ns or "", name)
            cur = self.objects.get(key)
            if cur is None:
                raise ApiException(404, "NotFound", f'{gvr[2]} "{name}" not found')
            want_rv = (obj.get("metadata") or {}).get("resourceVersion")
            if want_rv and want_rv != cur["metadata"]["resourceVersion"]:
                raise ApiException(409, "Conflict", f'Operation cannot be fulfilled on {gvr[2]} "{name}": '
                                                    "the object has been modified; please apply your changes "
                                                    "to the latest version and try again")
            new = copy.deepcopy(cur)
            if subresource == "status":
                new["status"] = copy.deepcopy(obj.get("status"))
            else:
                keep_status = new.get("status")
                new = copy.deepcopy(obj)
                md = new.setdefault("metadata", {})
                for k in ("uid", "creationTimestamp", "namespace", "name"):
                    if k in cur["metadata"]:
                        md[k] = cur["metadata"][k]
                if has_status:
                    if keep_status is None:
                        new.pop("status", None)
                    else:
                        new["status"] = keep_status
                if new.get("spec") != cur.get("spec"):
                    md["generation"] = int(cur["metadata"].get("generation", 1)) + 1
                self._validate(gvr, new)
            if new == cur:
                return copy.deepcopy(cur)
            new["metadata"]["resourceVersion"] = self._bump()
            self.objects[key] = new
            self._emit(gvr, "MODIFIED", new)
            return copy.deepcopy(new)

    def patch(self, gvr, ns, name, patch, subresource="") -> dict:
        with self.lock:
            cur = self.get(gvr, ns, name)
            if isinstance(patch, list):  # RFC 6902 JSON patch (subset: add/replace/remove)
                new = apply_json_patch(cur, patch)
            else:
                new = merge_patch(cur, patch)
            new["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            if subresource == "status":
                return self.update(gvr, ns, name, new, "status")
            out = self.update(gvr, ns, name, new)
            if "status" in (patch if isinstance(patch, dict) else {}) and RESOURCES[gvr][2]:
                out = self.update(gvr, ns, name, new, "status")
            return out

    def delete(self, gvr, ns, name) -> dict:
        with self.lock:
            key = (gvr, ns or "", name)
            cur = self.objects.pop(key, None)
            if cur is None:
                raise ApiException(404, "NotFound", f'{gvr[2]} "{name}" not found')
            cur["metadata"]["resourceVersion"] = self._bump()
            cur["metadata"]["deletionTimestamp"] = _now()
            self._emit(gvr, "DELETED", cur)
            self._cascade(cur["metadata"]["uid"])
            return copy.deepcopy(cur)

    def _cascade(self, owner_uid: str):
        victims = [(k, o) for k, o in self.objects.items()
                   if any(r.get("uid") == owner_uid for r in o["metadata"].get("ownerReferences") or [])]
        for (gvr, ns, name), _ in victims:
            if (gvr, ns, name) in self.objects:
                self.delete(gvr, ns, name)

    def events_since(self, rv: int, gvr, ns, label_sel):
        """(events after rv, newest rv) or raises 410 when rv is compacted."""
        if rv and rv < self.oldest_rv - 1:
            raise ApiException(410, "Expired", f"too old resource version: {rv} ({self.oldest_rv})")
        out = []
        for erv, g, etype, obj in self.events:
            if erv <= rv or g != gvr:
                continue
            if ns and obj["metadata"].get("namespace") != ns:
                continue
            if label_sel and not label_selector_matches(label_sel, obj["metadata"].get("labels")):
                continue
            out.append((erv, etype, obj))
        return out


def apply_json_patch(doc, ops):
    doc = copy.deepcopy(doc)
    for op in ops:
        parts = [p.replace("~1", "/").replace("~0", "~") for p in op["path"].split("/")[1:]]
        parent = doc
        for p in parts[:-1]:
            parent = parent[int(p)] if isinstance(parent, list) else parent.setdefault(p, {})
        last = parts[-1]
        if op["op"] in ("add", "replace"):
            if isinstance(parent, list):
                if last == "-":
                    parent.append(op["value"])
                elif op["op"] == "add":
                    parent.insert(int(last), op["value"])
                else:
                    parent[int(last)] = op["value"]
            else:
                parent[last] = op["value"]
        elif op["op"] == "remove":
            if isinstance(parent, list):
                parent.pop(int(last))
            else:
                parent.pop(last, None)
    return doc


# ----------------------------------------------------------------- HTTP layer
_PATH_RE = re.compile(r"^/(?:api/(?P<cv>v1)|apis/(?P<g>[^/]+)/(?P<v>[^/]+))"
                      r"(?:/namespaces/(?P<ns>[^/]+))?/(?P<plural>[^/]+)"
                      r"(?:/(?P<name>[^/]+))?(?:/(?P<sub>status|log))?/?$")


class Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "fake-kube-apiserver/1.0"
    store: Store = None  # set per server class
    auth_tokens = None  # None: no authentication (plain local cluster)

    def log_message(self, fmt, *args):  # quiet
        pass

    def setup(self):
        import ssl
        if isinstance(self.request, ssl.SSLSocket):  # TLS handshake in the handler thread
            self.request.settimeout(10)
            self.request.do_handshake()
            self.request.settimeout(None)
        super().setup()

    def _authenticated(self) -> bool:
        """Bearer token in ``auth_tokens`` or a client certificate the server's client CA
        verified (the API server's token and x509 authenticators)."""
        tokens = self.auth_tokens
        if tokens is None:
            return True
        h = self.headers.get("Authorization") or ""
        if h.startswith("Bearer ") and h[7:].strip() in tokens:
            return True
        try:
            return bool(self.connection.getpeercert())
        except (AttributeError, ValueError):
            return False

    def _send(self, code: int, body, ctype="application/json"):
        data = body if isinstance(body, (bytes, bytearray)) else json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n else b""
        if not raw:
            return None
        return json.loads(raw)

    def _route(self):
        u = urlparse(self.path)
        q = {k: v[-1] for k, v in parse_qs(u.query).items()}
        if u.path in ("/healthz", "/readyz", "/livez"):
            return None, q, u.path
        if u.path == "/version":
            return None, q, u.path
        if u.path in ("/api", "/apis"):
            return None, q, u.path
        m = _PATH_RE.match(u.path)
        if not m:
            raise ApiException(404, "NotFound", f"the server could not find the requested resource ({u.path})")
        d = m.groupdict()
        gvr = ("", "v1", d["plural"]) if d["cv"] else (d["g"], d["v"], d["plural"])
        # /api/v1/namespaces/{ns} itself
        if gvr == ("", "v1", "namespaces") and d["ns"] is None and d["name"]:
            pass
        if gvr not in RESOURCES:
            # /api/v1/namespaces/<name> parses as plural=<name> under ns=None
            if d["cv"] and d["plural"] and d["ns"] is None and d["name"] is None:
                raise ApiException(404, "NotFound", f"the server could not find the requested resource")
            raise ApiException(404, "NotFound", f"the server could not find the requested resource ({d['plural']})")
        return (gvr, d["ns"] or "", d["name"], d["sub"]), q, u.path

    def _handle(self, method):
        st = self.store
        st.request_count += 1
        if not self._authenticated():
            return self._send(401, {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                    "message": "Unauthorized", "reason": "Unauthorized", "code": 401})
        try:
            route, q, path = self._route()
            if route is None:
                if path == "/version":
                    return self._send(200, {"major": "1", "minor": "28", "gitVersion": "v1.28.0-fake"})
                if path in ("/api", "/apis"):
                    return self._send(200, {"kind": "APIVersions", "versions": ["v1"]})
                return self._send(200, b"ok", "text/plain")
            gvr, ns, name, sub = route
            if method == "GET" and sub == "log":
                return self._pod_log(ns, name, q)
            if method == "GET" and not name and q.get("watch") in ("true", "1"):
                return self._watch(gvr, ns, q)
            if method == "GET":
                if name:
                    return self._send(200, st.get(gvr, ns, name))
                items, rv = st.list(gvr, ns, q.get("labelSelector", ""), q.get("fieldSelector", ""))
                kind = RESOURCES[gvr][0]
                api = f"{gvr[0]}/{gvr[1]}" if gvr[0] else gvr[1]
                return self._send(200, {"kind": kind + "List", "apiVersion": api,
                                        "metadata": {"resourceVersion": rv}, "items": items})
            if method == "POST":
                return self._send(201, st.create(gvr, ns, self._body() or {}))
            if method == "PUT":
                return self._send(200, st.update(gvr, ns, name, self._body() or {}, sub or ""))
            if method == "PATCH":
                return self._send(200, st.patch(gvr, ns, name, self._body() or {}, sub or ""))
            if method == "DELETE":
                self._body()
                return self._send(200, st.delete(gvr, ns, name))
            raise ApiException(405, "MethodNotAllowed", method)
        except ApiException as e:
            return self._send(e.code, e.status())
        except (ValueError, KeyError) as e:
            return self._send(400, ApiException(400, "BadRequest", str(e)).status())

    def _pod_log(self, ns, name, q):
        import os
        st = self.store
        st.get(("", "v1", "pods"), ns, name)
        if q.get("follow") in ("true", "1"):
            return self._follow_log(ns, name)
        text = b""
        if st.log_dir:
            p = os.path.join(st.log_dir, f"{ns}_{name}.log")
            if os.path.exists(p):
                with open(p, "rb") as f:
                    text = f.read()
        tail = q.get("tailLines")
        if tail:
            text = b"\n".join(text.splitlines()[-int(tail):]) + b"\n"
        return self._send(200, text, "text/plain")

    def _follow_log(self, ns, name, max_s: float = 3600.0):
        """``follow=true``: stream the container log as it grows; end the response once the
        pod is terminal (Succeeded/Failed) or gone and the file is drained."""
        import os
        st = self.store
        path = os.path.join(st.log_dir, f"{ns}_{name}.log") if st.log_dir else None
        self.send_response(200)
        self.send_header("Content-Type", "text/plain")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        off, deadline = 0, time.time() + max_s
        try:
            while True:
                try:
                    phase = (st.get(("", "v1", "pods"), ns, name).get("status") or {}).get("phase")
                    done = phase in ("Succeeded", "Failed")
                except ApiException:
                    done = True
                data = b""
                if path and os.path.exists(path):
                    with open(path, "rb") as f:
                        f.seek(off)
                        data = f.read()
                if data:
                    off += len(data)
                    self.wfile.write(f"{len(data):x}\r\n".encode() + data + b"\r\n")
                    self.wfile.flush()
                if done or time.time() > deadline:
                    break
                time.sleep(0.05)
            self.wfile.write(b"0\r\n\r\n")
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        self.close_connection = True

    def _watch(self, gvr, ns, q):
        st = self.store
        sel = q.get("labelSelector", "")
        timeout = float(q.get("timeoutSeconds") or 1800)
        rv = int(q.get("resourceVersion") or 0)
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()

        def chunk(obj):
            data = (json.dumps(obj) + "\n").encode()
            self.wfile.write(f"{len(data):x}\r\n".encode() + data + b"\r\n")
            self.wfile.flush()

        deadline = time.time() + timeout
        try:
            with st.lock:
                if rv == 0:
                    # no RV: synthetic ADDED for the current state, then follow
                    items, cur = st.list(gvr, ns, sel)
                    pending = [(int(cur), "ADDED", o) for o in items]
                    rv = int(cur)
                else:
                    pending = st.events_since(rv, gvr, ns, sel)
            while True:
                for erv, etype, obj in pending:
                    chunk({"type": etype, "object": obj})
                    rv = max(rv, erv)
                left = deadline - time.time()
                if left <= 0:
                    break
                with st.lock:
                    pending = st.events_since(rv, gvr, ns, sel)
                    if not pending:
                        st.cond.wait(timeout=min(left, 1.0))
                        pending = st.events_since(rv, gvr, ns, sel)
            self.wfile.write(b"0\r\n\r\n")
        except ApiException as e:
            try:
                chunk({"type": "ERROR", "object": e.status()})
                self.wfile.write(b"0\r\n\r\n")
            except OSError:
                pass
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        self.close_connection = True

    def do_GET(self):
        self._handle("GET")

    def do_POST(self):
        self._handle("POST")

    def do_PUT(self):
        self._handle("PUT")

    def do_PATCH(self):
        self._handle("PATCH")

    def do_DELETE(self):
        self._handle("DELETE")


class FakeApiServer:
    """``with FakeApiServer() as api: api.url`` -- runs in a background thread.

    ``tls``: ``{"cert": path, "key": path, "client_ca": path | None}`` serves HTTPS (the
    client CA enables x509 client-certificate authentication); ``tokens``: accepted bearer
    tokens -- with it every request must present one of them or a verified client
    certificate (401 otherwise); ``url_host``: the host name put in ``url`` / kubeconfigs
    (e.g. ``localhost`` to exercise DNS-name certificate checks)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, log_dir: Optional[str] = None,
                 tls: Optional[dict] = None, tokens=None, url_host: Optional[str] = None):
        import ssl
        self.store = Store()
        self.store.log_dir = log_dir
        handler = type("BoundHandler", (Handler,), {"store": self.store,
                                                    "auth_tokens": None if tokens is None else set(tokens)})
        ctx = None
        if tls:
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(tls["cert"], tls["key"])
            if tls.get("client_ca"):
                ctx.load_verify_locations(tls["client_ca"])
                ctx.verify_mode = ssl.CERT_OPTIONAL
        self.tls = tls

        class Srv(ThreadingHTTPServer):
            daemon_threads = True
            allow_reuse_address = True

            def get_request(self):
                sock, addr = super().get_request()
                if ctx is not None:
                    sock = ctx.wrap_socket(sock, server_side=True, do_handshake_on_connect=False)
                return sock, addr

            def handle_error(self, request, client_address):
                import sys
                exc = sys.exc_info()[1]
                if isinstance(exc, (ssl.SSLError, ConnectionError, TimeoutError, OSError)):
                    return  # failed handshakes (e.g. a client rejecting our certificate) are expected
                super().handle_error(request, client_address)

        self.httpd = Srv((host, port), handler)
        self.host, self.port = self.httpd.server_address[:2]
        self.url_host = url_host or self.host
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="fake-apiserver", daemon=True)

    @property
    def url(self) -> str:
        return f"{'https' if self.tls else 'http'}://{self.url_host}:{self.port}"

    def start(self) -> "FakeApiServer":
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def install_crds(self, manifest_dir: Optional[str] = None):
        """Register the PyTorchJob (and PodGroup) CRDs from manifests/."""
        import os
        import yaml
        root = manifest_dir or os.path.join(os.path.dirname(__file__), "..", "..", "manifests")
        for fn in ("crd.yaml", "podgroup.yaml", "podgroup-volcano.yaml"):
            p = os.path.join(root, fn)
            if not os.path.exists(p):
                continue
            with open(p) as f:
                for doc in yaml.safe_load_all(f):
                    if doc and doc.get("kind") == "CustomResourceDefinition":
                        try:
                            self.store.create(("apiextensions.k8s.io", "v1", "customresourcedefinitions"), "", doc)
                        except ApiException:
                            pass

    def write_kubeconfig(self, path: str, namespace: str = "default", token: Optional[str] = "fake-token",
                         ca_file: Optional[str] = None, client_cert: Optional[str] = None,
                         client_key: Optional[str] = None, server: Optional[str] = None,
                         tls_server_name: Optional[str] = None, exec_plugin: Optional[dict] = None) -> str:
        """kubeconfig for this server; PEM files are embedded as ``*-data`` (base64)."""
        import base64

        def b64(p):
            with open(p, "rb") as f:
                return base64.b64encode(f.read()).decode()
        cluster = {"server": server or self.url}
        if ca_file:
            cluster["certificate-authority-data"] = b64(ca_file)
        if tls_server_name:
            cluster["tls-server-name"] = tls_server_name
        user = {}
        if token:
            user["token"] = token
        if client_cert:
            user["client-certificate-data"] = b64(client_cert)
            user["client-key-data"] = b64(client_key)
        if exec_plugin:
            user["exec"] = exec_plugin
        cfg = {"apiVersion": "v1", "kind": "Config", "current-context": "fake",
               "clusters": [{"name": "fake", "cluster": cluster}],
               "users": [{"name": "fake", "user": user}],
               "contexts": [{"name": "fake", "context": {"cluster": "fake", "user": "fake",
                                                         "namespace": namespace}}]}
        with open(path, "w") as f:
            json.dump(cfg, f)
        return path


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser(description="fake Kubernetes API server")
    p.add_argument("--port", type=int, default=8001)
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--log-dir", default=None)
    a = p.parse_args(argv)
    srv = FakeApiServer(a.host, a.port, a.log_dir).start()
    srv.install_crds()
    print(f"fake apiserver listening on {srv.url}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()


if __name__ == "__main__":
    main()
