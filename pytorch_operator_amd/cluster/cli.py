"""``python -m pytorch_operator_amd.cluster`` -- run a local cluster and drive it kubectl-style.

    python -m pytorch_operator_amd.cluster up [--gpus 0 1 ...] [--workdir DIR] [--port 8001]
        starts the fake API server, the kubelet emulator and the native operator, writes
        DIR/kubeconfig.json and serves until interrupted;
    python -m pytorch_operator_amd.cluster apply -f job.yaml      [--kubeconfig K]
    python -m pytorch_operator_amd.cluster get pytorchjobs|pods|services [-n NS]
    python -m pytorch_operator_amd.cluster describe pytorchjob NAME
    python -m pytorch_operator_amd.cluster logs POD
    python -m pytorch_operator_amd.cluster delete pytorchjob NAME

``get pytorchjobs`` prints the CRD's printer columns (NAME, STATE = last condition, AGE),
as ``kubectl get pytorchjobs`` does with manifests/crd.yaml.  The client commands work
against any API server the kubeconfig points at.
"""
from __future__ import annotations

import argparse
import calendar
import json
import os
import sys
import time

from kubeflow.pytorchjob.rest import PODS, PYTORCHJOBS, SERVICES, ApiException, KubeRest, load_kube_config

_KINDS = {"pytorchjob": PYTORCHJOBS, "pytorchjobs": PYTORCHJOBS, "ptj": PYTORCHJOBS,
          "pod": PODS, "pods": PODS, "service": SERVICES, "services": SERVICES, "svc": SERVICES}
_DEFAULT_WORKDIR = os.path.join(os.path.expanduser("~"), ".pytorch-operator-amd", "cluster")


def _age(ts: str) -> str:
    try:
        t = calendar.timegm(time.strptime(ts, "%Y-%m-%dT%H:%M:%SZ"))
    except (TypeError, ValueError):
        return "?"
    s = int(time.time() - t)
    for unit, n in (("d", 86400), ("h", 3600), ("m", 60)):
        if s >= n:
            return f"{s // n}{unit}"
    return f"{s}s"


def _client(a) -> KubeRest:
    path = a.kubeconfig or os.environ.get("KUBECONFIG") or os.path.join(_DEFAULT_WORKDIR, "kubeconfig.json")
    return KubeRest(load_kube_config(path))


def cmd_up(a) -> int:
    from .local import LocalCluster
    os.makedirs(a.workdir, exist_ok=True)
    c = LocalCluster(workdir=a.workdir, gpus=a.gpus, verbose=a.verbose)
    if a.port:
        from .fake_apiserver import FakeApiServer
        c.api = FakeApiServer(port=a.port, log_dir=c.log_dir)
    c.start()
    c.wait_operator_ready()
    print(f"cluster up: api {c.api.url}  kubeconfig {c.kubeconfig}  operator metrics "
          f"http://127.0.0.1:{c.monitoring_port}/metrics  gpus {a.gpus or []}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        pass
    finally:
        c.stop()
    return 0


def cmd_apply(a) -> int:
    import yaml
    r = _client(a)
    with open(a.filename) as f:
        docs = [d for d in yaml.safe_load_all(f) if d]
    for d in docs:
        gvr = _KINDS[d["kind"].lower()]
        ns = d.get("metadata", {}).get("namespace") or a.namespace
        try:
            r.create(gvr, d, ns)
            print(f"{d['kind'].lower()}/{d['metadata']['name']} created")
        except ApiException as e:
            if e.status != 409:
                raise
            cur = r.get(gvr, d["metadata"]["name"], ns)
            d.setdefault("metadata", {})["resourceVersion"] = cur["metadata"]["resourceVersion"]
            r.replace(gvr, d["metadata"]["name"], d, ns)
            print(f"{d['kind'].lower()}/{d['metadata']['name']} configured")
    return 0


def cmd_get(a) -> int:
    r = _client(a)
    gvr = _KINDS[a.kind]
    items = [r.get(gvr, a.name, a.namespace)] if a.name else r.list(gvr, a.namespace)["items"]
    if a.output == "json":
        print(json.dumps(items if not a.name else items[0], indent=1))
        return 0
    if gvr == PYTORCHJOBS:
        rows = [("NAME", "STATE", "AGE")]
        for j in items:
            conds = (j.get("status") or {}).get("conditions") or []
            rows.append((j["metadata"]["name"], conds[-1]["type"] if conds else "",
                         _age(j["metadata"].get("creationTimestamp"))))
    elif gvr == PODS:
        rows = [("NAME", "STATUS", "RESTARTS", "AGE")]
        for p in items:
            cs = (p.get("status") or {}).get("containerStatuses") or []
            rows.append((p["metadata"]["name"], p.get("status", {}).get("phase", ""),
                         str(sum(c.get("restartCount", 0) for c in cs)), _age(p["metadata"].get("creationTimestamp"))))
    else:
        rows = [("NAME", "TYPE", "CLUSTER-IP", "PORT(S)", "AGE")]
        for s in items:
            spec = s.get("spec", {})
            ports = ",".join(f"{p.get('port')}/{p.get('protocol', 'TCP')}" for p in spec.get("ports") or [])
            rows.append((s["metadata"]["name"], spec.get("type", "ClusterIP"), spec.get("clusterIP", ""), ports,
                         _age(s["metadata"].get("creationTimestamp"))))
    widths = [max(len(str(r[i])) for r in rows) + 3 for i in range(len(rows[0]))]
    for row in rows:
        print("".join(str(v).ljust(w) for v, w in zip(row, widths)).rstrip())
    return 0


def cmd_describe(a) -> int:
    r = _client(a)
    obj = r.get(_KINDS[a.kind], a.name, a.namespace)
    print(json.dumps(obj, indent=2))
    return 0


def cmd_logs(a) -> int:
    sys.stdout.write(_client(a).pod_log(a.pod, a.namespace, tail_lines=a.tail))
    return 0


def cmd_delete(a) -> int:
    _client(a).delete(_KINDS[a.kind], a.name, a.namespace)
    print(f"{a.kind}/{a.name} deleted")
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="python -m pytorch_operator_amd.cluster", description=__doc__.split("\n")[0])
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("-n", "--namespace", default="default")
    sub = p.add_subparsers(dest="cmd", required=True)
    up = sub.add_parser("up")
    up.add_argument("--gpus", type=int, nargs="*", default=None)
    up.add_argument("--workdir", default=_DEFAULT_WORKDIR)
    up.add_argument("--port", type=int, default=0)
    up.add_argument("--verbose", action="store_true")
    ap = sub.add_parser("apply")
    ap.add_argument("-f", "--filename", required=True)
    g = sub.add_parser("get")
    g.add_argument("kind", choices=sorted(_KINDS))
    g.add_argument("name", nargs="?")
    g.add_argument("-o", "--output", choices=["table", "json"], default="table")
    d = sub.add_parser("describe")
    d.add_argument("kind", choices=sorted(_KINDS))
    d.add_argument("name")
    lg = sub.add_parser("logs")
    lg.add_argument("pod")
    lg.add_argument("--tail", type=int, default=None)
    de = sub.add_parser("delete")
    de.add_argument("kind", choices=sorted(_KINDS))
    de.add_argument("name")
    a = p.parse_args(argv)
    return {"up": cmd_up, "apply": cmd_apply, "get": cmd_get, "describe": cmd_describe, "logs": cmd_logs,
            "delete": cmd_delete}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
