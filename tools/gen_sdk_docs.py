#!/usr/bin/env python3
"""Generate the SDK reference docs (sdk/python/docs/*.md) from the code itself: one page per
model from its declarative field table (models/*.py ``_fields`` / ``_required``) and one page
for ``PyTorchJobClient`` from its method signatures and docstrings.  Re-run after changing a
model or the client; tests/test_sdk.py checks the committed pages are current."""
from __future__ import annotations

import inspect
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sdk", "python"))
OUT = os.path.join(ROOT, "sdk", "python", "docs")

MODELS = ["V1JobCondition", "V1JobStatus", "V1PyTorchJob", "V1PyTorchJobList", "V1PyTorchJobSpec",
          "V1ReplicaSpec", "V1ReplicaStatus", "V1Time"]
DESCR = {
    "V1JobCondition": "One observed state of a job (Created, Running, Restarting, Succeeded, Failed).",
    "V1JobStatus": "Observed status of a PyTorchJob: conditions, per-replica-type counts and timestamps.",
    "V1PyTorchJob": "The kubeflow.org/v1 PyTorchJob custom resource.",
    "V1PyTorchJobList": "A list of PyTorchJobs (the LIST response of the API server).",
    "V1PyTorchJobSpec": "Desired state: replica specs (Master/Worker), clean-pod policy, backoff and deadlines.",
    "V1ReplicaSpec": "Replica count, restart policy and pod template of one replica type.",
    "V1ReplicaStatus": "Active / succeeded / failed pod counts of one replica type.",
    "V1Time": "An RFC 3339 timestamp as serialised by Kubernetes.",
}


def _link(t: str) -> str:
    names = re.findall(r"V1[A-Za-z]+", t)
    for n in names:
        if n in MODELS:
            t = t.replace(n, f"[{n}]({n}.md)")
    return t


def model_page(name: str) -> str:
    import kubeflow.pytorchjob as sdk
    cls = getattr(sdk, name)
    lines = [f"# {name}", "", DESCR.get(name, ""), "", "## Properties", "",
             "Name | JSON key | Type | Notes", "---- | -------- | ---- | -----"]
    for attr, key, typ in cls._fields:
        note = "required" if attr in cls._required else "[optional]"
        lines.append(f"**{attr}** | `{key}` | {_link(typ)} | {note}")
    lines += ["", "```python", f"from kubeflow.pytorchjob import {name}", f"obj = {name}(" +
              ", ".join(f"{a}=..." for a, _, _ in cls._fields[:2]) + ")",
              "obj.to_dict()  # snake_case keys; the client serialises with the JSON keys", "```", "",
              "[[Back to README]](../README.md)", ""]
    return "\n".join(lines)


def client_page() -> str:
    from kubeflow.pytorchjob import PyTorchJobClient
    lines = ["# PyTorchJobClient", "",
             "Client for the kubeflow.org/v1 `pytorchjobs` resource and its pods "
             "(`kubeflow.pytorchjob.api.py_torch_job_client`).  Construction takes the usual "
             "kubeconfig arguments; transport is the SDK's own stdlib REST client.", "",
             "Method | Signature", "------ | ---------"]
    meths = [(n, m) for n, m in inspect.getmembers(PyTorchJobClient, inspect.isfunction)
             if not n.startswith("_") or n == "__init__"]
    for n, m in meths:
        lines.append(f"[**{n}**](#{n.strip('_').lower()}) | `{n}{inspect.signature(m)}`")
    lines.append("")
    for n, m in meths:
        lines += [f"## {n}", "", "```python", f"PyTorchJobClient.{n}{inspect.signature(m)}", "```", ""]
        doc = inspect.getdoc(m)
        lines += [doc if doc else "(no docstring)", ""]
    lines += ["[[Back to README]](../README.md)", ""]
    return "\n".join(lines)


def pages() -> dict:
    out = {f"{n}.md": model_page(n) for n in MODELS}
    out["PyTorchJobClient.md"] = client_page()
    return out


def main() -> int:
    os.makedirs(OUT, exist_ok=True)
    for fn, text in pages().items():
        with open(os.path.join(OUT, fn), "w") as f:
            f.write(text)
        print("wrote", os.path.join("sdk/python/docs", fn))
    return 0


if __name__ == "__main__":
    sys.exit(main())
