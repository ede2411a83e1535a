#!/usr/bin/env python3
"""Emit the PyTorchJob OpenAPI v3 / JSON Schema from the SDK model tables.

The reference generates OpenAPI definitions from its Go types (pkg/apis/pytorch/v1/
openapi_generated.go) and feeds them to swagger-codegen for the SDK.  Here the SDK's
declarative field tables are the single source: this tool turns them into
``docs/pytorchjob.schema.json`` (definitions keyed like the reference's swagger:
``v1.PyTorchJob``, ``v1.PyTorchJobSpec``, ...).  ``--check`` fails if the file is stale.
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdk", "python")]

from kubeflow.pytorchjob import models  # noqa: E402

OURS = ["V1PyTorchJob", "V1PyTorchJobSpec", "V1PyTorchJobList", "V1ReplicaSpec", "V1ReplicaStatus", "V1JobStatus",
        "V1JobCondition"]
PRIM = {"str": {"type": "string"}, "int": {"type": "integer", "format": "int32"}, "bool": {"type": "boolean"},
        "float": {"type": "number"}, "object": {"type": "object"}, "datetime": {"type": "string", "format": "date-time"},
        "V1Time": {"type": "string", "format": "date-time"}}
K8S = {"V1ObjectMeta": "io.k8s.apimachinery.pkg.apis.meta.v1.ObjectMeta",
       "V1ListMeta": "io.k8s.apimachinery.pkg.apis.meta.v1.ListMeta",
       "V1PodTemplateSpec": "io.k8s.api.core.v1.PodTemplateSpec"}


def ref(t: str) -> dict:
    m = re.match(r"list\[(.*)\]$", t)
    if m:
        return {"type": "array", "items": ref(m.group(1))}
    m = re.match(r"dict\(([^,]*), (.*)\)$", t)
    if m:
        return {"type": "object", "additionalProperties": ref(m.group(2))}
    if t in PRIM:
        return dict(PRIM[t])
    if t in K8S:
        return {"$ref": f"#/definitions/{K8S[t]}"}
    return {"$ref": "#/definitions/v1." + t[2:]}


def schema() -> dict:
    defs = {}
    for name in OURS:
        cls = getattr(models, name)
        props = {cls.attribute_map[a]: ref(t) for a, t in cls.swagger_types.items()}
        d = {"type": "object", "properties": props}
        req = [cls.attribute_map[a] for a in cls._required]
        if req:
            d["required"] = req
        defs["v1." + name[2:]] = d
    # the CRD's validation rules (manifests/crd.yaml)
    spec = defs["v1.ReplicaSpec"]["properties"]
    spec["restartPolicy"]["enum"] = ["Always", "OnFailure", "Never", "ExitCode"]
    defs["v1.PyTorchJobSpec"]["properties"]["cleanPodPolicy"]["enum"] = ["All", "Running", "None"]
    return {"swagger": "2.0", "info": {"title": "pytorch", "version": "v1"}, "paths": {}, "definitions": defs}


def main(argv=None):
    out = os.path.join(ROOT, "docs", "pytorchjob.schema.json")
    text = json.dumps(schema(), indent=2, sort_keys=True) + "\n"
    if "--check" in (argv or sys.argv[1:]):
        return 0 if os.path.exists(out) and open(out).read() == text else 1
    with open(out, "w") as f:
        f.write(text)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
