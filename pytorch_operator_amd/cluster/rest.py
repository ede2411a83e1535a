"""Kubernetes REST client of the local cluster: the SDK's stdlib transport.

The transport lives in the standalone SDK (``sdk/python/kubeflow/pytorchjob/rest.py``,
distribution ``kubeflow-pytorchjob``); the fake API server tests, the kubelet emulator
and the benchmarks use the same code.  When the SDK is not installed, its in-repo source
directory is put on ``sys.path``.
"""
from __future__ import annotations

import os
import sys

try:
    from kubeflow.pytorchjob import rest as _rest
except ImportError:  # repo checkout without the SDK installed
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sdk", "python"))
    from kubeflow.pytorchjob import rest as _rest

ApiException = _rest.ApiException
GVR = _rest.GVR
KubeRest = _rest.KubeRest
Configuration = _rest.Configuration
load_kube_config = _rest.load_kube_config
load_incluster_config = _rest.load_incluster_config
PODS, SERVICES, EVENTS, NAMESPACES = _rest.PODS, _rest.SERVICES, _rest.EVENTS, _rest.NAMESPACES
LEASES, PYTORCHJOBS, PODGROUPS, CRDS = _rest.LEASES, _rest.PYTORCHJOBS, _rest.PODGROUPS, _rest.CRDS
VOLCANO_PODGROUPS = _rest.VOLCANO_PODGROUPS

__all__ = ["ApiException", "GVR", "KubeRest", "Configuration", "load_kube_config", "load_incluster_config",
           "PODS", "SERVICES", "EVENTS", "NAMESPACES", "LEASES", "PYTORCHJOBS", "PODGROUPS", "VOLCANO_PODGROUPS", "CRDS"]
