"""Local cluster: fake API server, kubelet emulator, LocalCluster, kubectl-like CLI.

Everything here talks to the API server through the SDK's stdlib transport
(``kubeflow.pytorchjob.rest``, distribution ``kubeflow-pytorchjob``).  In a repo checkout
without the SDK installed, its in-repo source directory is put on ``sys.path`` here, once.
"""
import os
import sys

try:
    import kubeflow.pytorchjob.rest  # noqa: F401
except ImportError:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sdk", "python"))
