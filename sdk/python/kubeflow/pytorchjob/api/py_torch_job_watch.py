"""Watch PyTorchJobs and print a NAME / STATE / TIME table (reference api/py_torch_job_watch.py).

The reference retries the whole watch up to 20 times, 1 s apart (``retrying``); this does
the same without the dependency, resuming from the last seen resourceVersion.
"""
import sys
import time

from kubeflow.pytorchjob.constants import constants
from kubeflow.pytorchjob.utils import utils
from kubeflow.pytorchjob import rest as k8s

_JOBS = k8s.GVR(constants.PYTORCHJOB_GROUP, constants.PYTORCHJOB_VERSION, constants.PYTORCHJOB_PLURAL)
_COLS = (("NAME", 30), ("STATE", 20), ("TIME", 30))


def _row(values, out):
    out.write("".join(str(v).ljust(w) for v, (_, w) in zip(values, _COLS)).rstrip() + "\n")
    out.flush()


def watch(name=None, namespace=None, timeout_seconds=600, api=None, out=None, max_attempts=20):
    """Stream job state changes until ``name`` finishes (or the timeout)."""
    if namespace is None:
        namespace = utils.get_default_target_namespace()
    api = api or k8s.KubeRest(k8s.load_kube_config())
    out = out or sys.stdout
    _row([c for c, _ in _COLS], out)
    deadline = time.monotonic() + timeout_seconds
    rv = ""
    attempts = 0
    while time.monotonic() < deadline:
        try:
            for _, job in api.watch(_JOBS, namespace, resource_version=rv,
                                    timeout_seconds=max(1, int(deadline - time.monotonic()))):
                rv = job.get("metadata", {}).get("resourceVersion", rv)
                job_name = job["metadata"]["name"]
                if name and name != job_name:
                    continue
                conds = (job.get("status") or {}).get("conditions") or []
                status = conds[-1].get("type", "") if conds else ""
                update_time = conds[-1].get("lastTransitionTime", "") if conds else ""
                _row([job_name, status, update_time], out)
                if name == job_name and status in ("Succeeded", "Failed"):
                    return job
        except (k8s.ApiException, OSError):
            attempts += 1
            if attempts >= max_attempts:
                raise
            if isinstance(sys.exc_info()[1], k8s.ApiException) and sys.exc_info()[1].status == 410:
                rv = ""
            time.sleep(1.0)
    return None
