"""PyTorchJobClient: create / get / patch / delete / wait / status / pods / logs.

Method-for-method the reference client (sdk/python/kubeflow/pytorchjob/api/
py_torch_job_client.py): same names, arguments, defaults and error behaviour
(``RuntimeError`` wrapping API errors; ``wait_for_condition`` raising on timeout).
Differences: jobs may be V1PyTorchJob models *or* plain dicts; ``get_logs`` also
returns ``{pod: log}`` (with ``follow=True`` each pod's log is streamed until its
container terminates, as ``read_namespaced_pod_log(follow=True)`` does); ``wait_for_condition`` sleeps at most the remaining timeout
(the reference rounds timeout/polling_interval and can overshoot); and the client can
be pointed at an explicit ``Configuration`` (used with the local test cluster).
"""
import logging
import time

from kubeflow.pytorchjob.api_client import ApiClient
from kubeflow.pytorchjob.constants import constants
from kubeflow.pytorchjob.utils import utils
from kubeflow.pytorchjob import rest as k8s

from .py_torch_job_watch import watch as pytorchjob_watch

logging.basicConfig(format="%(message)s")
logging.getLogger().setLevel(logging.INFO)

_JOBS = k8s.GVR(constants.PYTORCHJOB_GROUP, constants.PYTORCHJOB_VERSION, constants.PYTORCHJOB_PLURAL)


class PyTorchJobClient(object):
    def __init__(self, config_file=None, context=None, client_configuration=None, persist_config=True):
        """
        :param config_file: kubeconfig file, defaults to $KUBECONFIG / ~/.kube/config
        :param context: kubeconfig context
        :param client_configuration: a ``Configuration`` to use as-is (skips kubeconfig)
        :param persist_config: accepted for API compatibility
        """
        del persist_config
        if client_configuration is not None:
            cfg = client_configuration
        elif config_file or not utils.is_running_in_k8s():
            cfg = k8s.load_kube_config(config_file=config_file, context=context)
        else:
            cfg = k8s.load_incluster_config()
        self.api = k8s.KubeRest(cfg, timeout=constants.APISERVER_TIMEOUT)
        self.api_client = ApiClient(cfg)

    def _body(self, pytorchjob):
        return self.api_client.sanitize_for_serialization(pytorchjob)

    def create(self, pytorchjob, namespace=None):
        """Create the PyTorchJob; returns the created object (dict)."""
        if namespace is None:
            namespace = utils.set_pytorchjob_namespace(pytorchjob)
        try:
            return self.api.create(_JOBS, self._body(pytorchjob), namespace)
        except k8s.ApiException as e:
            raise RuntimeError("Exception when calling CustomObjectsApi->create_namespaced_custom_object:"
                               " %s\n" % e)

    def get(self, name=None, namespace=None, watch=False, timeout_seconds=600):  # pylint: disable=inconsistent-return-statements
        """Get one job (``name``) or the namespace's job list; ``watch`` streams a status table."""
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        if watch:
            pytorchjob_watch(name=name, namespace=namespace, timeout_seconds=timeout_seconds, api=self.api)
            return None
        try:
            if name:
                return self.api.get(_JOBS, name, namespace)
            return self.api.list(_JOBS, namespace)
        except k8s.ApiException as e:
            verb = "get_namespaced_custom_object" if name else "list_namespaced_custom_object"
            raise RuntimeError("Exception when calling CustomObjectsApi->%s: %s\n" % (verb, e))
        except OSError as e:
            raise RuntimeError("There was a problem to get PyTorchJob {0} in namespace {1}. Exception: {2} "
                               .format(name, namespace, e))

    def patch(self, name, pytorchjob, namespace=None):
        """Merge-patch an existing job."""
        if namespace is None:
            namespace = utils.set_pytorchjob_namespace(pytorchjob)
        try:
            return self.api.patch(_JOBS, name, self._body(pytorchjob), namespace)
        except k8s.ApiException as e:
            raise RuntimeError("Exception when calling CustomObjectsApi->patch_namespaced_custom_object:"
                               " %s\n" % e)

    def delete(self, name, namespace=None):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        try:
            return self.api.delete(_JOBS, name, namespace)
        except k8s.ApiException as e:
            raise RuntimeError("Exception when calling CustomObjectsApi->delete_namespaced_custom_object:"
                               " %s\n" % e)

    def wait_for_job(self, name, namespace=None, watch=False, timeout_seconds=600, polling_interval=30,
                     status_callback=None):  # pylint: disable=inconsistent-return-statements
        """Wait until the job is Succeeded or Failed."""
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        if watch:
            pytorchjob_watch(name=name, namespace=namespace, timeout_seconds=timeout_seconds, api=self.api)
            return None
        return self.wait_for_condition(name, ["Succeeded", "Failed"], namespace=namespace,
                                       timeout_seconds=timeout_seconds, polling_interval=polling_interval,
                                       status_callback=status_callback)

    def wait_for_condition(self, name, expected_condition, namespace=None, timeout_seconds=600,
                           polling_interval=30, status_callback=None):
        """Poll until any condition in ``expected_condition`` appears; returns the job."""
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        deadline = time.monotonic() + timeout_seconds
        pytorchjob = None
        while True:
            pytorchjob = self.get(name, namespace=namespace)
            if pytorchjob:
                if status_callback:
                    status_callback(pytorchjob)
                conditions = (pytorchjob.get("status") or {}).get("conditions") or []
                for c in conditions:
                    if c.get("type", "") in expected_condition:
                        return pytorchjob
            left = deadline - time.monotonic()
            if left <= 0:
                break
            time.sleep(min(polling_interval, left))
        raise RuntimeError(
            "Timeout waiting for PyTorchJob {0} in namespace {1} to enter one of the "
            "conditions {2}.".format(name, namespace, expected_condition), pytorchjob)

    def get_job_status(self, name, namespace=None):
        """Type of the job's last condition (Created/Running/Restarting/Succeeded/Failed)."""
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        pytorchjob = self.get(name, namespace=namespace)
        conditions = (pytorchjob.get("status") or {}).get("conditions") or []
        if not conditions:
            return ""
        return conditions[-1].get("type", "")

    def is_job_running(self, name, namespace=None):
        return self.get_job_status(name, namespace=namespace).lower() == "running"

    def is_job_succeeded(self, name, namespace=None):
        return self.get_job_status(name, namespace=namespace).lower() == "succeeded"

    def get_pod_names(self, name, namespace=None, master=False, replica_type=None,
                      replica_index=None):  # pylint: disable=inconsistent-return-statements
        """Set of the job's pod names (optionally only master / one type / one index)."""
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        labels = utils.get_labels(name, master=master, replica_type=replica_type, replica_index=replica_index)
        try:
            resp = self.api.list(k8s.PODS, namespace, label_selector=utils.to_selector(labels))
        except k8s.ApiException as e:
            raise RuntimeError("Exception when calling CoreV1Api->list_namespaced_pod: %s\n" % e)
        pod_names = [p["metadata"]["name"] for p in resp.get("items", []) if p.get("metadata", {}).get("name")]
        if not pod_names:
            logging.warning("Not found Pods of the PyTorchJob %s with the labels %s.", name, labels)
            return None
        return set(pod_names)

    def get_logs(self, name, namespace=None, master=True, replica_type=None, replica_index=None,
                 follow=False):
        """Log the (master's, by default) pod logs; returns {pod_name: log_text}.

        ``follow``: stream each pod's log until its container terminates; complete lines are
        logged as they arrive."""
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        pod_names = self.get_pod_names(name, namespace=namespace, master=master, replica_type=replica_type,
                                       replica_index=replica_index)
        if not pod_names:
            raise RuntimeError("Not found Pods of the PyTorchJob {} in namespace {}".format(name, namespace))
        out = {}
        for pod in sorted(pod_names):
            try:
                if follow:
                    pending = [b""]

                    def on_chunk(data, pod=pod, pending=pending):
                        pending[0] += data
                        *lines, pending[0] = pending[0].split(b"\n")
                        for line in lines:
                            logging.info("[%s] %s", pod, line.decode(errors="replace"))
                    out[pod] = self.api.pod_log(pod, namespace, follow=True, on_chunk=on_chunk)
                    if pending[0]:
                        logging.info("[%s] %s", pod, pending[0].decode(errors="replace"))
                    continue
                out[pod] = self.api.pod_log(pod, namespace)
            except k8s.ApiException as e:
                raise RuntimeError("Exception when calling CoreV1Api->read_namespaced_pod_log: %s\n" % e)
            logging.info("The logs of Pod %s:\n %s", pod, out[pod])
        return out
