"""Prometheus text endpoint of the MNIST DDP worker (``harness/mnist.py --metrics-port``).

The reference worker only prints log lines and writes TensorBoard scalars
(examples/mnist/mnist.py:44-49,65); its monitoring guide (docs/monitoring/README.md) therefore
watches pods from the outside (cAdvisor) and the operator's counters.  On an MI355X node the
numbers a user wants next to those are the worker's own: training throughput, step-time
percentiles, the first-step timestamp (BASELINE's create-to-first-step metric) and whether the
xGMI gradient exchange flagged an error.  This serves them in the Prometheus text format from a
daemon thread (stdlib only: the worker image needs no client library); ``docs/monitoring.md``
has the scrape config and queries.
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Optional, Tuple

# name -> (type, help); the guide quotes these names and tests/test_monitoring.py pins them
METRICS: Dict[str, Tuple[str, str]] = {
    "pto_worker_info": ("gauge", "Worker identity (labels: rank, world_size, backend, kernels, grad_allreduce); value 1"),
    "pto_worker_steps_total": ("counter", "Training steps completed by this rank"),
    "pto_worker_samples_per_second": ("gauge", "Job-wide training samples/s over the last log interval (rank-local clock)"),
    "pto_worker_step_seconds": ("gauge", "Per-step time of the last log interval (device events)"),
    "pto_worker_loss": ("gauge", "Training loss of the last logged batch"),
    "pto_worker_accuracy": ("gauge", "Test accuracy after the last epoch"),
    "pto_worker_first_step_unix_seconds": ("gauge", "Wall-clock time of this rank's first optimizer step"),
    "pto_worker_startup_phase_seconds": ("gauge", "Process start -> first step, per phase (label: phase)"),
    "pto_worker_allreduce_trial_ms": ("gauge", "Start-up race: per-step ms of each DDP gradient-path candidate (label: candidate)"),
    "pto_worker_grad_exchange_errors": ("gauge", "Non-zero when the xGMI gradient exchange timed out (the worker then exits 138)"),
}


class WorkerMetrics:
    def __init__(self):
        self._lock = threading.Lock()
        self._v: Dict[str, Dict[Tuple[Tuple[str, str], ...], float]] = {k: {} for k in METRICS}
        self._srv: Optional[ThreadingHTTPServer] = None

    def set(self, name: str, value: float, replace: bool = False, **labels) -> None:
        """Set one series; ``replace`` drops the metric's other series first (info metrics)."""
        if name not in METRICS:
            raise KeyError(name)
        with self._lock:
            if replace:
                self._v[name].clear()
            self._v[name][tuple(sorted((k, str(v)) for k, v in labels.items()))] = float(value)

    def inc(self, name: str, value: float = 1.0, **labels) -> None:
        key = tuple(sorted((k, str(v)) for k, v in labels.items()))
        with self._lock:
            self._v[name][key] = self._v[name].get(key, 0.0) + float(value)

    def exposition(self) -> str:
        out = []
        with self._lock:
            for name, (typ, help_) in METRICS.items():
                out.append(f"# HELP {name} {help_}\n# TYPE {name} {typ}\n")
                for key, v in sorted(self._v[name].items()):
                    lab = ",".join(f'{k}="{val}"' for k, val in key)
                    out.append(f"{name}{{{lab}}} {v!r}\n" if lab else f"{name} {v!r}\n")
        return "".join(out)

    def serve(self, port: int, addr: str = "0.0.0.0") -> int:
        """Serve ``/metrics`` on ``port`` (0: an ephemeral port) from a daemon thread; returns the port."""
        metrics = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802 -- http.server API
                if self.path.split("?")[0] != "/metrics":
                    self.send_error(404)
                    return
                body = metrics.exposition().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):  # quiet
                pass

        self._srv = ThreadingHTTPServer((addr, port), H)
        threading.Thread(target=self._srv.serve_forever, name="worker-metrics", daemon=True).start()
        return self._srv.server_address[1]

    def close(self) -> None:
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None
