"""docs/monitoring.md quotes only metric names the operator and the worker really export.

The operator: the real ``pytorch-operator`` binary on the fake API server, scraped over HTTP.
The worker: ``harness.mnist`` run in-process on the CPU (torch kernels, world 1) with
``--metrics-port 0``, scraped after its epoch (the endpoint thread outlives ``run``).
"""
import json
import re
import urllib.request
from pathlib import Path

GUIDE = Path(__file__).resolve().parent.parent / "docs" / "monitoring.md"


def _names(prefix: str):
    # metric names only: module paths (pytorch_operator_amd/...) are not metrics
    names = set(re.findall(prefix + r"[a-z_]+(?![a-z_./])", GUIDE.read_text())) - {"pytorch_operator_amd"}
    return {re.sub(r"_(bucket|sum|count)$", "", n) for n in names}


def _exported(text: str):
    return {ln.split("{")[0].split(" ")[0] for ln in text.splitlines() if ln and not ln.startswith("#")}


def test_guide_operator_metrics_are_exported(tmp_path):
    from pytorch_operator_amd.cluster.local import LocalCluster
    quoted = _names("pytorch_operator_")
    assert {"pytorch_operator_jobs_created_total", "pytorch_operator_is_leader",
            "pytorch_operator_sync_duration_seconds"} <= quoted
    with LocalCluster(workdir=str(tmp_path / "c")) as c:
        c.wait_operator_ready()
        text = c.metrics()
    exported = {re.sub(r"_(bucket|sum|count)$", "", n) for n in _exported(text)}
    assert quoted <= exported, quoted - exported


def test_guide_worker_metrics_are_exported(tmp_path, capsys, monkeypatch):
    from pytorch_operator_amd.harness import mnist
    from pytorch_operator_amd.utils.worker_metrics import METRICS
    for k in ("WORLD_SIZE", "RANK", "PTO_WORKER_METRICS_PORT"):
        monkeypatch.delenv(k, raising=False)
    quoted = _names("pto_worker_")
    assert quoted == set(METRICS), quoted ^ set(METRICS)
    mnist.main(["--no-cuda", "--dataset-size", "640", "--test-size", "200", "--log-interval", "5",
                "--synthetic", "--dir", str(tmp_path / "tb"), "--metrics-port", "0"])
    out = capsys.readouterr().out
    ev = [json.loads(x) for x in out.splitlines() if x.startswith('{"event"')]
    port = next(e["port"] for e in ev if e["event"] == "metrics_endpoint")
    text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
    exported = _exported(text)
    # every series the training run could produce on a CPU world-1 job (no xGMI path, so no
    # exchange-error series; no gradient-path race, so no trial series) is present; every metric is at least described
    assert quoted - {"pto_worker_grad_exchange_errors", "pto_worker_samples_per_second",
                     "pto_worker_step_seconds", "pto_worker_allreduce_trial_ms"} <= exported, quoted - exported
    assert all(f"# TYPE {n} " in text for n in quoted)
    steps = float(re.search(r"^pto_worker_steps_total (\S+)$", text, re.M).group(1))
    assert steps == 10  # 640 / 64
    assert 'kernels="torch"' in text and 'phase="first_step"' in text
