"""kubectl-style CLI against a running local cluster (apply -> get -> logs -> delete)."""
import io
import time
from contextlib import redirect_stdout
from pathlib import Path

from pytorch_operator_amd.cluster.cli import main
from pytorch_operator_amd.cluster.local import LocalCluster

ROOT = Path(__file__).resolve().parent.parent


def _run(*argv):
    buf = io.StringIO()
    with redirect_stdout(buf):
        rc = main(list(argv))
    return rc, buf.getvalue()


def test_apply_get_logs_delete(tmp_path):
    job = tmp_path / "job.yaml"
    job.write_text((ROOT / "examples/mnist/pytorch_job_mnist_gloo.yaml").read_text()
                   .replace('args: ["--backend", "gloo", "--no-cuda"]',
                            'args: ["--backend", "gloo", "--no-cuda", "--dataset-size", "640", "--test-size", "64"]'))
    with LocalCluster(workdir=str(tmp_path / "c")) as c:
        c.wait_operator_ready()
        kc = ["--kubeconfig", c.kubeconfig]
        rc, out = _run(*kc, "apply", "-f", str(job))
        assert rc == 0 and "pytorchjob/pytorch-dist-mnist-gloo created" in out
        t0 = time.time()
        while time.time() - t0 < 120:
            rc, out = _run(*kc, "get", "pytorchjobs")
            if "Succeeded" in out:
                break
            time.sleep(0.5)
        assert out.splitlines()[0].split() == ["NAME", "STATE", "AGE"]
        assert "pytorch-dist-mnist-gloo" in out and "Succeeded" in out
        rc, out = _run(*kc, "get", "pods")
        assert "pytorch-dist-mnist-gloo-master-0" in out and "Succeeded" in out
        rc, out = _run(*kc, "logs", "pytorch-dist-mnist-gloo-master-0")
        assert "accuracy=" in out
        rc, out = _run(*kc, "apply", "-f", str(job))
        assert "configured" in out
        rc, out = _run(*kc, "delete", "pytorchjob", "pytorch-dist-mnist-gloo")
        assert rc == 0
        rc, out = _run(*kc, "get", "pytorchjobs")
        assert "pytorch-dist-mnist-gloo" not in out
