"""tools/rccl_tune.py: one torchrun job per RCCL env candidate, per-step all-reduce cost of the
MNIST gradient buckets, the winner as operator --rccl-env flags.  CPU: the gloo
plumbing at world 2; GPU (tests/test_rccl_gpu.py): every candidate under a real RCCL communicator."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_bucket_sizes_are_the_gradient_path_buckets():
    import rccl_tune
    from pytorch_operator_amd.models.mnist import NUM_PARAMS, flat_layout
    s = rccl_tune.bucket_sizes()
    lay = flat_layout()
    assert s["conv"] == lay.conv_end and s["fc"] + s["conv"] == lay.total >= NUM_PARAMS
    assert 400000 < s["fc"] * 1 < 410000 and s["conv"] < 26000


def test_race_at_world2_on_gloo(tmp_path):
    out = tmp_path / "tune.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_tune.py"), "--nproc", "2", "--backend",
                        "gloo", "--device", "cpu", "--candidates", "default,proto-LL", "--iters", "2", "--reps", "2",
                        "--warmup", "1", "--out", str(out)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert [c["name"] for c in res["candidates"]] == ["default", "proto-LL"]
    for c in res["candidates"]:
        assert c["correct"] and c["world"] == 2 and c["step_us"] > 0 and c["fc_us"] > 0 and c["conv_us"] > 0
    assert res["candidates"][1]["nccl_env"].get("NCCL_PROTO") == "LL"  # the candidate's env reached the ranks
    w = res["winner"]
    assert w["step_us"] == min(c["step_us"] for c in res["candidates"])
    flags = w["operator_flags"]
    assert flags[0::2] == ["--rccl-env"] * (len(flags) // 2)
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in flags[1::2]
    for k, v in w["env"].items():
        assert f"{k}={v}" in flags[1::2]


def test_unknown_candidate_is_refused():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_tune.py"), "--candidates", "nope"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "unknown candidates" in r.stderr


def test_env_file_reaches_the_operator(tmp_path):
    """--env-out writes the winner as KEY=VALUE lines; pytorch-operator --rccl-env-file reads them
    (comments and blank lines skipped, a malformed line refused with its line number)."""
    from pytorch_operator_amd.cluster.local import operator_binary
    out, env = tmp_path / "tune.json", tmp_path / "rccl.env"
    def tune(nproc):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_tune.py"), "--nproc", str(nproc),
                            "--backend", "gloo", "--device", "cpu", "--candidates", "proto-LL", "--iters", "2",
                            "--reps", "1", "--warmup", "1", "--out", str(out), "--env-out", str(env)],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        return r, [ln for ln in env.read_text().splitlines() if ln and not ln.startswith("#")]
    # one rank: the ranking is noise, so no protocol is pinned -- only the base environment
    r, lines = tune(1)
    assert lines == ["HSA_ENABLE_IPC_MODE_LEGACY=0"] and "--nproc < 2" in r.stderr
    r, lines = tune(2)
    assert lines == ["HSA_ENABLE_IPC_MODE_LEGACY=0", "NCCL_PROTO=LL"]
    bin_ = operator_binary()
    r = subprocess.run([bin_, "--inject-rccl-env", "--rccl-env-file", str(env), "--version"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    bad = tmp_path / "bad.env"
    bad.write_text("# ok\n\nNCCL_ALGO=Ring\nNOVALUE\n")
    r = subprocess.run([bin_, "--rccl-env-file", str(bad), "--version"], capture_output=True, text=True)
    assert r.returncode != 0 and "bad.env:4" in (r.stderr + r.stdout)
    r = subprocess.run([bin_, "--rccl-env-file", str(tmp_path / "missing.env"), "--version"],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "cannot read" in (r.stderr + r.stdout)
    # empty / comments-only: refused (it would drop HSA_ENABLE_IPC_MODE_LEGACY=0 from every pod)
    for body in ("", "# nothing measured\n\n"):
        empty = tmp_path / "empty.env"
        empty.write_text(body)
        r = subprocess.run([bin_, "--inject-rccl-env", "--rccl-env-file", str(empty), "--version"],
                           capture_output=True, text=True)
        assert r.returncode != 0 and "no KEY=VALUE" in (r.stderr + r.stdout), (body, r.stderr)


def test_candidate_timeout_kills_its_job(tmp_path):
    """A candidate job over --timeout is killed with its process group and reported; with no
    candidate left the tool exits 1 and names no winner."""
    out = tmp_path / "tune.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_tune.py"), "--nproc", "2", "--backend",
                        "gloo", "--device", "cpu", "--candidates", "default", "--timeout", "0.5", "--out", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert "winner" not in res and res["candidates"][0]["error"].startswith("timeout")
