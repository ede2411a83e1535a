"""Release and licensing deliverables (VERDICT r4 "next round" #6; reference: developer_guide.md,
releasing.md, third_party_licenses/license_info.csv).

* the developer guide and the release procedure exist and name the commands this repository has;
* every base image and every package the Dockerfiles install has a row in the licence inventory.
"""
import csv
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _dockerfile_packages():
    pkgs = set()
    for df in sorted((ROOT / "docker").glob("Dockerfile.*")):
        text = df.read_text().replace("\\\n", " ")
        for m in re.finditer(r"^\s*FROM\s+(\S+)", text, re.M):
            img = m.group(1)
            if img.startswith("${"):  # ARG-defaulted base: resolve from the ARG line
                arg = img.strip("${}").split(":")[0]
                am = re.search(rf"^\s*ARG\s+{arg}=(\S+)", text, re.M)
                img = am.group(1) if am else img
            pkgs.add(img.split(":latest")[0])
        for m in re.finditer(r"apt-get install\s+([^&;]+)", text):
            pkgs.update(t for t in m.group(1).split() if not t.startswith("-"))
        for m in re.finditer(r"pip3? install\s+([^&;]+)", text):
            pkgs.update(t for t in m.group(1).split() if not t.startswith("-"))
    return pkgs


def test_every_dockerfile_package_is_in_the_licence_inventory():
    with open(ROOT / "third_party_licenses" / "license_info.csv", newline="") as f:
        rows = list(csv.DictReader(f))
    assert rows and set(rows[0]) == {"name", "url", "license", "license_url"}
    assert all(r["license"].strip() and r["url"].startswith("http") for r in rows), rows
    names = {r["name"].split(" (")[0].strip() for r in rows} | {r["name"] for r in rows}
    pkgs = _dockerfile_packages()
    assert {"ubuntu:22.04", "libssl3", "rocm/pytorch", "pybind11"} <= pkgs, pkgs  # the parser sees them
    missing = sorted(p for p in pkgs if p not in names)
    assert not missing, f"add {missing} to third_party_licenses/license_info.csv"


def test_developer_guide_and_release_procedure_exist():
    dev = (ROOT / "docs" / "developer_guide.md").read_text()
    rel = (ROOT / "docs" / "releasing.md").read_text()
    for needle in ("make build", "pytorch_operator_amd.cluster up", 'pytest tests -m "not gpu"', "-m gpu",
                   "tools/gpu/profile.sh", "step_timeline.py"):
        assert needle in dev, needle
    for needle in ("docker build -f docker/Dockerfile.operator", "docker build -f docker/Dockerfile.worker",
                   "manifests/crd.yaml", "make verify", "license_info.csv"):
        assert needle in rel, needle
    # the commands the guide names exist
    for path in ("tools/gpu/profile.sh", "tools/gpu/pmc.sh", "tools/step_timeline.py", "tools/build_exp.sh",
                 "examples/mnist/pytorch_job_mnist_gloo.yaml", "manifests/legacy/crd-v1beta1.yaml",
                 "benchmarks/job_latency.py", "sdk/python/setup.py"):
        assert (ROOT / path).exists(), path
