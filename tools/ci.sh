#!/bin/bash
# CI entry point (the reference's .travis.yml + Argo e2e workflow roles, run locally or by
# .github/workflows/ci.yml):
#   tools/ci.sh cpu   build everything (HIP kernels cross-compiled for gfx950 with hipcc,
#                     C++ operator + _opcore + C++ tests with g++), generated-file check,
#                     CPU suite: operator unit/ported Go tests, sanitizer builds (ASan/UBSan/
#                     TSan), fake-API-server e2e with real worker processes, SDK, harness
#   tools/ci.sh gpu   on an MI355X runner: kernel numerics, xGMI protocol, GPU job e2e,
#                     smoke, 1-GPU bench (each step under its own time limit)
set -euo pipefail
cd "$(dirname "$0")/.."
mode=${1:-cpu}
export PYTHONUNBUFFERED=1
case "$mode" in
  cpu)
    python -c "import __graft_entry__ as g; g.build()"
    python tools/gen_schema.py --check
    python -m pytest tests -m "not gpu" -q -x --timeout 900
    ;;
  gpu)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
    timeout -k 10 300 python bench.py --steps 2000 --warmup 50
    ;;
  *)
    echo "usage: tools/ci.sh cpu|gpu" >&2
    exit 2
    ;;
esac
