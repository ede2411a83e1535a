#!/usr/bin/env python3
"""Reproduce the world-8 one-GPU exchange self-test failure context: run the attention GPU tests
in this process first (it then keeps its GPU context), then the 8-rank exchange stress
(tools/dbg/xar_stress.py) as a child, with and without --discriminate (the exchange and gloo's
GPU-tensor all_reduce checked separately against a host float64 mean).  Writes OUT/stress*.log.

    python tools/dbg/stress_after_attention.py OUT_DIR
"""
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r6_w8_attn"
    os.makedirs(out, exist_ok=True)
    import pytest
    rc = pytest.main(["-q", "-m", "gpu", os.path.join(ROOT, "tests/test_attention_gpu.py"), "-p", "no:cacheprovider",
                      "--timeout", "120", "--timeout-method", "thread"])
    print(f"attention tests rc={rc}", flush=True)
    env = dict(os.environ, GPU_MAX_HW_QUEUES="1", OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    for mode in (["--discriminate"], []):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
               "--master-addr", "127.0.0.1", "--master-port", str(29500 + random.randrange(1000)),
               os.path.join(ROOT, "tools/dbg/xar_stress.py"), "--steps", "40", *mode]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=ROOT, env=env)
        with open(os.path.join(out, f"stress{''.join(mode)}.log"), "w") as f:
            f.write(r.stdout + r.stderr)
        print(f"stress {mode} rc={r.returncode}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
