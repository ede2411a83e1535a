import time

_T_MAIN = time.time_ns()  # before the worker's imports (startup breakdown: harness/mnist.py)

from .mnist import main  # noqa: E402

raise SystemExit(main(t_main_ns=_T_MAIN))
