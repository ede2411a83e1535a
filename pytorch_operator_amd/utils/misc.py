"""Python twins of the reference's pkg/util helpers (pkg/util/util.go:33-74).

``pformat`` pretty-prints anything JSON-serialisable (strings pass through verbatim) --
the e2e suite uses it to dump a job's status when an assertion fails; ``rand_string``
builds the random lowercase-alphanumeric suffix the reference's e2e programs append to
job names so concurrent runs never collide.  The C++ operator has the same pair in
``csrc/operator/include/pto/util.hpp``.
"""
from __future__ import annotations

import json
import secrets

_LETTERS = "0123456789abcdefghijklmnopqrstuvwxyz"


def pformat(value) -> str:
    if isinstance(value, str):
        return value
    try:
        return json.dumps(value, indent=2, sort_keys=False, default=str)
    except (TypeError, ValueError):
        return repr(value)


def rand_string(n: int) -> str:
    return "".join(secrets.choice(_LETTERS) for _ in range(max(0, n)))
