"""Small shared helpers of the host mirror."""
from __future__ import annotations

import itertools
import threading

_birth = itertools.count()
_birth_lock = threading.Lock()


def get_birth_order() -> int:
    """src/Utils.jl:9-19 get_birth_order (the deterministic counter form): a process-wide,
    thread-safe, strictly increasing birth stamp for PopMembers (regularized evolution replaces the
    oldest member, src/RegularizedEvolution.jl:53,85)."""
    with _birth_lock:
        return next(_birth)
