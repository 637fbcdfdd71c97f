"""Small shared helpers of the host mirror."""
from __future__ import annotations

import threading

_birth_lock = threading.Lock()
_next_birth = 0


def get_birth_order() -> int:
    """src/Utils.jl:9-19 get_birth_order (the deterministic counter form): a process-wide,
    thread-safe, strictly increasing birth stamp for PopMembers (regularized evolution replaces the
    oldest member, src/RegularizedEvolution.jl:53,85)."""
    global _next_birth
    with _birth_lock:
        b = _next_birth
        _next_birth += 1
        return b


def advance_birth_order(past: int) -> None:
    """Make every later birth stamp of this process exceed `past` (a :multiprocessing worker gets
    the populations of the head process, whose members were stamped by the head's counter; the head
    then advances past the stamps its workers returned).  Only the order of stamps within one
    population matters, and that order is the one the threaded search produces."""
    global _next_birth
    with _birth_lock:
        _next_birth = max(_next_birth, int(past) + 1)
