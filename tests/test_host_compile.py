"""Host-side compiler (no device): a population compiled on the library's host thread pool gives the
same program metadata whether compiled alone or from several threads at once (callers that find the
pool busy compile their ranges themselves)."""
import threading

import numpy as np

from conftest import ROOT  # noqa: F401  (puts the package on sys.path)


def _stats(sr, prog):
    st = prog.stats()
    return (st["total_nodes"], st["total_opnodes"], st["max_stack"], tuple(prog.num_constants()),
            tuple(prog.derived_columns()))


def test_concurrent_host_compiles_agree():
    import srhip as sr
    from srhip import workloads

    opts, _, _, _, nodes, offs = workloads.c2(0, 1024, 4096)
    ref = _stats(sr, sr.Program(None, nodes, offs, opts, np.float32))
    out, errs = [], []

    def work():
        try:
            for _ in range(3):
                out.append(_stats(sr, sr.Program(None, nodes, offs, opts, np.float32)))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert len(out) == 12 and all(o == ref for o in out)
    assert ref[4], "the C2 population has derived columns"
