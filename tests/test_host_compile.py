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


def test_malformed_node_tables_are_rejected_cleanly():
    """A bad child index or a bad unary operator index in a node table (C ABI / coalescer clients)
    is a clean SRHIP_ERR_INVALID, never an out-of-bounds read -- including in the derived-column
    pass that scans the tables before the trees are validated."""
    import pytest
    import srhip as sr
    from srhip import _lib

    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos", "exp"))
    # cos(x1) + cos(x1) twice over, so cos(x1) is a derived-column candidate
    good = [sr.Node(1, sr.Node(1, sr.Node(feature=1)), sr.Node(1, sr.Node(feature=1))) for _ in range(3)]
    nodes, offs = sr.flatten(good, opts, np.float32)
    sr.Program(None, nodes, offs, opts, np.float32)  # compiles
    unary = np.nonzero(nodes["degree"] == 1)[0]
    for field, bad in (("l", 1000), ("l", -3), ("op", 0), ("op", 77)):
        nd = nodes.copy()
        nd[unary[0]][field] = bad
        with pytest.raises(_lib.SrhipError) as e:
            sr.Program(None, nd, offs, opts, np.float32)
        assert e.value.code == _lib.ERR_INVALID, (field, bad, e.value)


def test_host_pool_back_to_back_jobs_from_many_threads():
    """Many small compiles from several threads back to back (the host pool's jobs follow each other
    closely, and callers that find it busy compile themselves): every result is the sequential one."""
    import srhip as sr
    from srhip import workloads

    opts, _, _, _, nodes, offs = workloads.c2(0, 256, 4096)
    ref = _stats(sr, sr.Program(None, nodes, offs, opts, np.float32))
    out, errs = [], []

    def work():
        try:
            for _ in range(40):
                out.append(_stats(sr, sr.Program(None, nodes, offs, opts, np.float32)))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work) for _ in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert len(out) == 240 and all(o == ref for o in out)


def test_code_cache_hits_equal_fresh_compiles(tmp_path, monkeypatch):
    """The per-tree code cache (csrc/srhip_host.cpp CodeCache): a population compiled from cached
    entries (second compile of the same trees, and a population mixing cached and new trees) has
    exactly the instructions (handler, operand, immediate), stack needs and costs of a compile with the
    cache off -- plain and derived programs -- and the superinstruction switch is part of the key."""
    import srhip as sr
    from srhip import workloads

    opts, _, _, _, nodes, offs = workloads.c2(0, 512, 4096)
    _, _, _, _, nodes2, offs2 = workloads.c2(1, 512, 4096)
    # a population of half old trees (cache hits) and half new ones
    half = int(offs[256])
    mixed = np.concatenate([nodes[:half], nodes2[: int(offs2[256])]])
    moffs = np.concatenate([offs[:257], half + offs2[1:257]])

    def dump(nd, of, tag, cache, nosuper=False):
        path = str(tmp_path / f"{tag}.bin")
        monkeypatch.setenv("SRHIP_DUMP_CODE", path)
        monkeypatch.setenv("SRHIP_NO_CODE_CACHE", "0" if cache else "1")
        monkeypatch.setenv("SRHIP_NO_SUPER", "1" if nosuper else "0")
        p = sr.Program(None, nd, of, opts, np.float32)
        st = _stats(sr, p)
        monkeypatch.delenv("SRHIP_DUMP_CODE")
        return open(path, "rb").read(), open(path + ".plain", "rb").read(), st

    import ctypes

    from srhip import _lib

    def cache_stats():
        h, m, i = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        assert _lib.load().srhip_code_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(i)) == 0
        return h.value, m.value, i.value

    for nosuper in (False, True):
        fresh = dump(nodes, offs, f"fresh{nosuper}", False, nosuper)
        h0 = cache_stats()
        first = dump(nodes, offs, f"first{nosuper}", True, nosuper)    # first sighting: hashes recorded
        h1 = cache_stats()
        again = dump(nodes, offs, f"again{nosuper}", True, nosuper)    # second: compiled, entries made
        h2 = cache_stats()
        third = dump(nodes, offs, f"third{nosuper}", True, nosuper)    # third: served from the cache
        h3 = cache_stats()
        assert first == fresh and again == fresh and third == fresh
        assert h1[2] - h0[2] < 512 // 8, "a first sighting makes (almost) no entries"
        assert h2[2] - h1[2] > 512 // 2, "a second sighting makes entries"
        assert h3[0] - h2[0] > 512 // 2, "a third compile hits"
    assert dump(nodes, offs, "s", True)[0] != dump(nodes, offs, "n", True, True)[0]
    assert dump(mixed, moffs, "mixc", True) == dump(mixed, moffs, "mixf", False)
