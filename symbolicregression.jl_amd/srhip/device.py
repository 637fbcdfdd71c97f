"""Handles over libsrhip objects: Context (device + stream), DeviceDataset, Program.

One Context per (host thread, device): libsrhip contexts are not thread-safe, which matches
the reference's concurrency model (one task per population, src/SearchUtils.jl:108-127).
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import check, ptr


class Context:
    def __init__(self, device: int = 0):
        lib = _lib.load()
        h = ctypes.c_void_p()
        check(lib.srhip_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = int(device)
        self._lib = lib

    def synchronize(self):
        check(self._lib.srhip_ctx_synchronize(self.handle))

    def last_kernel_ms(self) -> float:
        return float(self._lib.srhip_last_kernel_ms(self.handle))

    def last_work(self) -> dict:
        """Work of the last evaluation launch, counted on the device (srhip_last_work): node-rows
        evaluated, nominal node-rows (every live tree on every row), operator-node rows and tree-rows
        evaluated.  A failed tree (the reference's early return) stops at its failing tile."""
        out = (ctypes.c_int64 * 4)()
        check(self._lib.srhip_last_work(self.handle, out))
        return {"node_rows": int(out[0]), "nominal_node_rows": int(out[1]), "opnode_rows": int(out[2]),
                "tree_rows": int(out[3])}

    def close(self):
        if self.handle:
            self._lib.srhip_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def get_context(device: int = 0) -> Context:
    """The calling thread's context for `device` (created on first use)."""
    cache = getattr(_tls, "ctxs", None)
    if cache is None:
        cache = _tls.ctxs = {}
    ctx = cache.get(device)
    if ctx is None:
        ctx = cache[device] = Context(device)
    return ctx


def device_count() -> int:
    try:
        return int(_lib.load().srhip_device_count())
    except _lib.SrhipError:
        return 0


class DeviceDataset:
    """A dataset uploaded to HBM (X as [nfeatures][n] padded SoA, y, weights)."""

    def __init__(self, ctx: Context, X: np.ndarray, y=None, weights=None):
        X = np.asarray(X)
        if X.ndim != 2:
            raise ValueError("X must be (nfeatures, n)")
        self.dtype = X.dtype
        code = _lib.dtype_code(X.dtype)
        nfeat, n = X.shape
        # element (f, j) at X[f*sf + j*sr] in elements
        es = X.itemsize
        sf, sr = X.strides[0] // es, X.strides[1] // es
        if X.strides[0] % es or X.strides[1] % es:
            X = np.ascontiguousarray(X)
            sf, sr = n, 1
        yv = None if y is None else np.ascontiguousarray(y, dtype=X.dtype)
        wv = None if weights is None else np.ascontiguousarray(weights, dtype=X.dtype)
        h = ctypes.c_void_p()
        check(_lib.load().srhip_dataset_create(ctx.handle, code, ptr(X), nfeat, n, sf, sr, ptr(yv), ptr(wv),
                                               ctypes.byref(h)))
        self.handle = h
        self.ctx = ctx
        self.nfeatures = nfeat
        self.n = n
        self.weighted = weights is not None

    def close(self):
        if self.handle:
            _lib.load().srhip_dataset_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Program:
    """A compiled batch of trees (bytecode resident on the device).

    ctx=None makes a host-only program: compiled, with the did_succeed metadata that the
    row-sharded finalize steps need, but not evaluable (no device is touched)."""

    def __init__(self, ctx: Context | None, nodes: np.ndarray, offsets: np.ndarray, options, dtype):
        self.ctx = ctx
        self.nodes = np.ascontiguousarray(nodes)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.ntrees = len(self.offsets) - 1
        self.options = options
        self.dtype = np.dtype(dtype)
        h = ctypes.c_void_p()
        self._ops = options.c_operators()
        check(_lib.load().srhip_program_create(None if ctx is None else ctx.handle, _lib.dtype_code(dtype),
                                               ptr(self.nodes),
                                               ptr(self.offsets), self.ntrees, ctypes.byref(self._ops),
                                               ctypes.byref(h)))
        self.handle = h

    def num_constants(self) -> np.ndarray:
        out = np.zeros(self.ntrees, dtype=np.int32)
        check(_lib.load().srhip_program_num_constants(self.handle, ptr(out)))
        return out

    def set_constants(self, consts: np.ndarray) -> None:
        c = np.ascontiguousarray(consts, dtype=np.float64)
        check(_lib.load().srhip_program_set_constants(self.handle, ptr(c)))

    def stats(self):
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        check(_lib.load().srhip_program_stats(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return dict(total_nodes=a.value, total_opnodes=b.value, max_stack=c.value)

    def derived_columns(self) -> list:
        """[(device unary op, 0-based feature)] computed once per workgroup and shared by the trees."""
        n = ctypes.c_int32()
        spec = np.zeros(64, dtype=np.uint32)
        check(_lib.load().srhip_program_derived(self.handle, ctypes.byref(n), ptr(spec), 64))
        return [(int(s) >> 16, int(s) & 0xffff) for s in spec[:n.value]]

    def eval_loss(self, ds: DeviceDataset, loss, idx=None):
        out = np.empty(self.ntrees, dtype=np.float64)
        ok = np.empty(self.ntrees, dtype=np.uint8)
        ls = loss.c_struct()
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        check(_lib.load().srhip_eval_loss(self.ctx.handle, ds.handle, self.handle, ctypes.byref(ls), ptr(idxa),
                                          0 if idxa is None else len(idxa), ptr(out), ptr(ok)))
        return out, ok.astype(bool)

    def eval_loss_submit(self, ds: DeviceDataset, loss, idx=None) -> "EvalTicket":
        """srhip_eval_loss_submit: the evaluation's launches queued behind whatever is in flight on the
        context; .wait() -> (loss[T], ok[T]), the same bits as eval_loss.  At most 3 outstanding per
        context; this program and ds must stay alive until the ticket is waited."""
        ls = loss.c_struct()
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        h = ctypes.c_void_p()
        check(_lib.load().srhip_eval_loss_submit(self.ctx.handle, ds.handle, self.handle, ctypes.byref(ls), ptr(idxa),
                                                 0 if idxa is None else len(idxa), ctypes.byref(h)))
        return EvalTicket(h, self, ds)

    def eval_predict(self, ds: DeviceDataset, idx=None):
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        m = ds.n if idxa is None else len(idxa)
        out = np.empty((self.ntrees, m), dtype=self.dtype)
        ok = np.empty(self.ntrees, dtype=np.uint8)
        check(_lib.load().srhip_eval_predict(self.ctx.handle, ds.handle, self.handle, ptr(idxa),
                                             0 if idxa is None else len(idxa), ptr(out), ptr(ok)))
        return out, ok.astype(bool)

    # ---- constant optimisation (src/ConstantOptimization.jl) ---------------------------------
    def get_constants(self) -> list:
        """Per tree, its current constants in get_constants order."""
        nconst = self.num_constants()
        c = np.empty(int(nconst.sum()), dtype=np.float64)
        check(_lib.load().srhip_program_get_constants(self.handle, ptr(c)))
        return np.split(c, np.cumsum(nconst)[:-1])

    def eval_loss_grad(self, ds: DeviceDataset, loss, idx=None):
        """(loss[T], grads: list of per-tree arrays (get_constants order), ok[T])."""
        nconst = self.num_constants()
        out = np.empty(self.ntrees, dtype=np.float64)
        grad = np.empty(int(nconst.sum()), dtype=np.float64)
        ok = np.empty(self.ntrees, dtype=np.uint8)
        ls = loss.c_struct()
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        check(_lib.load().srhip_eval_loss_grad(self.ctx.handle, ds.handle, self.handle, ctypes.byref(ls), ptr(idxa),
                                               0 if idxa is None else len(idxa), ptr(out), ptr(grad), ptr(ok)))
        splits = np.cumsum(nconst)[:-1]
        return out, np.split(grad, splits), ok.astype(bool)

    def eval_grad_predict(self, ds: DeviceDataset, variable: bool = False, direction: int = 0, idx=None):
        """Per-row derivatives (srhip_eval_grad_predict): (pred[T, m], grads: list of per-tree arrays
        [rows, m], ok[T]); rows = the tree's constants (variable=False, get_constants order), every
        feature (variable=True), or feature `direction` alone (direction >= 1)."""
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        m = ds.n if idxa is None else len(idxa)
        if variable:
            rows = np.full(self.ntrees, 1 if direction else ds.nfeatures, dtype=np.int64)
        else:
            rows = self.num_constants().astype(np.int64)
        pred = np.empty((self.ntrees, m), dtype=self.dtype)
        grad = np.empty((int(rows.sum()), m), dtype=self.dtype)
        ok = np.empty(self.ntrees, dtype=np.uint8)
        check(_lib.load().srhip_eval_grad_predict(self.ctx.handle, ds.handle, self.handle, 1 if variable else 0,
                                                  int(direction), ptr(idxa), 0 if idxa is None else len(idxa),
                                                  ptr(pred), ptr(grad), ptr(ok)))
        return pred, np.split(grad, np.cumsum(rows)[:-1]), ok.astype(bool)

    def optimize_constants(self, ds: DeviceDataset, loss, iterations=8, nrestarts=2, seed=0, g_tol=1e-8, idx=None,
                           starts=None, return_starts=False):
        """Batched optimize_constants; updates this program's constants in place.

        starts: optional [nrestarts, sum nconst] restart points (get_constants order, tree-major)
        used instead of the library's draws.  Returns (loss[T] of the returned trees, improved[T],
        fcalls[T]), plus the restart points used ([nrestarts, sum nconst]) if return_starts."""
        opt = _lib.OptimOptions(int(iterations), int(nrestarts), int(seed) & (2**64 - 1), float(g_tol))
        out = np.empty(self.ntrees, dtype=np.float64)
        imp = np.empty(self.ntrees, dtype=np.uint8)
        fc = np.empty(self.ntrees, dtype=np.int64)
        ls = loss.c_struct()
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        nall = int(self.num_constants().sum())
        sin = None
        if starts is not None:
            sin = np.ascontiguousarray(starts, dtype=np.float64).reshape(int(nrestarts), nall)
        sout = np.empty((int(nrestarts), nall), dtype=np.float64) if return_starts else None
        if sin is None and sout is None:  # the library's own draws, not reported: the plain entry point
            check(_lib.load().srhip_optimize_constants(
                self.ctx.handle, ds.handle, self.handle, ctypes.byref(ls), ptr(idxa), 0 if idxa is None else len(idxa),
                ctypes.byref(opt), ptr(out), ptr(imp), ptr(fc)))
        else:
            check(_lib.load().srhip_optimize_constants_starts(
                self.ctx.handle, ds.handle, self.handle, ctypes.byref(ls), ptr(idxa), 0 if idxa is None else len(idxa),
                ctypes.byref(opt), ptr(sin), ptr(sout), ptr(out), ptr(imp), ptr(fc)))
        if return_starts:
            return out, imp.astype(bool), fc, sout
        return out, imp.astype(bool), fc

    # ---- row-sharded evaluation (include/srhip.h "row-sharded evaluation") ----------------------
    def chk_reduce_op(self) -> str:
        """How chk combines across shards: "max" (Float32) or "sum" (Float64 / Int32)."""
        return "max" if _lib.load().srhip_chk_reduce_op(_lib.dtype_code(self.dtype)) == 0 else "sum"

    def max_ops(self) -> int:
        return int(_lib.load().srhip_program_max_ops(self.handle))

    def eval_loss_partials(self, ds: DeviceDataset, loss, idx=None):
        """This shard's (sums[2T + 2F + 1], chk[T]) — combine across shards, then finalize()."""
        sums = np.empty(2 * self.ntrees + 2 * ds.nfeatures + 1, dtype=np.float64)
        chk = np.empty(self.ntrees, dtype=np.float64)
        ls = loss.c_struct()
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        check(_lib.load().srhip_eval_loss_partials(self.ctx.handle, ds.handle, self.handle, ctypes.byref(ls), ptr(idxa),
                                                   0 if idxa is None else len(idxa), ptr(sums), ptr(chk)))
        return sums, chk

    def finalize(self, nfeatures: int, sums, chk):
        """Decision from globally combined partials: (loss[T], ok[T], status[T]); status 2 = undecided."""
        sums = np.ascontiguousarray(sums, dtype=np.float64)
        chk = np.ascontiguousarray(chk, dtype=np.float64)
        loss = np.empty(self.ntrees, dtype=np.float64)
        ok = np.empty(self.ntrees, dtype=np.uint8)
        st = np.empty(self.ntrees, dtype=np.uint8)
        check(_lib.load().srhip_partials_finalize(self.handle, int(nfeatures), ptr(sums), ptr(chk), ptr(loss), ptr(ok),
                                                  ptr(st)))
        return loss, ok.astype(bool), st

    def eval_precise_partials(self, ds: DeviceDataset, trees, idx=None):
        trees = np.ascontiguousarray(trees, dtype=np.int32)
        out = np.empty(len(trees) * self.max_ops(), dtype=np.float64)
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        check(_lib.load().srhip_eval_precise_partials(self.ctx.handle, ds.handle, self.handle, ptr(idxa),
                                                      0 if idxa is None else len(idxa), ptr(trees), len(trees),
                                                      ptr(out)))
        return out

    def precise_finalize(self, trees, opsums):
        trees = np.ascontiguousarray(trees, dtype=np.int32)
        opsums = np.ascontiguousarray(opsums, dtype=np.float64)
        ok = np.empty(len(trees), dtype=np.uint8)
        check(_lib.load().srhip_precise_finalize(self.handle, ptr(trees), len(trees), ptr(opsums), ptr(ok)))
        return ok.astype(bool)

    def close(self):
        if self.handle:
            _lib.load().srhip_program_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Coalescer:
    """Cross-population request coalescer over libsrhip's batcher (include/srhip.h,
    SURVEY.md §8(f)-1).  Any number of threads call :meth:`score_loss` with ONE flattened tree;
    a native worker thread batches concurrent requests into one launch.  The result equals
    ``Program(ctx, tree).eval_loss(ds, loss)`` for that tree alone.  The context is owned by the
    batcher for its lifetime (do not evaluate on it from other threads meanwhile)."""

    def __init__(self, ctx: Context, ds: DeviceDataset, options, loss, max_batch: int = 256,
                 max_wait_us: int = 200, nclients: int = 0):
        self.ctx, self.ds, self.options, self.loss = ctx, ds, options, loss
        self._ops = options.c_operators()
        self._loss = loss.c_struct()
        h = ctypes.c_void_p()
        check(_lib.load().srhip_batcher_create(ctx.handle, ds.handle, ctypes.byref(self._ops),
                                               ctypes.byref(self._loss), int(max_batch), int(max_wait_us),
                                               ctypes.byref(h)))
        self.handle = h
        if nclients:
            self.set_clients(nclients)

    def set_clients(self, n: int) -> None:
        check(_lib.load().srhip_batcher_set_clients(self.handle, int(n)))

    def score_loss(self, nodes: np.ndarray, idx=None):
        """(loss, did_succeed) of one tree given as a srhip_node run (root first).  Blocks; the
        GIL is released while waiting (ctypes), so island threads overlap."""
        nodes = np.ascontiguousarray(nodes)
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        loss, ok = ctypes.c_double(), ctypes.c_uint8()
        check(_lib.load().srhip_batcher_eval(self.handle, ptr(nodes), len(nodes), ptr(idxa),
                                             0 if idxa is None else len(idxa), ctypes.byref(loss),
                                             ctypes.byref(ok)))
        return float(loss.value), bool(ok.value)

    def submit(self, nodes: np.ndarray, idx=None) -> int:
        nodes = np.ascontiguousarray(nodes)
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        t = ctypes.c_uint64()
        check(_lib.load().srhip_batcher_submit(self.handle, ptr(nodes), len(nodes), ptr(idxa),
                                               0 if idxa is None else len(idxa), ctypes.byref(t)))
        return int(t.value)

    def wait(self, ticket: int):
        loss, ok = ctypes.c_double(), ctypes.c_uint8()
        check(_lib.load().srhip_batcher_wait(self.handle, ctypes.c_uint64(ticket), ctypes.byref(loss),
                                             ctypes.byref(ok)))
        return float(loss.value), bool(ok.value)

    def stats(self) -> dict:
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(_lib.load().srhip_batcher_stats(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        busy, kern = ctypes.c_double(), ctypes.c_double()
        check(_lib.load().srhip_batcher_timing(self.handle, ctypes.byref(busy), ctypes.byref(kern)))
        return dict(requests=a.value, launches=b.value, max_batch=c.value, busy_ms=busy.value, kernel_ms=kern.value)

    def close(self):
        if getattr(self, "handle", None):
            _lib.load().srhip_batcher_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EvalTicket:
    """An evaluation in flight (Program.eval_loss_submit); wait() exactly once."""

    def __init__(self, handle, prog, ds):
        self.handle, self._prog, self._ds = handle, prog, ds  # (keeps both alive until waited)

    def wait(self):
        if self.handle is None:
            raise RuntimeError("ticket already waited")
        out = np.empty(self._prog.ntrees, dtype=np.float64)
        ok = np.empty(self._prog.ntrees, dtype=np.uint8)
        h, self.handle = self.handle, None  # the library frees the ticket on every path
        check(_lib.load().srhip_eval_loss_wait(h, ptr(out), ptr(ok)))
        self._prog = self._ds = None
        return out, ok.astype(bool)
