"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/build/liboracle.so, the C restatement of the reference's hot path
(DynamicExpressions v0.16 eval_tree_array + src/LossFunctions.jl _loss/_weighted_loss/_eval_loss;
see sr_oracle.c for the file:line map).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product (srhip / libsrhip.so) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
_lib = None

_SFX = {np.dtype(np.float32): "f32", np.dtype(np.float64): "f64", np.dtype(np.int32): "i32"}


def build() -> None:
    subprocess.run(["make", "-C", HERE], check=True, capture_output=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def use_variant(name=None) -> None:
    """Switch this process's oracle to a libm-sensitivity build (oracle/Makefile `variants`):
    "jtrig" (Julia's Float32 sin / cos kernels), "glibc64" (glibc Float64 exp / log / sin / cos), or
    None for the default checker.  oracle/libm_sensitivity.py only -- the parity tests use the default."""
    global _lib
    if name is None:
        _lib = None
        return
    path = os.path.join(HERE, "build", f"liboracle_{name}.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", HERE, "variants"], check=True, capture_output=True)
    _lib = ctypes.CDLL(path)


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _setup(fn, restype, argtypes):
    fn.restype = restype
    fn.argtypes = argtypes
    return fn


def eval_tree(nodes, binops, unaops, X):
    """eval_tree_array(tree, X, operators) -> (out, ok); X is (nfeatures, n)."""
    lib = load()
    X = np.ascontiguousarray(X)
    sfx = _SFX[X.dtype]
    n = X.shape[1]
    out = np.empty(n, dtype=X.dtype)
    nodes = np.ascontiguousarray(nodes)
    b = np.ascontiguousarray(binops, dtype=np.int32)
    u = np.ascontiguousarray(unaops, dtype=np.int32)
    fn = _setup(getattr(lib, f"oracle_eval_tree_{sfx}"), ctypes.c_int,
                [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p])
    ok = fn(_p(nodes), _p(b), _p(u), _p(X), n, _p(out))
    return out, bool(ok)


def eval_loss(nodes, binops, unaops, X, y, w=None, kind=0, p0=0.0):
    """_eval_loss(regularization=false) -> (loss_exact, loss_reference_order, ok)."""
    lib = load()
    X = np.ascontiguousarray(X)
    sfx = _SFX[X.dtype]
    n = X.shape[1]
    y = np.ascontiguousarray(y, dtype=X.dtype)
    w = None if w is None else np.ascontiguousarray(w, dtype=X.dtype)
    nodes = np.ascontiguousarray(nodes)
    b = np.ascontiguousarray(binops, dtype=np.int32)
    u = np.ascontiguousarray(unaops, dtype=np.int32)
    le, lr = ctypes.c_double(), ctypes.c_double()
    fn = _setup(getattr(lib, f"oracle_eval_loss_{sfx}"), ctypes.c_int,
                [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)])
    ok = fn(_p(nodes), _p(b), _p(u), _p(X), _p(y), _p(w), n, int(kind), float(p0), ctypes.byref(le),
            ctypes.byref(lr))
    return le.value, lr.value, bool(ok)


def eval_loss_batch(nodes, offsets, binops, unaops, X, y, w=None, kind=0, p0=0.0, nthreads=0):
    """Every tree, OpenMP over trees. Returns (loss_exact, loss_ref, ok, threads_used)."""
    lib = load()
    X = np.ascontiguousarray(X)
    sfx = _SFX[X.dtype]
    n = X.shape[1]
    y = np.ascontiguousarray(y, dtype=X.dtype)
    w = None if w is None else np.ascontiguousarray(w, dtype=X.dtype)
    nodes = np.ascontiguousarray(nodes)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    nt = len(offsets) - 1
    b = np.ascontiguousarray(binops, dtype=np.int32)
    u = np.ascontiguousarray(unaops, dtype=np.int32)
    le = np.empty(nt, dtype=np.float64)
    lr = np.empty(nt, dtype=np.float64)
    ok = np.empty(nt, dtype=np.uint8)
    nr = np.zeros(nt, dtype=np.int64)
    fn = _setup(getattr(lib, f"oracle_eval_loss_batch_work_{sfx}"), ctypes.c_int,
                [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                 ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p])
    used = fn(_p(nodes), _p(offsets), nt, _p(b), _p(u), _p(X), _p(y), _p(w), n, int(kind), float(p0),
              int(nthreads), _p(le), _p(lr), _p(ok), _p(nr))
    eval_loss_batch.last_node_rows = int(nr.sum())  # node-rows evaluated (the early return stops a failed tree)
    return le, lr, ok.astype(bool), used


def loss_grad(nodes, binops, unaops, X, y, w=None, kind=0):
    """Exact d loss / d constants (get_constants order) of ONE Float64 tree by forward-mode dual
    numbers (sr_oracle_grad.h); kind 0 = L2, 1 = L1."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    nodes = np.ascontiguousarray(nodes)
    b = np.ascontiguousarray(binops, dtype=np.int32)
    u = np.ascontiguousarray(unaops, dtype=np.int32)
    out = np.empty(64, dtype=np.float64)
    fn = _setup(lib.oracle_loss_grad_f64, ctypes.c_int,
                [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p])
    nc = fn(_p(nodes), len(nodes), _p(b), _p(u), _p(X), _p(y), _p(w), X.shape[1], int(kind), _p(out))
    if nc < 0:
        raise ValueError("too many constants for the gradient oracle")
    return out[:nc].copy()


def loss_grad_devorder(nodes, binops, unaops, X, y, w=None, kind=0, rb=256):
    """(loss, gradient) of ONE tree -- the loss value and exact gradient summed in libsrhip's
    dual-number kernel's row order (sr_oracle_grad.h dev_order_sum; no did_succeed decision).  Float32
    X: the kernel's Float32 arithmetic (constants rounded to Float32), oracle_loss_grad_devorder_f32."""
    lib = load()
    dt = np.float32 if np.asarray(X).dtype == np.float32 else np.float64
    X = np.ascontiguousarray(X, dtype=dt)
    y = np.ascontiguousarray(y, dtype=dt)
    w = None if w is None else np.ascontiguousarray(w, dtype=dt)
    nodes = np.ascontiguousarray(nodes)
    b = np.ascontiguousarray(binops, dtype=np.int32)
    u = np.ascontiguousarray(unaops, dtype=np.int32)
    out = np.empty(65, dtype=np.float64)
    fn = _setup(lib.oracle_loss_grad_devorder_f32 if dt == np.float32 else lib.oracle_loss_grad_devorder_f64,
                ctypes.c_int,
                [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p])
    nc = fn(_p(nodes), len(nodes), _p(b), _p(u), _p(X), _p(y), _p(w), X.shape[1], int(kind), int(rb), _p(out))
    if nc < 0:
        raise ValueError("too many constants for the gradient oracle")
    return float(out[0]), out[1:nc + 1].copy()


def scalar_bin(op, a, b, dtype):
    lib = load()
    sfx = _SFX[np.dtype(dtype)]
    ct = {"f32": ctypes.c_float, "f64": ctypes.c_double, "i32": ctypes.c_int32}[sfx]
    fn = _setup(getattr(lib, f"oracle_bin_{sfx}"), ct, [ctypes.c_int, ct, ct])
    return np.dtype(dtype).type(fn(int(op), ct(a), ct(b)))


def scalar_un(op, x, dtype):
    lib = load()
    sfx = _SFX[np.dtype(dtype)]
    ct = {"f32": ctypes.c_float, "f64": ctypes.c_double, "i32": ctypes.c_int32}[sfx]
    fn = _setup(getattr(lib, f"oracle_un_{sfx}"), ct, [ctypes.c_int, ct])
    return np.dtype(dtype).type(fn(int(op), ct(x)))


_SRM = {"exp": 0, "log": 1, "sin": 2, "cos": 3, "tan": 4, "jsin": 5, "jcos": 6}  # j*: Julia's Float32 sin / cos restated (srm_jtrigf)


def srm(name, x):
    """The shared libm (include/srhip_math.h) on an array: Float64 or Float32 by x's dtype."""
    lib = load()
    x = np.ascontiguousarray(x)
    y = np.empty_like(x)
    sfx = "f64" if x.dtype == np.float64 else "f32"
    fn = _setup(getattr(lib, f"oracle_srm_{sfx}"), None,
                [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64])
    fn(_SRM[name], _p(x), _p(y), len(x))
    return y


def partials(nodes, offsets, binops, unaops, X, y, w=None, loss_kind=0, p0=0.0):
    """One row shard's (sums, chk) in libsrhip's srhip_eval_loss_partials layout (row-wise)."""
    lib = load()
    X = np.ascontiguousarray(X)
    sfx = _SFX[X.dtype]
    nfeat, n = X.shape
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    T = len(offsets) - 1
    sums = np.zeros(2 * T + 2 * nfeat + 1, dtype=np.float64)
    chk = np.zeros(T, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=X.dtype)
    w = None if w is None else np.ascontiguousarray(w, dtype=X.dtype)
    fn = _setup(getattr(lib, f"oracle_partials_{sfx}"), None,
                [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                 ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p])
    fn(_p(np.ascontiguousarray(nodes)), _p(offsets), T, _p(np.ascontiguousarray(binops, dtype=np.int32)),
       _p(np.ascontiguousarray(unaops, dtype=np.int32)), _p(X), nfeat, _p(y), _p(w), n, int(loss_kind),
       float(p0), _p(sums), _p(chk))
    return sums, chk
