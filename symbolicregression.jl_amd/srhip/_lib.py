"""ctypes binding of libsrhip.so (the C ABI in include/srhip.h).

The library is built in-tree (``make -C symbolicregression.jl_amd``) and loaded from
``symbolicregression.jl_amd/build/libsrhip.so``.  There is no CPU fallback: if the library is
missing, or no gfx950 device is visible, calls raise :class:`SrhipError` loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "SRHIP_LIB", os.path.join(os.path.dirname(_PKG_DIR), "build", "libsrhip.so")
)

# ---- constants mirrored from include/srhip.h (tests/test_abi.py checks them against the header)
OK, ERR_INVALID, ERR_UNSUPPORTED, ERR_DEVICE, ERR_NOMEM = 0, 1, 2, 3, 4
COMM_ID_BYTES = 128
REDUCE_SUM, REDUCE_MAX = 0, 1
F32, F64, I32 = 0, 1, 2

OP = dict(
    ADD=1, SUB=2, MUL=3, DIV=4, POW=5, GREATER=6, COND=7, LOGICAL_OR=8, LOGICAL_AND=9,
    MAX=10, MIN=11, MOD=12, ATAN2=13,
    NEG=32, SQUARE=33, CUBE=34, ABS=35, RELU=36, COS=37, SIN=38, TAN=39, EXP=40, LOG=41,
    LOG2=42, LOG10=43, LOG1P=44, SQRT=45, ACOSH=46, ATANH_CLIP=47, SINH=48, COSH=49, TANH=50,
    ASIN=51, ACOS=52, ATAN=53, ASINH=54, ERF=55, ERFC=56, GAMMA=57, ROUND=58, FLOOR=59,
    CEIL=60, SIGN=61, EXP2=62, EXPM1=63, CBRT=64,
)
LOSS = dict(
    L2=0, L1=1, LP=2, HUBER=3, L1_EPS_INS=4, L2_EPS_INS=5, LOGIT_DIST=6, PERIODIC=7, QUANTILE=8,
    ZERO_ONE=9, PERCEPTRON=10, LOGIT_MARGIN=11, L1_HINGE=12, L2_HINGE=13, SMOOTHED_L1_HINGE=14,
    MODIFIED_HUBER=15, L2_MARGIN=16, EXP=17, SIGMOID=18, DWD_MARGIN=19,
)

# struct srhip_node (24 bytes)
NODE_DTYPE = np.dtype(
    [("degree", "u1"), ("constant", "u1"), ("op", "<u2"), ("feature", "<u2"), ("pad", "<u2"),
     ("l", "<i4"), ("r", "<i4"), ("val", "<f8")],
    align=True,
)
assert NODE_DTYPE.itemsize == 24


class Operators(ctypes.Structure):
    _fields_ = [("nbin", ctypes.c_int32), ("nuna", ctypes.c_int32),
                ("binops", ctypes.POINTER(ctypes.c_int32)), ("unaops", ctypes.POINTER(ctypes.c_int32))]


class Loss(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("p0", ctypes.c_double), ("p1", ctypes.c_double)]


class OptimOptions(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("nrestarts", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("g_tol", ctypes.c_double)]


class SrhipError(RuntimeError):
    """A nonzero status from libsrhip (message from srhip_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"srhip error {code}: {msg}")
        self.code = code


# Every symbol include/srhip.h declares, with its ctypes signature.
_vp, _i32, _i64, _dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
SIGNATURES = {
    "srhip_last_error": (ctypes.c_char_p, []),
    "srhip_version": (ctypes.c_char_p, []),
    "srhip_device_count": (ctypes.c_int, []),
    "srhip_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "srhip_ctx_destroy": (None, [_vp]),
    "srhip_ctx_synchronize": (ctypes.c_int, [_vp]),
    "srhip_dataset_create": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _i64, _i64, _i64, _i64, _vp, _vp,
                                            ctypes.POINTER(_vp)]),
    "srhip_dataset_destroy": (None, [_vp]),
    "srhip_program_create": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _i32, ctypes.POINTER(Operators),
                                            ctypes.POINTER(_vp)]),
    "srhip_program_destroy": (None, [_vp]),
    "srhip_program_num_constants": (ctypes.c_int, [_vp, _vp]),
    "srhip_program_set_constants": (ctypes.c_int, [_vp, _vp]),
    "srhip_program_get_constants": (ctypes.c_int, [_vp, _vp]),
    "srhip_eval_loss": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64, _vp, _vp]),
    "srhip_eval_predict": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "srhip_eval_loss_submit": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64, ctypes.POINTER(_vp)]),
    "srhip_eval_loss_wait": (ctypes.c_int, [_vp, _vp, _vp]),
    "srhip_eval_loss_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, ctypes.POINTER(Operators),
                                             ctypes.POINTER(Loss), _vp, _i64, _vp, _vp]),
    "srhip_eval_loss_partials": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64, _vp, _vp]),
    "srhip_partials_finalize": (ctypes.c_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "srhip_eval_precise_partials": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _i32, _vp]),
    "srhip_precise_finalize": (ctypes.c_int, [_vp, _vp, _i32, _vp, _vp]),
    "srhip_chk_reduce_op": (ctypes.c_int, [ctypes.c_int]),
    "srhip_program_max_ops": (_i32, [_vp]),
    "srhip_eval_loss_grad": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64, _vp, _vp, _vp]),
    "srhip_eval_grad_predict": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp, _vp, _vp]),
    "srhip_optimize_constants": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64,
                                                ctypes.POINTER(OptimOptions), _vp, _vp, _vp]),
    "srhip_optimize_constants_starts": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64,
                                                       ctypes.POINTER(OptimOptions), _vp, _vp, _vp, _vp, _vp]),
    "srhip_batcher_create": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(Operators), ctypes.POINTER(Loss), _i32, _i32,
                                            ctypes.POINTER(_vp)]),
    "srhip_batcher_set_clients": (ctypes.c_int, [_vp, _i32]),
    "srhip_batcher_submit": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, ctypes.POINTER(ctypes.c_uint64)]),
    "srhip_batcher_wait": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(_dbl), ctypes.POINTER(ctypes.c_uint8)]),
    "srhip_batcher_eval": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, ctypes.POINTER(_dbl),
                                          ctypes.POINTER(ctypes.c_uint8)]),
    "srhip_batcher_stats": (ctypes.c_int, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "srhip_batcher_timing": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "srhip_batcher_destroy": (None, [_vp]),
    "srhip_comm_unique_id": (ctypes.c_int, [_vp]),
    "srhip_comm_create": (ctypes.c_int, [_vp, _vp, _i32, _i32, ctypes.POINTER(_vp)]),
    "srhip_comm_destroy": (None, [_vp]),
    "srhip_comm_size": (ctypes.c_int, [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "srhip_comm_stats": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "srhip_comm_allreduce_f64": (ctypes.c_int, [_vp, _vp, _i64, _i32]),
    "srhip_comm_allgather": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "srhip_comm_migrate_start": (ctypes.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _i32]),
    "srhip_comm_migrate_wait": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "srhip_eval_loss_sharded": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.POINTER(Loss), _vp, _i64, _vp, _vp]),
    "srhip_last_kernel_ms": (_dbl, [_vp]),
    "srhip_last_work": (ctypes.c_int, [_vp, ctypes.POINTER(_i64)]),
    "srhip_program_stats": (ctypes.c_int, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                                           ctypes.POINTER(_i32)]),
    "srhip_program_derived": (ctypes.c_int, [_vp, ctypes.POINTER(_i32), _vp, _i32]),
    "srhip_code_cache_stats": (ctypes.c_int, [ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
}

_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Load libsrhip.so (once). Raises SrhipError if the in-tree build is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise SrhipError(ERR_DEVICE, f"{LIB_PATH} not built: run `make -C symbolicregression.jl_amd` "
                                         "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                # an older library build (same-box A/B of builds via SRHIP_LIB): the call raises when used;
                # tests/test_abi.py requires every symbol of the in-tree build
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(code: int) -> None:
    if code != OK:
        msg = load().srhip_last_error().decode(errors="replace")
        raise SrhipError(code, msg)


def ptr(a: np.ndarray | None) -> ctypes.c_void_p | None:
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


def dtype_code(dt) -> int:
    dt = np.dtype(dt)
    if dt == np.float32:
        return F32
    if dt == np.float64:
        return F64
    if dt == np.int32:
        return I32
    raise SrhipError(ERR_UNSUPPORTED, f"element type {dt} is not supported on the device "
                                      "(Float32, Float64, Int32 only)")
