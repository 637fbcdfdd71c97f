"""Operator table: reference operator names -> device op codes.

Mirrors the reference's operator aliasing (``binopmap`` / ``unaopmap``, src/Options.jl:92-150:
``^`` -> ``safe_pow``, ``log`` -> ``safe_log``, ``sqrt`` -> ``safe_sqrt``, ``acosh`` ->
``safe_acosh``, ``atanh`` -> ``atanh_clip``, ``plus``/``sub``/``mult`` -> ``+ - *``) and the
scalar semantics of src/Operators.jl (implemented on the device in csrc/srhip_ops.h).

Operators may be given as names (``"+"``, ``"cos"``, ``"safe_log"``), as NumPy ufuncs /
``math`` functions (matched by ``__name__``), or as the builder functions exported by this module.
"""
from __future__ import annotations

import math

import numpy as np

from ._lib import OP

# name -> (canonical name, device code)
BINARY = {
    "+": ("+", OP["ADD"]), "plus": ("+", OP["ADD"]), "add": ("+", OP["ADD"]),
    "-": ("-", OP["SUB"]), "sub": ("-", OP["SUB"]), "subtract": ("-", OP["SUB"]),
    "*": ("*", OP["MUL"]), "mult": ("*", OP["MUL"]), "multiply": ("*", OP["MUL"]),
    "/": ("/", OP["DIV"]), "div": ("/", OP["DIV"]), "divide": ("/", OP["DIV"]), "true_divide": ("/", OP["DIV"]),
    "^": ("^", OP["POW"]), "pow": ("^", OP["POW"]), "safe_pow": ("^", OP["POW"]), "power": ("^", OP["POW"]),
    "greater": ("greater", OP["GREATER"]), "cond": ("cond", OP["COND"]),
    "logical_or": ("logical_or", OP["LOGICAL_OR"]), "logical_and": ("logical_and", OP["LOGICAL_AND"]),
    "max": ("max", OP["MAX"]), "maximum": ("max", OP["MAX"]),
    "min": ("min", OP["MIN"]), "minimum": ("min", OP["MIN"]),
    "mod": ("mod", OP["MOD"]), "atan2": ("atan2", OP["ATAN2"]), "arctan2": ("atan2", OP["ATAN2"]),
}
UNARY = {
    "neg": ("neg", OP["NEG"]), "negative": ("neg", OP["NEG"]),
    "square": ("square", OP["SQUARE"]), "cube": ("cube", OP["CUBE"]),
    "abs": ("abs", OP["ABS"]), "absolute": ("abs", OP["ABS"]), "fabs": ("abs", OP["ABS"]),
    "relu": ("relu", OP["RELU"]),
    "cos": ("cos", OP["COS"]), "sin": ("sin", OP["SIN"]), "tan": ("tan", OP["TAN"]),
    "exp": ("exp", OP["EXP"]),
    "log": ("safe_log", OP["LOG"]), "safe_log": ("safe_log", OP["LOG"]),
    "log2": ("safe_log2", OP["LOG2"]), "safe_log2": ("safe_log2", OP["LOG2"]),
    "log10": ("safe_log10", OP["LOG10"]), "safe_log10": ("safe_log10", OP["LOG10"]),
    "log1p": ("safe_log1p", OP["LOG1P"]), "safe_log1p": ("safe_log1p", OP["LOG1P"]),
    "sqrt": ("safe_sqrt", OP["SQRT"]), "safe_sqrt": ("safe_sqrt", OP["SQRT"]),
    "acosh": ("safe_acosh", OP["ACOSH"]), "safe_acosh": ("safe_acosh", OP["ACOSH"]),
    "arccosh": ("safe_acosh", OP["ACOSH"]),
    "atanh": ("atanh_clip", OP["ATANH_CLIP"]), "atanh_clip": ("atanh_clip", OP["ATANH_CLIP"]),
    "arctanh": ("atanh_clip", OP["ATANH_CLIP"]),
    "sinh": ("sinh", OP["SINH"]), "cosh": ("cosh", OP["COSH"]), "tanh": ("tanh", OP["TANH"]),
    "asin": ("asin", OP["ASIN"]), "arcsin": ("asin", OP["ASIN"]),
    "acos": ("acos", OP["ACOS"]), "arccos": ("acos", OP["ACOS"]),
    "atan": ("atan", OP["ATAN"]), "arctan": ("atan", OP["ATAN"]),
    "asinh": ("asinh", OP["ASINH"]), "arcsinh": ("asinh", OP["ASINH"]),
    "erf": ("erf", OP["ERF"]), "erfc": ("erfc", OP["ERFC"]), "gamma": ("gamma", OP["GAMMA"]),
    "round": ("round", OP["ROUND"]), "rint": ("round", OP["ROUND"]),
    "floor": ("floor", OP["FLOOR"]), "ceil": ("ceil", OP["CEIL"]), "sign": ("sign", OP["SIGN"]),
    "exp2": ("exp2", OP["EXP2"]), "expm1": ("expm1", OP["EXPM1"]), "cbrt": ("cbrt", OP["CBRT"]),
}
INT_BINARY = {"+", "-", "*", "greater", "cond", "logical_or", "logical_and", "max", "min"}
INT_UNARY = {"neg", "square", "cube", "abs", "relu", "sign"}


def _name_of(op) -> str:
    if isinstance(op, str):
        return op
    name = getattr(op, "__srhip_name__", None) or getattr(op, "__name__", None)
    if name is None:
        raise ValueError(f"cannot identify operator {op!r}")
    return name


def resolve_binary(op) -> tuple[str, int]:
    """binopmap (src/Options.jl:92-107): return (canonical name, device code)."""
    name = _name_of(op)
    if name not in BINARY:
        raise ValueError(f"binary operator {name!r} has no device implementation")
    return BINARY[name]


def resolve_unary(op) -> tuple[str, int]:
    """unaopmap (src/Options.jl:114-131): return (canonical name, device code)."""
    name = _name_of(op)
    if name not in UNARY:
        raise ValueError(f"unary operator {name!r} has no device implementation")
    return UNARY[name]


# ---- tree-building helpers (operate on Node, fall back to math on numbers) ---------------------
def _unary_builder(name, fallback):
    def f(x):
        from .node import Node

        if isinstance(x, Node):
            return Node(name, x)
        return fallback(x)

    f.__name__ = name
    f.__srhip_name__ = name
    return f


def _binary_builder(name, fallback):
    def f(x, y):
        from .node import Node

        if isinstance(x, Node) or isinstance(y, Node):
            return Node(name, Node.lift(x), Node.lift(y))
        return fallback(x, y)

    f.__name__ = name
    f.__srhip_name__ = name
    return f


def _safe_pow(x, y):
    if float(y).is_integer():
        if y < 0 and x == 0:
            return math.nan
    else:
        if y > 0 and x < 0:
            return math.nan
        if y < 0 and x <= 0:
            return math.nan
    return x ** y


cos = _unary_builder("cos", np.cos)
sin = _unary_builder("sin", np.sin)
tan = _unary_builder("tan", np.tan)
exp = _unary_builder("exp", np.exp)
safe_log = _unary_builder("safe_log", lambda x: np.log(x) if x > 0 else math.nan)
safe_log2 = _unary_builder("safe_log2", lambda x: np.log2(x) if x > 0 else math.nan)
safe_log10 = _unary_builder("safe_log10", lambda x: np.log10(x) if x > 0 else math.nan)
safe_log1p = _unary_builder("safe_log1p", lambda x: np.log1p(x) if x > -1 else math.nan)
safe_sqrt = _unary_builder("safe_sqrt", lambda x: np.sqrt(x) if x >= 0 else math.nan)
safe_acosh = _unary_builder("safe_acosh", lambda x: np.arccosh(x) if x >= 1 else math.nan)
square = _unary_builder("square", lambda x: x * x)
cube = _unary_builder("cube", lambda x: x * x * x)
neg = _unary_builder("neg", lambda x: -x)
relu = _unary_builder("relu", lambda x: x if x > 0 else math.copysign(0.0, x))
sinh = _unary_builder("sinh", np.sinh)
cosh = _unary_builder("cosh", np.cosh)
tanh = _unary_builder("tanh", np.tanh)
atan = _unary_builder("atan", np.arctan)
exp2 = _unary_builder("exp2", np.exp2)
safe_pow = _binary_builder("^", _safe_pow)
greater = _binary_builder("greater", lambda x, y: 1.0 if x > y else 0.0)
cond = _binary_builder("cond", lambda x, y: y if x > 0 else math.copysign(0.0, y))
logical_or = _binary_builder("logical_or", lambda x, y: 1.0 if (x > 0 or y > 0) else 0.0)
logical_and = _binary_builder("logical_and", lambda x, y: 1.0 if (x > 0 and y > 0) else 0.0)
plus = _binary_builder("+", lambda x, y: x + y)
sub = _binary_builder("-", lambda x, y: x - y)
mult = _binary_builder("*", lambda x, y: x * y)


def _jl_mod(x, y):
    """Julia mod: floored, sign of the divisor."""
    r = np.fmod(x, y)
    return r + y if (r != 0 and (r < 0) != (y < 0)) else r


# Host scalar semantics by canonical name (src/Operators.jl; Julia Base): used by the search's
# simplification (constant folding), never by evaluation — the device does that.
_SCALAR_UNARY = {
    "neg": lambda x: -x, "square": lambda x: x * x, "cube": lambda x: x * x * x, "abs": abs,
    "relu": lambda x: x if x > 0 else x * 0, "cos": np.cos, "sin": np.sin, "tan": np.tan, "exp": np.exp,
    "safe_log": lambda x: np.log(x) if x > 0 else math.nan, "safe_log2": lambda x: np.log2(x) if x > 0 else math.nan,
    "safe_log10": lambda x: np.log10(x) if x > 0 else math.nan,
    "safe_log1p": lambda x: np.log1p(x) if x > -1 else math.nan,
    "safe_sqrt": lambda x: np.sqrt(x) if x >= 0 else math.nan,
    "safe_acosh": lambda x: np.arccosh(x) if x >= 1 else math.nan,
    "atanh_clip": lambda x: np.arctanh(_jl_mod(x + 1, type(x)(2)) - 1),
    "sinh": np.sinh, "cosh": np.cosh, "tanh": np.tanh, "asin": np.arcsin, "acos": np.arccos, "atan": np.arctan,
    "asinh": np.arcsinh, "erf": lambda x: type(x)(math.erf(x)), "erfc": lambda x: type(x)(math.erfc(x)),
    "gamma": lambda x: type(x)(math.gamma(x)) if np.isfinite(x) and not (x <= 0 and x == int(x)) else math.nan,
    "round": np.rint, "floor": np.floor, "ceil": np.ceil, "sign": np.sign, "exp2": np.exp2, "expm1": np.expm1,
    "cbrt": np.cbrt,
}
_SCALAR_BINARY = {
    "+": lambda x, y: x + y, "-": lambda x, y: x - y, "*": lambda x, y: x * y, "/": lambda x, y: x / y,
    "^": _safe_pow, "greater": lambda x, y: type(x)(1) if x > y else type(x)(0),
    "cond": lambda x, y: y if x > 0 else y * 0,
    "logical_or": lambda x, y: type(x)(1) if (x > 0 or y > 0) else type(x)(0),
    "logical_and": lambda x, y: type(x)(1) if (x > 0 and y > 0) else type(x)(0),
    "max": lambda x, y: x if (x != x or x > y) else y, "min": lambda x, y: x if (x != x or x < y) else y,
    "mod": _jl_mod, "atan2": np.arctan2,
}


def scalar_op(name: str, vals):
    """Apply the operator `name` (canonical) to scalar NumPy values (host, for simplification)."""
    try:
        if len(vals) == 1:
            return vals[0].dtype.type(_SCALAR_UNARY[name](vals[0]))
        return vals[0].dtype.type(_SCALAR_BINARY[name](vals[0], vals[1]))
    except (ValueError, OverflowError, ZeroDivisionError, KeyError):
        return math.nan
