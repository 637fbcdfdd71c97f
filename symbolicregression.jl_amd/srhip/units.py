"""Dimensional analysis for ``dimensional_regularization``.

Restates src/DimensionalAnalysis.jl:1-216 and src/LossFunctions.jl:217-227: a tree violates its
dataset's units when evaluating it on ROW 1 of X with WildcardQuantity values breaks a dimensional
rule, or when its output dimension differs from y_units (unless the output is a wildcard).  The
penalty (1000, or options.dimensional_constraint_penalty) is added to the device loss by
``eval_loss(...; regularization=true)``: the check is O(nodes) scalar host work per tree, and the
device never needs it.

DynamicQuantities (the reference's unit library, absent here) is restated only as far as this path
uses it: a Quantity is a value with a vector of 7 rational SI exponents (length, mass, time, current,
temperature, luminosity, amount); ``uparse`` reads unit strings such as "m/s^2", "km/s", "kg",
"m^3", "hr", "1".

WildcardQuantity semantics (DimensionalAnalysis.jl:41-154), per device operator:
  + -          same dimensions -> ok (wildcard iff both are); one side a wildcard -> it takes the
               other's dimensions; otherwise violation
  * /          dimensions add / subtract, wildcard if either is
  ^ (safe_pow) both sides dimensionless or wildcards -> dimensionless value; otherwise violation
  sqrt, cbrt, abs   halve / third / keep the dimensions (sqrt of a negative value -> NaN)
  square, cube      x * x, x * x * x
  every other operator: no WildcardQuantity method, so only all-wildcard arguments pass
               (a dimensionless, non-wildcard result); anything else is a violation
  a non-finite argument is a violation (deg1_eval / deg2_eval :144,157)
"""
from __future__ import annotations

import math
import re
from fractions import Fraction

import numpy as np

from .operators import scalar_op

NDIM = 7  # length, mass, time, current, temperature, luminosity, amount
_ZERO = (Fraction(0),) * NDIM


def _dims(**kw):
    order = ("length", "mass", "time", "current", "temperature", "luminosity", "amount")
    return tuple(Fraction(kw.get(k, 0)) for k in order)


class Quantity:
    __slots__ = ("value", "dims")

    def __init__(self, value, dims=_ZERO):
        self.value = value
        self.dims = tuple(dims)

    def __repr__(self):
        return f"Quantity({self.value!r}, {self.dims})"

    def __eq__(self, o):
        return isinstance(o, Quantity) and self.value == o.value and self.dims == o.dims

    def dimensionless(self):
        return all(d == 0 for d in self.dims)


# ---- unit strings (uparse) -----------------------------------------------------------------------
_BASE = {
    "m": (1.0, _dims(length=1)), "g": (1e-3, _dims(mass=1)), "s": (1.0, _dims(time=1)),
    "A": (1.0, _dims(current=1)), "K": (1.0, _dims(temperature=1)), "cd": (1.0, _dims(luminosity=1)),
    "mol": (1.0, _dims(amount=1)),
    "N": (1.0, _dims(mass=1, length=1, time=-2)), "J": (1.0, _dims(mass=1, length=2, time=-2)),
    "W": (1.0, _dims(mass=1, length=2, time=-3)), "Pa": (1.0, _dims(mass=1, length=-1, time=-2)),
    "Hz": (1.0, _dims(time=-1)), "C": (1.0, _dims(current=1, time=1)),
    "V": (1.0, _dims(mass=1, length=2, time=-3, current=-1)),
    "Ω": (1.0, _dims(mass=1, length=2, time=-3, current=-2)), "Ohm": (1.0, _dims(mass=1, length=2, time=-3, current=-2)),
    "F": (1.0, _dims(mass=-1, length=-2, time=4, current=2)), "T": (1.0, _dims(mass=1, time=-2, current=-1)),
    "Wb": (1.0, _dims(mass=1, length=2, time=-2, current=-1)), "H": (1.0, _dims(mass=1, length=2, time=-2, current=-2)),
    "L": (1e-3, _dims(length=3)), "min": (60.0, _dims(time=1)), "hr": (3600.0, _dims(time=1)),
    "h": (3600.0, _dims(time=1)), "day": (86400.0, _dims(time=1)), "yr": (31557600.0, _dims(time=1)),
    "eV": (1.602176634e-19, _dims(mass=1, length=2, time=-2)),
}
_PREFIX = {"Y": 1e24, "Z": 1e21, "E": 1e18, "P": 1e15, "T": 1e12, "G": 1e9, "M": 1e6, "k": 1e3, "h": 1e2,
           "da": 1e1, "d": 1e-1, "c": 1e-2, "m": 1e-3, "μ": 1e-6, "u": 1e-6, "n": 1e-9, "p": 1e-12,
           "f": 1e-15, "a": 1e-18, "z": 1e-21, "y": 1e-24}
_NO_PREFIX = {"min", "hr", "h", "day", "yr"}


def _symbol(name: str) -> Quantity:
    if name in _BASE:
        v, d = _BASE[name]
        return Quantity(v, d)
    for p in sorted(_PREFIX, key=len, reverse=True):
        if name.startswith(p) and name[len(p):] in _BASE and name[len(p):] not in _NO_PREFIX:
            v, d = _BASE[name[len(p):]]
            return Quantity(_PREFIX[p] * v, d)
    raise ValueError(f"unknown unit {name!r}")


_TOKEN = re.compile(r"\s*(?:(\d+(?:\.\d*)?(?:[eE][-+]?\d+)?)|([A-Za-zΩμ]+)|(\*\*|[*/^()·]|-))")


def uparse(s) -> Quantity:
    """DynamicQuantities.uparse for products / quotients / integer or rational powers of the symbols
    above; "" and "1" are dimensionless."""
    if isinstance(s, Quantity):
        return s
    if isinstance(s, (int, float, np.number)):
        return Quantity(float(s))
    s = str(s).strip()
    if s in ("", "1"):
        return Quantity(1.0)
    toks = []
    pos = 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise ValueError(f"cannot parse unit {s!r}")
        toks.append(m.group(1) or m.group(2) or m.group(3))
        pos = m.end()
    toks = ["^" if t == "**" else ("*" if t == "·" else t) for t in toks]
    it = iter(toks + [None])
    cur = [next(it)]

    def take():
        t = cur[0]
        cur[0] = next(it)
        return t

    def power():
        neg = False
        if cur[0] == "-":
            take()
            neg = True
        if cur[0] == "(":
            take()
            num = Fraction(take())
            if cur[0] == "/":
                take()
                num /= Fraction(take())
            assert take() == ")"
        else:
            num = Fraction(take())
        return -num if neg else num

    def factor():
        t = take()
        if t == "(":
            q = expr()
            if take() != ")":
                raise ValueError(f"unbalanced parentheses in {s!r}")
        elif re.fullmatch(r"\d+(?:\.\d*)?(?:[eE][-+]?\d+)?", t or ""):
            q = Quantity(float(t))
        elif t:
            q = _symbol(t)
        else:
            raise ValueError(f"cannot parse unit {s!r}")
        if cur[0] == "^":
            take()
            e = power()
            q = Quantity(q.value ** float(e), tuple(d * e for d in q.dims))
        return q

    def expr():
        q = factor()
        while cur[0] in ("*", "/"):
            op = take()
            r = factor()
            if op == "*":
                q = Quantity(q.value * r.value, tuple(a + b for a, b in zip(q.dims, r.dims)))
            else:
                q = Quantity(q.value / r.value, tuple(a - b for a, b in zip(q.dims, r.dims)))
        return q

    q = expr()
    if cur[0] is not None:
        raise ValueError(f"trailing tokens in unit {s!r}")
    return q


def get_units(units, nfeatures=None):
    """get_si_units (src/InterfaceDynamicQuantities.jl): a list of Quantity or None."""
    if units is None:
        return None
    if isinstance(units, (str, Quantity, int, float)):
        return uparse(units)
    out = [uparse(u) for u in units]
    if nfeatures is not None and len(out) != nfeatures:
        raise ValueError(f"{len(out)} units for {nfeatures} features")
    return out


# ---- WildcardQuantity ----------------------------------------------------------------------------
class W:
    __slots__ = ("q", "wildcard", "violates")

    def __init__(self, q: Quantity, wildcard: bool, violates: bool):
        self.q, self.wildcard, self.violates = q, wildcard, violates


def _bad(T):
    return W(Quantity(T(1)), False, True)


def _finite(w):
    return math.isfinite(float(w.q.value))


def _addsub(op, l, r, T):
    f = (lambda a, b: T(a) + T(b)) if op == "+" else (lambda a, b: T(a) - T(b))
    if l.q.dims == r.q.dims:
        return W(Quantity(T(f(l.q.value, r.q.value)), l.q.dims), l.wildcard and r.wildcard, False)
    if l.wildcard and r.wildcard:
        return W(Quantity(T(f(l.q.value, r.q.value)), l.q.dims), True, False)
    if l.wildcard:
        return W(Quantity(T(f(l.q.value, r.q.value)), r.q.dims), False, False)
    if r.wildcard:
        return W(Quantity(T(f(l.q.value, r.q.value)), l.q.dims), False, False)
    return _bad(T)


def _muldiv(op, l, r, T):
    a, b = T(l.q.value), T(r.q.value)  # IEEE in T (numpy scalars; errors ignored by the caller)
    if op == "*":
        q = Quantity(a * b, tuple(x + y for x, y in zip(l.q.dims, r.q.dims)))
    else:
        q = Quantity(a / b, tuple(x - y for x, y in zip(l.q.dims, r.q.dims)))
    return W(q, l.wildcard or r.wildcard, False)


def _unary(name, l, T):
    if name == "abs":
        return W(Quantity(abs(T(l.q.value)), l.q.dims), l.wildcard, False)
    if name == "safe_sqrt":  # safe_sqrt(x) = sqrt(x) on W; DimensionalAnalysis.jl:33-36 for the Quantity
        v = T(l.q.value)
        val = np.sqrt(abs(v)) * (T(math.nan) if v < 0 else T(1))
        return W(Quantity(val, tuple(d / 2 for d in l.q.dims)), l.wildcard, False)
    if name == "cbrt":
        return W(Quantity(T(np.cbrt(l.q.value)), tuple(d / 3 for d in l.q.dims)), l.wildcard, False)
    if name == "square":
        return _muldiv("*", l, l, T)
    if name == "cube":
        return _muldiv("*", _muldiv("*", l, l, T), l, T)
    if l.wildcard:  # deg1_eval fallback: op on the stripped value, dimensionless result
        return W(Quantity(scalar_op(name, [T(l.q.value)])), False, False)
    return _bad(T)


def _binary(name, l, r, T):
    if name in ("+", "-"):
        res = _addsub(name, l, r, T)
    elif name in ("*", "/"):
        res = _muldiv(name, l, r, T)
    elif name == "^":  # safe_pow(x, y) = x ^ y on W (DimensionalAnalysis.jl:95-106)
        if (l.q.dimensionless() or l.wildcard) and (r.q.dimensionless() or r.wildcard):
            res = W(Quantity(scalar_op("^", [T(l.q.value), T(r.q.value)])), False, False)
        else:
            res = _bad(T)
    else:
        res = _bad(T)
    if not res.violates:
        return res
    if l.wildcard and r.wildcard:  # deg2_eval fallback (:159-161)
        return W(Quantity(scalar_op(name, [T(l.q.value), T(r.q.value)])), False, False)
    return _bad(T)


def _eval(tree, x, x_units, options, allow_wildcards, T):
    if tree.degree == 0:
        if tree.constant:
            return W(Quantity(T(tree.val)), allow_wildcards, False)
        u = x_units[tree.feature - 1]
        return W(Quantity(T(x[tree.feature - 1]) * T(u.value), u.dims), False, False)  # x[f] * X_units[f]
    if tree.degree == 1:
        l = _eval(tree.l, x, x_units, options, allow_wildcards, T)
        if l.violates:
            return l
        if not _finite(l):
            return _bad(T)
        return _unary(options.unary_operators[options.unary_index(tree.op) - 1], l, T)
    l = _eval(tree.l, x, x_units, options, allow_wildcards, T)
    r = _eval(tree.r, x, x_units, options, allow_wildcards, T)
    if l.violates:
        return l
    if r.violates:
        return r
    if not (_finite(l) and _finite(r)):
        return _bad(T)
    return _binary(options.binary_operators[options.binary_index(tree.op) - 1], l, r, T)


def violates_dimensional_constraints(tree, dataset, options) -> bool:
    """src/DimensionalAnalysis.jl:187-216 (evaluated on row 1 of X)."""
    if dataset.X_units is None:
        return False
    T = dataset.X.dtype.type if dataset.X.dtype != np.int32 else np.float64
    allow = not getattr(options, "dimensionless_constants_only", False)
    with np.errstate(all="ignore"):
        out = _eval(tree, dataset.X[:, 0], dataset.X_units, options, allow, T)
    violates = out.violates
    if dataset.y_units is not None:
        violates |= (not out.wildcard) and out.q.dims != dataset.y_units.dims
    return bool(violates)
