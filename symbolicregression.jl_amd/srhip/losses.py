"""Elementwise losses (LossFunctions.jl 0.10/0.11 supervised losses: distance losses of
``diff = output - target``, margin losses of the agreement ``a = target * output``), as used by the
reference's ``_loss`` / ``_weighted_loss`` (src/LossFunctions.jl:13-33) and listed in its options
(src/Options.jl:209-229; re-exported at src/SymbolicRegression.jl:101-126).

Each class carries its device kind code; the device computes the loss per row in T and
reduces it (fused into the evaluation kernel).  A plain Python callable ``f(pred, target)``
(or ``f(pred, target, w)``) is also accepted as ``elementwise_loss``: predictions then come from
the device and the callable runs on the host, like a user-defined Julia loss in the reference.
"""
from __future__ import annotations

import numpy as np

from ._lib import LOSS, Loss


class SupervisedLoss:
    kind = None
    p0 = 0.0

    def c_struct(self) -> Loss:
        s = Loss()
        s.kind = self.kind
        s.p0 = float(self.p0)
        s.p1 = 0.0
        return s

    def __call__(self, pred, target):  # host value (numpy), same formulas as the device
        return self.value(np.asarray(pred), np.asarray(target))

    def __repr__(self):
        return f"{type(self).__name__}()"


class L2DistLoss(SupervisedLoss):
    kind = LOSS["L2"]

    def value(self, p, t):
        d = p - t
        return d * d


class L1DistLoss(SupervisedLoss):
    kind = LOSS["L1"]

    def value(self, p, t):
        return np.abs(p - t)


class LPDistLoss(SupervisedLoss):
    kind = LOSS["LP"]

    def __init__(self, P):
        self.p0 = float(P)

    def value(self, p, t):
        return np.abs(p - t) ** p.dtype.type(self.p0)


class HuberLoss(SupervisedLoss):
    kind = LOSS["HUBER"]

    def __init__(self, d=1.0):
        self.p0 = float(d)

    def value(self, p, t):
        d = p - t
        a = np.abs(d)
        dd = p.dtype.type(self.p0)
        half = p.dtype.type(0.5)
        return np.where(a <= dd, half * (d * d), dd * (a - half * dd))


class L1EpsilonInsLoss(SupervisedLoss):
    kind = LOSS["L1_EPS_INS"]

    def __init__(self, eps):
        self.p0 = float(eps)

    def value(self, p, t):
        return np.maximum(p.dtype.type(0), np.abs(p - t) - p.dtype.type(self.p0))


class L2EpsilonInsLoss(SupervisedLoss):
    kind = LOSS["L2_EPS_INS"]

    def __init__(self, eps):
        self.p0 = float(eps)

    def value(self, p, t):
        e = np.maximum(p.dtype.type(0), np.abs(p - t) - p.dtype.type(self.p0))
        return e * e


class LogitDistLoss(SupervisedLoss):
    kind = LOSS["LOGIT_DIST"]

    def value(self, p, t):
        er = np.exp(p - t)
        den = p.dtype.type(1) + er
        return -np.log(p.dtype.type(4) * er / (den * den))


class PeriodicLoss(SupervisedLoss):
    kind = LOSS["PERIODIC"]

    def __init__(self, c=2 * np.pi):
        self.p0 = float(c)

    def value(self, p, t):
        T = p.dtype.type
        return T(1) - np.cos((p - t) * (T(2) * T(np.pi)) / T(self.p0))


class QuantileLoss(SupervisedLoss):
    kind = LOSS["QUANTILE"]

    def __init__(self, tau):
        self.p0 = float(tau)

    def value(self, p, t):
        d = p - t
        T = p.dtype.type
        return d * (T(self.p0) - (d < 0).astype(p.dtype))


# ---- margin losses (LossFunctions.jl 0.11 src/losses/margin.jl, restated; the package is not in
# the container, so parity with it is unpinned -- the device is checked against the C oracle and
# these numpy forms) ----------------------------------------------------------------------------
class MarginLoss(SupervisedLoss):
    """value(pred, target) = L(target * pred)."""

    def value(self, p, t):
        return self.margin(t * p, p.dtype.type)


def _max0(x, T):
    return np.maximum(T(0), x)


class ZeroOneLoss(MarginLoss):
    kind = LOSS["ZERO_ONE"]

    def margin(self, a, T):
        return np.where(a < 0, T(1), T(0)).astype(a.dtype)


class PerceptronLoss(MarginLoss):
    kind = LOSS["PERCEPTRON"]

    def margin(self, a, T):
        return _max0(-a, T)


class LogitMarginLoss(MarginLoss):
    kind = LOSS["LOGIT_MARGIN"]

    def margin(self, a, T):
        return np.log1p(np.exp(-a))


class L1HingeLoss(MarginLoss):
    kind = LOSS["L1_HINGE"]

    def margin(self, a, T):
        return _max0(T(1) - a, T)


HingeLoss = L1HingeLoss


class L2HingeLoss(MarginLoss):
    kind = LOSS["L2_HINGE"]

    def margin(self, a, T):
        h = T(1) - a
        return np.where(a >= 1, T(0), h * h).astype(a.dtype)


class SmoothedL1HingeLoss(MarginLoss):
    kind = LOSS["SMOOTHED_L1_HINGE"]

    def __init__(self, gamma):
        self.p0 = float(gamma)

    def margin(self, a, T):
        g = T(self.p0)
        h = _max0(T(1) - a, T)
        return np.where(a >= T(1) - g, T(0.5) / g * (h * h), T(1) - g / T(2) - a).astype(a.dtype)


class ModifiedHuberLoss(MarginLoss):
    kind = LOSS["MODIFIED_HUBER"]

    def margin(self, a, T):
        h = _max0(T(1) - a, T)
        return np.where(a >= T(-1), h * h, -T(4) * a).astype(a.dtype)


class L2MarginLoss(MarginLoss):
    kind = LOSS["L2_MARGIN"]

    def margin(self, a, T):
        h = T(1) - a
        return h * h


class ExpLoss(MarginLoss):
    kind = LOSS["EXP"]

    def margin(self, a, T):
        return np.exp(-a)


class SigmoidLoss(MarginLoss):
    kind = LOSS["SIGMOID"]

    def margin(self, a, T):
        return T(1) - np.tanh(a)


class DWDMarginLoss(MarginLoss):
    kind = LOSS["DWD_MARGIN"]

    def __init__(self, q):
        self.p0 = float(q)

    def margin(self, a, T):
        q = T(self.p0)
        with np.errstate(divide="ignore", invalid="ignore"):
            far = (q ** q / (q + T(1)) ** (q + T(1))) / a ** q
        return np.where(a <= q / (q + T(1)), T(1) - a, far).astype(a.dtype)


_BY_NAME = {c.__name__: c for c in (L2DistLoss, L1DistLoss, LPDistLoss, HuberLoss, L1EpsilonInsLoss,
                                    L2EpsilonInsLoss, LogitDistLoss, PeriodicLoss, QuantileLoss,
                                    ZeroOneLoss, PerceptronLoss, LogitMarginLoss, L1HingeLoss, L2HingeLoss,
                                    ModifiedHuberLoss, L2MarginLoss, ExpLoss, SigmoidLoss)}
_BY_NAME["HingeLoss"] = L1HingeLoss


def by_name(name: str) -> SupervisedLoss:
    name = name.replace("()", "")
    if name not in _BY_NAME:
        raise ValueError(f"unknown loss {name!r}")
    return _BY_NAME[name]()


def is_device_loss(loss) -> bool:
    return isinstance(loss, SupervisedLoss)
