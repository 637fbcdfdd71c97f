"""Options: the subset of the reference's ``Options`` (src/OptionsStruct.jl:123-195,
src/Options.jl:379-801) that the evaluation / scoring path reads.

Defaults follow the reference: parsimony 0.0032 (src/Options.jl), elementwise_loss
L2DistLoss() (src/Options.jl:534-535), batch_size 50, maxsize 20, optimizer_iterations 8,
optimizer_nrestarts 2.  ``turbo`` / ``bumper`` are accepted and ignored (CPU-evaluator switches).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import losses as _losses
from ._lib import Operators
from .operators import INT_BINARY, INT_UNARY, resolve_binary, resolve_unary


@dataclass
class ComplexityMapping:
    """src/OptionsStruct.jl ComplexityMapping: per-operator / variable / constant complexity."""
    use: bool = False
    binop_complexities: tuple = ()
    unaop_complexities: tuple = ()
    variable_complexity: object = 1
    constant_complexity: float = 1


class Options:
    def __init__(
        self,
        binary_operators=("+", "-", "/", "*"),
        unary_operators=(),
        elementwise_loss=None,
        loss_function=None,
        parsimony: float = 0.0032,
        complexity_of_operators=None,
        complexity_of_constants=None,
        complexity_of_variables=None,
        batching: bool = False,
        batch_size: int = 50,
        maxsize: int = 20,
        turbo: bool = False,
        bumper: bool = False,
        optimizer_iterations: int = 8,
        optimizer_nrestarts: int = 2,
        optimizer_probability: float = 0.14,
        deterministic: bool = False,
        seed=None,
        device: int = 0,
        dimensional_constraint_penalty=None,
        dimensionless_constants_only: bool = False,
        **unused,
    ):
        # operator aliasing: binopmap / unaopmap (src/Options.jl:92-150)
        b = [resolve_binary(op) for op in binary_operators]
        u = [resolve_unary(op) for op in unary_operators]
        self.binary_operators = tuple(n for n, _ in b)
        self.unary_operators = tuple(n for n, _ in u)
        self.binop_codes = np.array([c for _, c in b], dtype=np.int32)
        self.unaop_codes = np.array([c for _, c in u], dtype=np.int32)
        self.nbin = len(b)
        self.nuna = len(u)
        if elementwise_loss is None:
            elementwise_loss = _losses.L2DistLoss()
        elif isinstance(elementwise_loss, str):
            elementwise_loss = _losses.by_name(elementwise_loss)
        self.elementwise_loss = elementwise_loss
        self.loss_function = loss_function
        self.parsimony = np.float32(parsimony)
        self.batching = batching
        self.batch_size = int(batch_size)
        self.maxsize = int(maxsize)
        self.turbo = turbo
        self.bumper = bumper
        self.optimizer_iterations = optimizer_iterations
        self.optimizer_nrestarts = optimizer_nrestarts
        self.optimizer_probability = optimizer_probability
        self.deterministic = deterministic
        self.seed = seed
        self.device = device
        # dimensional_regularization (src/LossFunctions.jl:217-227, src/OptionsStruct.jl)
        self.dimensional_constraint_penalty = (None if dimensional_constraint_penalty is None
                                               else np.float32(dimensional_constraint_penalty))
        self.dimensionless_constants_only = bool(dimensionless_constants_only)
        self.unused = unused
        use_cm = any(x is not None for x in (complexity_of_operators, complexity_of_constants, complexity_of_variables))
        cop = dict(complexity_of_operators or {})
        cop = {resolve_binary(k)[0] if self._is_bin(k) else resolve_unary(k)[0]: v for k, v in cop.items()}
        self.complexity_mapping = ComplexityMapping(
            use=use_cm,
            binop_complexities=tuple(cop.get(n, 1) for n in self.binary_operators),
            unaop_complexities=tuple(cop.get(n, 1) for n in self.unary_operators),
            variable_complexity=1 if complexity_of_variables is None else complexity_of_variables,
            constant_complexity=1 if complexity_of_constants is None else complexity_of_constants,
        )
        self._c_ops = None

    @staticmethod
    def _is_bin(k):
        try:
            resolve_binary(k)
            return True
        except ValueError:
            return False

    # ---- operator index resolution (Node.op may be a name or a 1-based index) -------------------
    def binary_index(self, op) -> int:
        if isinstance(op, (int, np.integer)):
            if not 1 <= op <= self.nbin:
                raise ValueError(f"binary op index {op} out of range 1..{self.nbin}")
            return int(op)
        name = resolve_binary(op)[0]
        try:
            return self.binary_operators.index(name) + 1
        except ValueError:
            raise ValueError(f"binary operator {name!r} is not in options.binary_operators "
                             f"{self.binary_operators}") from None

    def unary_index(self, op) -> int:
        if isinstance(op, (int, np.integer)):
            if not 1 <= op <= self.nuna:
                raise ValueError(f"unary op index {op} out of range 1..{self.nuna}")
            return int(op)
        name = resolve_unary(op)[0]
        try:
            return self.unary_operators.index(name) + 1
        except ValueError:
            raise ValueError(f"unary operator {name!r} is not in options.unary_operators "
                             f"{self.unary_operators}") from None

    def supports_int(self) -> bool:
        return all(n in INT_BINARY for n in self.binary_operators) and all(
            n in INT_UNARY for n in self.unary_operators)

    def __getstate__(self):
        # the cached C operator table holds raw pointers into this object's arrays: rebuilt on use
        d = dict(self.__dict__)
        d["_c_ops"] = None
        return d

    def c_operators(self) -> Operators:
        if self._c_ops is None:
            ops = Operators()
            ops.nbin = self.nbin
            ops.nuna = self.nuna
            ops.binops = self.binop_codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            ops.unaops = self.unaop_codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            self._c_ops = ops
        return self._c_ops
