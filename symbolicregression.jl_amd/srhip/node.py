"""Expression trees: the Python mirror of DynamicExpressions' ``Node{T}``.

Fields follow the reference's usage (src/Complexity.jl:36-42, src/MutationFunctions.jl:39-57):
``degree`` (0/1/2), ``constant`` (leaf), ``val``, ``feature`` (1-based), ``op`` and children
``l``/``r``.  ``op`` may be a 1-based index into the Options' operator list (as in Julia) or an
operator name resolved against the Options when the tree is flattened for the device.

Trees are built like in the reference tests: ``Node("x1")``, ``Node(val=3.0)``,
``Node(feature=2)``, ``x1 * Node(val=3.0)``, ``srhip.cos(x1 - 1.0)``, ``Node("cos", x1)``,
``Node(5, l, r)`` (binary op #5).
"""
from __future__ import annotations

import math
from typing import Iterable

import numpy as np

from ._lib import NODE_DTYPE


class Node:
    __slots__ = ("degree", "constant", "val", "feature", "op", "l", "r")

    def __init__(self, *args, val=None, feature=None, op=None, l=None, r=None):
        self.degree = 0
        self.constant = False
        self.val = 0.0
        self.feature = 0
        self.op = 0
        self.l = None
        self.r = None
        if args and isinstance(args[0], str) and len(args) == 1 and args[0][:1] == "x" and args[0][1:].isdigit():
            feature = int(args[0][1:])  # Node("x1")
            args = ()
        if len(args) == 2:
            op, l = args
        elif len(args) == 3:
            op, l, r = args
        elif len(args) == 1 and val is None and feature is None:
            # Node(T) in Julia: leaf with zero value; Node(3.0): constant
            if isinstance(args[0], (int, float, np.number)):
                val = args[0]
            else:
                raise TypeError(f"cannot build Node from {args!r}")
        elif args:
            raise TypeError(f"cannot build Node from {args!r}")
        if val is not None:
            self.constant = True
            self.val = val
        elif feature is not None:
            self.feature = int(feature)
        elif op is not None:
            self.op = op
            self.l = Node.lift(l)
            self.degree = 1
            if r is not None:
                self.r = Node.lift(r)
                self.degree = 2
        else:
            self.constant = True
            self.val = 0.0

    # ---- helpers ------------------------------------------------------------------------------
    @staticmethod
    def lift(x) -> "Node":
        if isinstance(x, Node):
            return x
        if isinstance(x, (int, float, np.number)):
            return Node(val=x)
        if isinstance(x, str):
            return Node(x)
        raise TypeError(f"cannot use {x!r} as a tree")

    def copy(self) -> "Node":
        n = Node.__new__(Node)
        n.degree, n.constant, n.val, n.feature, n.op = self.degree, self.constant, self.val, self.feature, self.op
        n.l = self.l.copy() if self.l is not None else None
        n.r = self.r.copy() if self.r is not None else None
        return n

    def set_node(self, other: "Node") -> None:
        """set_node! (DynamicExpressions): overwrite this node in place with other's fields."""
        self.degree, self.constant, self.val, self.feature, self.op = (
            other.degree, other.constant, other.val, other.feature, other.op)
        self.l, self.r = other.l, other.r

    def __iter__(self):  # depth-first, node before children (DynamicExpressions foreach order)
        stack = [self]
        while stack:
            n = stack.pop()
            yield n
            if n.degree == 2:
                stack.append(n.r)
            if n.degree >= 1:
                stack.append(n.l)

    # ---- operator overloading (needs the operator in Options when flattened) -------------------
    def __add__(self, o): return Node("+", self, Node.lift(o))
    def __radd__(self, o): return Node("+", Node.lift(o), self)
    def __sub__(self, o): return Node("-", self, Node.lift(o))
    def __rsub__(self, o): return Node("-", Node.lift(o), self)
    def __mul__(self, o): return Node("*", self, Node.lift(o))
    def __rmul__(self, o): return Node("*", Node.lift(o), self)
    def __truediv__(self, o): return Node("/", self, Node.lift(o))
    def __rtruediv__(self, o): return Node("/", Node.lift(o), self)
    def __pow__(self, o): return Node("^", self, Node.lift(o))
    def __rpow__(self, o): return Node("^", Node.lift(o), self)
    def __neg__(self): return Node("neg", self)

    def __repr__(self):
        return string_tree(self)


# ---- tree utilities ---------------------------------------------------------------------------
def count_nodes(tree: Node) -> int:
    return sum(1 for _ in tree)


def count_constants(tree: Node) -> int:
    return sum(1 for n in tree if n.degree == 0 and n.constant)


def get_constants(tree: Node) -> np.ndarray:
    """Constants in DynamicExpressions get_constants order (depth-first, left to right)."""
    return np.array([n.val for n in tree if n.degree == 0 and n.constant], dtype=np.float64)


def set_constants(tree: Node, consts: Iterable[float]) -> None:
    it = iter(consts)
    for n in tree:
        if n.degree == 0 and n.constant:
            n.val = next(it)


def count_depth(tree: Node) -> int:
    if tree.degree == 0:
        return 1
    if tree.degree == 1:
        return 1 + count_depth(tree.l)
    return 1 + max(count_depth(tree.l), count_depth(tree.r))


def _op_name(op, ops, deg):
    if isinstance(op, str):
        return op
    if ops is not None:
        lst = ops.binary_operators if deg == 2 else ops.unary_operators
        return lst[op - 1]
    return f"op{op}"


def string_tree(tree: Node, options=None) -> str:
    if tree.degree == 0:
        if tree.constant:
            return repr(float(tree.val)) if not isinstance(tree.val, (int, np.integer)) else str(tree.val)
        return f"x{tree.feature}"
    name = _op_name(tree.op, options, tree.degree)
    if tree.degree == 1:
        return f"{name}({string_tree(tree.l, options)})"
    a, b = string_tree(tree.l, options), string_tree(tree.r, options)
    if name in ("+", "-", "*", "/", "^"):
        return f"({a} {name} {b})"
    return f"{name}({a}, {b})"


def flatten(trees, options, dtype=np.float32):
    """Flatten trees into the srhip_node table + tree offsets (C ABI layout, include/srhip.h).

    Node 0 of each run is the root; children are indices within the run.  Operator names are
    mapped to the 1-based indices of ``options.binary_operators`` / ``unary_operators``.
    """
    if isinstance(trees, Node):
        trees = [trees]
    rows = []
    offsets = [0]
    for tree in trees:
        start = len(rows)
        # iterative preorder with explicit indices
        stack = [(tree, -1, 0)]  # node, parent row, which child (1 = l, 2 = r)
        while stack:
            n, parent, side = stack.pop()
            idx = len(rows) - start
            if n.degree == 0:
                if n.constant:
                    rows.append((0, 1, 0, 0, 0, -1, -1, float(n.val)))
                else:
                    rows.append((0, 0, 0, int(n.feature), 0, -1, -1, 0.0))
            elif n.degree == 1:
                rows.append((1, 0, options.unary_index(n.op), 0, 0, -1, -1, 0.0))
                stack.append((n.l, idx, 1))
            else:
                rows.append((2, 0, options.binary_index(n.op), 0, 0, -1, -1, 0.0))
                stack.append((n.r, idx, 2))
                stack.append((n.l, idx, 1))
            if parent >= 0:
                prow = list(rows[start + parent])
                prow[5 if side == 1 else 6] = idx
                rows[start + parent] = tuple(prow)
        offsets.append(len(rows))
    arr = np.array(rows, dtype=NODE_DTYPE) if rows else np.zeros(0, dtype=NODE_DTYPE)
    if np.dtype(dtype) == np.float32:
        # Node{Float32} stores Float32 constants: round once here (exact afterwards)
        arr["val"] = arr["val"].astype(np.float32).astype(np.float64)
    elif np.dtype(dtype) == np.int32:
        v = arr["val"]
        if np.any(np.isfinite(v) & (v != np.round(v))):
            raise ValueError("non-integer constant in an Int32 tree")
    return arr, np.asarray(offsets, dtype=np.int64)


def unflatten(nodes: np.ndarray, offsets: np.ndarray, options=None) -> list:
    """Inverse of flatten (operator indices are kept as 1-based ints)."""
    out = []
    for t in range(len(offsets) - 1):
        base = int(offsets[t])

        def build(i):
            rec = nodes[base + i]
            d = int(rec["degree"])
            if d == 0:
                if rec["constant"]:
                    return Node(val=float(rec["val"]))
                return Node(feature=int(rec["feature"]))
            if d == 1:
                return Node(int(rec["op"]), build(int(rec["l"])))
            return Node(int(rec["op"]), build(int(rec["l"])), build(int(rec["r"])))

        out.append(build(0))
    return out


def is_finite_scalar(x) -> bool:
    try:
        return math.isfinite(float(x))
    except (TypeError, ValueError):
        return False
