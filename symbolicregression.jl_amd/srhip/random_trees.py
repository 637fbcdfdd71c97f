"""Random trees with the reference's distribution, for synthetic benchmark / test populations.

Restates src/MutationFunctions.jl: ``make_random_leaf`` (:167-175: 50 % randn constant / 50 %
uniform feature), ``append_random_op`` (:95-125: a uniformly random leaf becomes an operator
node, binary with probability nbin / (nbin + nuna), children random leaves) and
``gen_random_tree_fixed_size`` (:249-268).  NumPy's Generator replaces Julia's RNG, so the
streams differ; the distribution is the same.
"""
from __future__ import annotations

import numpy as np

from .node import Node, count_nodes


def make_random_leaf(nfeatures: int, dtype, rng) -> Node:
    if rng.random() < 0.5:
        v = rng.standard_normal()
        return Node(val=float(np.dtype(dtype).type(v)))
    return Node(feature=int(rng.integers(1, nfeatures + 1)))


def append_random_op(tree: Node, options, nfeatures: int, dtype, rng, make_new_bin_op=None) -> Node:
    leaves = [n for n in tree if n.degree == 0]
    node = leaves[int(rng.integers(0, len(leaves)))]
    if make_new_bin_op is None:
        make_new_bin_op = rng.random() < options.nbin / (options.nuna + options.nbin)
    if make_new_bin_op:
        new = Node(int(rng.integers(1, options.nbin + 1)), make_random_leaf(nfeatures, dtype, rng),
                   make_random_leaf(nfeatures, dtype, rng))
    else:
        new = Node(int(rng.integers(1, options.nuna + 1)), make_random_leaf(nfeatures, dtype, rng))
    node.set_node(new)
    return tree


def gen_random_tree_fixed_size(node_count: int, options, nfeatures: int, dtype, rng) -> Node:
    tree = make_random_leaf(nfeatures, dtype, rng)
    cur = count_nodes(tree)
    while cur < node_count:
        if cur == node_count - 1:  # only a unary operator fits
            if options.nuna == 0:
                break
            tree = append_random_op(tree, options, nfeatures, dtype, rng, make_new_bin_op=False)
        else:
            tree = append_random_op(tree, options, nfeatures, dtype, rng)
        cur = count_nodes(tree)
    return tree


def random_population(ntrees: int, options, nfeatures: int, dtype, seed: int, max_size: int = 30):
    """C2's tree set: sizes ~ U{1..max_size} (as src/Mutate.jl:186 draws), fixed-size generator."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(1, max_size + 1, size=ntrees)
    return [gen_random_tree_fixed_size(int(s), options, nfeatures, dtype, rng) for s in sizes]
