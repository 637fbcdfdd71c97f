"""srhip — MI355X-native (gfx950) batched expression evaluation for SymbolicRegression.jl's hot
path, behind the reference's own API names (eval_tree_array, eval_loss, score_func, Options,
Dataset, Node).  The compute runs in libsrhip.so (HIP kernels + C ABI, include/srhip.h);
this package is the host-side mirror of the reference interface.
"""
from ._lib import SrhipError, LIB_PATH
from .api import (
    batch_sample,
    compile_trees,
    compute_complexity,
    dimensional_regularization,
    eval_loss,
    eval_loss_batch,
    eval_loss_batched,
    eval_diff_tree_array,
    eval_grad_loss_batch,
    eval_grad_tree_array,
    eval_tree_array,
    eval_tree_array_batch,
    finalize_scores,
    LossCache,
    optimize_constants,
    loss_to_score,
    rescore_hall_of_fame,
    rescore_population_batched,
    score_func,
    score_func_batch,
    score_func_batched,
    trees_equal,
    update_baseline_loss,
)
from .dataset import Dataset
from .device import Coalescer, Context, DeviceDataset, Program, device_count, get_context
from .losses import (
    DWDMarginLoss,
    ExpLoss,
    HingeLoss,
    L1HingeLoss,
    L2HingeLoss,
    L2MarginLoss,
    LogitMarginLoss,
    MarginLoss,
    ModifiedHuberLoss,
    PerceptronLoss,
    SigmoidLoss,
    SmoothedL1HingeLoss,
    ZeroOneLoss,
    HuberLoss,
    L1DistLoss,
    L1EpsilonInsLoss,
    L2DistLoss,
    L2EpsilonInsLoss,
    LogitDistLoss,
    LPDistLoss,
    PeriodicLoss,
    QuantileLoss,
)
from .node import Node, count_constants, count_depth, count_nodes, flatten, get_constants, set_constants, string_tree, unflatten
from .operators import (
    cond,
    cos,
    cosh,
    cube,
    exp,
    exp2,
    greater,
    logical_and,
    logical_or,
    mult,
    neg,
    plus,
    relu,
    safe_acosh,
    safe_log,
    safe_log1p,
    safe_log2,
    safe_log10,
    safe_pow,
    safe_sqrt,
    sin,
    sinh,
    square,
    sub,
    tan,
    tanh,
)
from .options import Options
from .random_trees import gen_random_tree_fixed_size, random_population
from .search import HallOfFame, MutationWeights, PopMember, SearchResult, equation_search

__version__ = "0.1.0"
