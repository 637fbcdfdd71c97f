/*
 * srhip.h — C ABI of libsrhip.so, the MI355X (gfx950) batched expression-evaluation
 * engine for SymbolicRegression.jl's hot path (eval_tree_array -> _eval_loss -> score_func).
 *
 * Every entry point is plain C: opaque handles, plain pointers and sizes, integer status.
 * No C++ exception crosses this boundary.  `did_succeed == false` is DATA (out_ok[t] == 0),
 * not an error.  On a nonzero status, srhip_last_error() returns a thread-local message.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   srhip_eval_loss        <- _eval_loss / eval_loss            src/LossFunctions.jl:45-75, 97-112
 *                             (batched over a population:       src/Population.jl:36-62,162-176,
 *                              src/SingleIteration.jl:64-82)
 *   srhip_eval_predict     <- eval_tree_array(tree, X, options) src/InterfaceDynamicExpressions.jl:56-63
 *                             (-> DynamicExpressions.eval_tree_array, external v0.16)
 *   srhip_dataset_create   <- Dataset{T,L}(X, y; weights)      src/Dataset.jl:98-225
 *   srhip_program_create   <- the Node{T} trees + options.operators (OperatorEnum)
 *                                                               src/Options.jl:92-150,673-681
 *   srhip_program_set_constants <- set_constants!/Optim's constant vector (constant optimizer)
 *                                                               src/ConstantOptimization.jl:43-81
 *   srhip_eval_loss_batch  <- score_func over many members (convenience: create+eval+destroy)
 *                                                               src/LossFunctions.jl:161-174
 */
#ifndef SRHIP_H
#define SRHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
enum {
  SRHIP_OK = 0,
  SRHIP_ERR_INVALID = 1,     /* malformed argument (bad tree, out-of-range feature, ...) */
  SRHIP_ERR_UNSUPPORTED = 2, /* operator / dtype / loss the device does not implement,  */
                             /* or a tree needing > 8 interpreter stack slots           */
  SRHIP_ERR_DEVICE = 3,      /* HIP runtime error                                       */
  SRHIP_ERR_NOMEM = 4
};

/* ---- element types (Dataset{T}) --------------------------------------------------------- */
enum { SRHIP_F32 = 0, SRHIP_F64 = 1, SRHIP_I32 = 2 };

/* ---- operator codes: the device's op table (reference src/Operators.jl + Julia Base).
 * options.operators.binops[i] / unaops[i] (1-based op index stored in Node.op) are mapped to
 * these codes by the host binding (Julia glue / Python mirror), after the reference's own
 * aliasing binopmap/unaopmap (src/Options.jl:92-150): ^ -> safe_pow, log -> safe_log, ...    */
enum {
  /* binary */
  SRHIP_OP_ADD = 1, SRHIP_OP_SUB = 2, SRHIP_OP_MUL = 3, SRHIP_OP_DIV = 4,
  SRHIP_OP_POW = 5,         /* safe_pow   src/Operators.jl:28-36 */
  SRHIP_OP_GREATER = 6,     /* greater    src/Operators.jl:82-84 */
  SRHIP_OP_COND = 7,        /* cond       src/Operators.jl:85-87 */
  SRHIP_OP_LOGICAL_OR = 8,  /* src/Operators.jl:91-93 */
  SRHIP_OP_LOGICAL_AND = 9, /* src/Operators.jl:94-96 */
  SRHIP_OP_MAX = 10, SRHIP_OP_MIN = 11, /* Julia Base max/min (NaN-propagating) */
  SRHIP_OP_MOD = 12,        /* Julia Base mod (floored, sign of divisor) */
  SRHIP_OP_ATAN2 = 13,      /* Julia Base atan(y, x) */
  /* unary */
  SRHIP_OP_NEG = 32, SRHIP_OP_SQUARE = 33, SRHIP_OP_CUBE = 34, SRHIP_OP_ABS = 35,
  SRHIP_OP_RELU = 36,       /* src/Operators.jl:88-90 (Bool strong zero) */
  SRHIP_OP_COS = 37, SRHIP_OP_SIN = 38, SRHIP_OP_TAN = 39, SRHIP_OP_EXP = 40,
  SRHIP_OP_LOG = 41,        /* safe_log   src/Operators.jl:37-40 */
  SRHIP_OP_LOG2 = 42, SRHIP_OP_LOG10 = 43, SRHIP_OP_LOG1P = 44,
  SRHIP_OP_SQRT = 45,       /* safe_sqrt  src/Operators.jl:57-60 */
  SRHIP_OP_ACOSH = 46,      /* safe_acosh src/Operators.jl:53-56 */
  SRHIP_OP_ATANH_CLIP = 47, /* atanh_clip src/Operators.jl:17   */
  SRHIP_OP_SINH = 48, SRHIP_OP_COSH = 49, SRHIP_OP_TANH = 50,
  SRHIP_OP_ASIN = 51, SRHIP_OP_ACOS = 52, SRHIP_OP_ATAN = 53, SRHIP_OP_ASINH = 54,
  SRHIP_OP_ERF = 55, SRHIP_OP_ERFC = 56,
  SRHIP_OP_GAMMA = 57,      /* gamma (Inf -> NaN) src/Operators.jl:11-15 */
  SRHIP_OP_ROUND = 58, SRHIP_OP_FLOOR = 59, SRHIP_OP_CEIL = 60, SRHIP_OP_SIGN = 61,
  SRHIP_OP_EXP2 = 62, SRHIP_OP_EXPM1 = 63, SRHIP_OP_CBRT = 64
};

/* ---- loss kinds (LossFunctions.jl 0.10/0.11 supervised losses; src/LossFunctions.jl:13-33,
 * the list src/Options.jl:209-229 documents).  Distance losses take r = output - target, margin
 * losses the agreement a = target * output (LossFunctions' MarginLoss convention). */
enum {
  SRHIP_LOSS_L2 = 0,          /* L2DistLoss (default, src/Options.jl:534-535) */
  SRHIP_LOSS_L1 = 1,          /* L1DistLoss */
  SRHIP_LOSS_LP = 2,          /* LPDistLoss{P}: p0 = P */
  SRHIP_LOSS_HUBER = 3,       /* HuberLoss(d): p0 = d */
  SRHIP_LOSS_L1_EPS_INS = 4,  /* L1EpsilonInsLoss(eps): p0 = eps */
  SRHIP_LOSS_L2_EPS_INS = 5,  /* L2EpsilonInsLoss(eps): p0 = eps */
  SRHIP_LOSS_LOGIT_DIST = 6,  /* LogitDistLoss */
  SRHIP_LOSS_PERIODIC = 7,    /* PeriodicLoss(c): p0 = c */
  SRHIP_LOSS_QUANTILE = 8,    /* QuantileLoss(tau): p0 = tau */
  SRHIP_LOSS_ZERO_ONE = 9,            /* ZeroOneLoss */
  SRHIP_LOSS_PERCEPTRON = 10,         /* PerceptronLoss */
  SRHIP_LOSS_LOGIT_MARGIN = 11,       /* LogitMarginLoss */
  SRHIP_LOSS_L1_HINGE = 12,           /* L1HingeLoss (= HingeLoss) */
  SRHIP_LOSS_L2_HINGE = 13,           /* L2HingeLoss */
  SRHIP_LOSS_SMOOTHED_L1_HINGE = 14,  /* SmoothedL1HingeLoss(gamma): p0 = gamma */
  SRHIP_LOSS_MODIFIED_HUBER = 15,     /* ModifiedHuberLoss */
  SRHIP_LOSS_L2_MARGIN = 16,          /* L2MarginLoss */
  SRHIP_LOSS_EXP = 17,                /* ExpLoss */
  SRHIP_LOSS_SIGMOID = 18,            /* SigmoidLoss */
  SRHIP_LOSS_DWD_MARGIN = 19          /* DWDMarginLoss(q): p0 = q */
};

/* One Node{T} (DynamicExpressions v0.16 fields: degree, constant, val, feature, op, l, r;
 * used in the reference at src/Complexity.jl:36-42, src/MutationFunctions.jl:39,52-57).
 * A tree is a contiguous run of nodes; node 0 of the run is the root; l/r index into the run. */
typedef struct srhip_node {
  uint8_t degree;   /* 0 = leaf, 1 = unary, 2 = binary */
  uint8_t constant; /* leaf only: 1 = constant (val), 0 = feature */
  uint16_t op;      /* 1-based index into the binary (degree 2) or unary (degree 1) op list */
  uint16_t feature; /* 1-based feature index (feature leaf) */
  uint16_t pad;
  int32_t l, r;     /* child indices within the tree's node run (-1 = none) */
  double val;       /* constant value; converted to T (exact for F32/I32 values of that type) */
} srhip_node;

typedef struct srhip_operators {
  int32_t nbin, nuna;
  const int32_t* binops; /* [nbin] SRHIP_OP_* code of options.operators.binops[i] */
  const int32_t* unaops; /* [nuna] */
} srhip_operators;

typedef struct srhip_loss {
  int32_t kind; /* SRHIP_LOSS_* */
  int32_t pad;
  double p0, p1;
} srhip_loss;

typedef struct srhip_ctx srhip_ctx;
typedef struct srhip_dataset srhip_dataset;
typedef struct srhip_program srhip_program;

/* thread-local description of the last nonzero status on this thread */
const char* srhip_last_error(void);
/* version string, e.g. "srhip 0.1.0 gfx950" */
const char* srhip_version(void);
/* number of visible HIP devices (0 if none / no driver); never fails */
int srhip_device_count(void);

/* A context owns one device, one stream and device scratch. Not thread-safe: use one
 * context per host thread (e.g. one per Julia task / per island), any number per device. */
int srhip_ctx_create(int device_ordinal, srhip_ctx** out);
void srhip_ctx_destroy(srhip_ctx* ctx);
int srhip_ctx_synchronize(srhip_ctx* ctx);

/* Dataset{T} upload.  Element (feature f, row j) is read from X[f*stride_feature + j*stride_row]
 * (Julia's features x rows column-major matrix: stride_feature = 1, stride_row = nfeatures;
 *  a C/NumPy (nfeatures, n) array: stride_feature = n, stride_row = 1).
 * y may be NULL (prediction-only dataset); weights may be NULL (unweighted).
 * The library copies everything before returning: no host pointer is retained. */
int srhip_dataset_create(srhip_ctx* ctx, int dtype, const void* X, int64_t nfeatures, int64_t n,
                         int64_t stride_feature, int64_t stride_row, const void* y,
                         const void* weights, srhip_dataset** out);
void srhip_dataset_destroy(srhip_dataset* ds);

/* Compile + upload a batch of trees (the population) for one operator table.  ctx may be NULL:
 * a host-only program (compiled, with its did_succeed metadata) usable by srhip_*_finalize and
 * srhip_program_* queries but not by the evaluation calls. */
int srhip_program_create(srhip_ctx* ctx, int dtype, const srhip_node* nodes,
                         const int64_t* tree_offsets /* [ntrees+1] into nodes */, int32_t ntrees,
                         const srhip_operators* ops, srhip_program** out);
void srhip_program_destroy(srhip_program* prog);
/* Number of constant leaves of each tree (DynamicExpressions count_constants order). */
int srhip_program_num_constants(const srhip_program* prog, int32_t* out_nconst /*[ntrees]*/);
/* Replace constant leaves (depth-first, left-to-right = get_constants order), all trees:
 * consts holds sum(nconst) values, tree-major. Re-folds and re-uploads. */
int srhip_program_set_constants(srhip_program* prog, const double* consts);
/* Read the constants back (same layout), e.g. after srhip_optimize_constants. */
int srhip_program_get_constants(const srhip_program* prog, double* consts);

/* Fused evaluate + loss for every tree of prog on ds (rows = all, or idx[0..nidx) 0-based).
 * out_loss[t] = loss in double (L(Inf) = +Inf when !ok), out_ok[t] = did_succeed. */
int srhip_eval_loss(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog,
                    const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                    double* out_loss, uint8_t* out_ok);

/* srhip_eval_loss in two halves, for callers that keep the device busy across populations (the
 * reference scores populations from concurrent tasks: Threads.@spawn per population,
 * src/SearchUtils.jl:121-122, @threads_if in src/SingleIteration.jl:112).  _submit queues the
 * evaluation's launches on the context's stream -- behind any evaluation still in flight there -- and
 * returns a ticket at once; _wait blocks until that evaluation has completed, takes its did_succeed
 * decisions and writes out_loss / out_ok exactly as srhip_eval_loss would (same bits), then frees the
 * ticket.  At most 3 tickets per context may be outstanding; tickets may be waited in any order, on
 * the thread that uses the context.  The program and dataset must outlive the ticket.  A row subset
 * (idx != NULL) is evaluated inside _submit (its gather synchronises the stream). */
typedef struct srhip_eval_ticket srhip_eval_ticket;
int srhip_eval_loss_submit(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog,
                           const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                           srhip_eval_ticket** out_ticket);
int srhip_eval_loss_wait(srhip_eval_ticket* ticket, double* out_loss, uint8_t* out_ok);

/* eval_tree_array for every tree: out_pred is T[ntrees][m] (m = n or nidx), row-contiguous. */
int srhip_eval_predict(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog,
                       const int64_t* idx, int64_t nidx, void* out_pred, uint8_t* out_ok);

/* Convenience: program_create + eval_loss + program_destroy. */
int srhip_eval_loss_batch(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_node* nodes,
                          const int64_t* tree_offsets, int32_t ntrees, const srhip_operators* ops,
                          const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                          double* out_loss, uint8_t* out_ok);

/* ---- row-sharded evaluation (several GPUs / processes, each holding a block of rows) -------
 * Replaces nothing in the reference (it has no row parallelism): the reduction
 * of src/LossFunctions.jl:13-33 and the did_succeed checks split into per-shard partials that
 * combine by an all-reduce, then a decision every rank computes identically.
 *   1. srhip_eval_loss_partials on each shard:
 *        sums[2*T + 2*F + 1] (T trees, F features): per tree {sum of (w*)loss, sum of w (or rows)},
 *        per feature {column sum (Float64 data: sum of x * 2^-64), non-finite count}, rows;
 *        chk[T]: operator-output check statistic.
 *   2. all-reduce: sums by SUM; chk by srhip_chk_reduce_op(dtype) (0 = MAX, 1 = SUM).
 *   3. srhip_partials_finalize(prog, F, sums, chk, loss, ok, status): status 2 = undecided
 *      (a near-overflow sum): then 4.
 *   4. srhip_eval_precise_partials for the undecided trees on each shard -> opsums
 *      [n_sel * srhip_program_max_ops(prog)], all-reduce SUM, srhip_precise_finalize -> ok.
 * srhip_eval_loss runs exactly these steps on one device. */
int srhip_eval_loss_partials(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog,
                             const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                             double* sums, double* chk);
int srhip_partials_finalize(const srhip_program* prog, int64_t nfeatures, const double* sums,
                            const double* chk, double* out_loss, uint8_t* out_ok,
                            uint8_t* out_status);
int srhip_eval_precise_partials(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog,
                                const int64_t* idx, int64_t nidx, const int32_t* trees,
                                int32_t ntrees_sel, double* opsums);
int srhip_precise_finalize(const srhip_program* prog, const int32_t* trees, int32_t ntrees_sel,
                           const double* opsums, uint8_t* out_ok);
int srhip_chk_reduce_op(int dtype);
int32_t srhip_program_max_ops(const srhip_program* prog);

/* ---- multi-GPU exchanges on RCCL (csrc/srhip_comm.cpp; one process per GPU) ------------------
 * Replace the reference's head-node copies between worker processes (Distributed over TCP,
 * src/SearchUtils.jl:108-127): migration (src/Migration.jl:16-38, applied at
 * src/SymbolicRegression.jl:933-943) becomes one all-gather of hall-of-fame / best_sub_pop node
 * tables over xGMI, and row shards combine their partials with one all-reduce.
 * Setup: rank 0 calls srhip_comm_unique_id and broadcasts the SRHIP_COMM_ID_BYTES bytes with the
 * job's launcher; every rank then calls srhip_comm_create with its context (collective: all ranks
 * must call it concurrently).  A communicator owns a HIP stream on its context's device; one
 * exchange at a time (srhip_comm_migrate_start ... srhip_comm_migrate_wait). */
typedef struct srhip_comm srhip_comm;
enum { SRHIP_COMM_ID_BYTES = 128 };
enum { SRHIP_REDUCE_SUM = 0, SRHIP_REDUCE_MAX = 1 };
int srhip_comm_unique_id(uint8_t* out_id /* [SRHIP_COMM_ID_BYTES] */);
int srhip_comm_create(srhip_ctx* ctx, const uint8_t* id, int32_t nranks, int32_t rank, srhip_comm** out);
void srhip_comm_destroy(srhip_comm* comm);
int srhip_comm_size(const srhip_comm* comm, int32_t* nranks, int32_t* rank);
/* Host wall time of the communicator's exchanges (issue -> completion seen; a migration counts from
 * srhip_comm_migrate_start to its _wait): the last one, the total, and how many (any may be NULL). */
int srhip_comm_stats(const srhip_comm* comm, double* ms_last, double* ms_total, int64_t* calls);
/* In-place all-reduce of a float64 vector: on device memory in place, no host staging; a host vector is
 * staged through the communicator's device buffer.  Device memory: the collective runs on the
 * communicator's own stream and is NOT ordered after other streams, so whatever produced buf must be
 * complete when this is called (synchronise the producing stream or event first); the call returns
 * after the collective has completed.  Every exchange waits at most SRHIP_COMM_TIMEOUT_S seconds
 * (default 300) -- past that, or on an asynchronous RCCL error, the communicator is aborted and this
 * and every later call on it fail. */
int srhip_comm_allreduce_f64(srhip_comm* comm, double* buf, int64_t n, int32_t op);
/* Fixed-size all-gather: recv[r * bytes .. (r + 1) * bytes) = rank r's send.  Both device pointers: no
 * staging, and (as for srhip_comm_allreduce_f64) send must be complete before the call; otherwise both
 * are staged through pinned host memory. */
int srhip_comm_allgather(srhip_comm* comm, const void* send, int64_t bytes, void* recv);
/* Migration: this rank's k best trees of (nodes, offsets[ntrees+1], losses[ntrees]) -- by loss,
 * non-finite last, ties by index; trees longer than max_nodes skipped -- packed into one fixed-size
 * payload and all-gathered (issued on the communicator's stream; returns at once).  _wait collects it:
 * out_counts[nranks] trees per rank, out_offsets[nranks][k+1] node offsets within each rank's
 * out_nodes[nranks][k * max_nodes] records, out_losses[nranks][k] (any output may be NULL). */
int srhip_comm_migrate_start(srhip_comm* comm, const srhip_node* nodes, const int64_t* offsets,
                             int32_t ntrees, const double* losses, int32_t k, int32_t max_nodes);
int srhip_comm_migrate_wait(srhip_comm* comm, int32_t* out_counts, int64_t* out_offsets,
                            double* out_losses, srhip_node* out_nodes);
/* Row-sharded eval_loss: ds holds THIS rank's rows (every rank the same features); runs steps 1-4
 * above with the all-reduces on RCCL -- the per-tree partials are written by the reduction straight
 * into the communicator's device buffer and all-reduced there (one group: loss sums, check statistics,
 * the shard's weight / feature / row totals), then copied to the host once; out_loss / out_ok
 * identical on every rank.  With one rank it equals srhip_eval_loss bit for bit. */
int srhip_eval_loss_sharded(srhip_ctx* ctx, srhip_comm* comm, const srhip_dataset* ds,
                            const srhip_program* prog, const srhip_loss* loss, const int64_t* idx,
                            int64_t nidx, double* out_loss, uint8_t* out_ok);

/* ---- constant optimisation (src/ConstantOptimization.jl) ------------------------------------ */
/* Loss and its exact gradient with respect to every tree's constants (forward-mode dual numbers
 * on the device), for every tree of prog: out_loss[T] (+Inf where did_succeed fails; as eval_loss,
 * also +Inf for a succeeding tree whose loss overflows), out_grad[sum nconst] in get_constants order
 * per tree (srhip_program_num_constants), out_ok[T] = did_succeed (srhip_eval_loss's decision).
 * Replaces the finite-difference gradient Optim derives from f(t) = eval_loss(t, dataset,
 * options; regularization=false) (src/ConstantOptimization.jl:48-50); the counterpart of
 * eval_grad_tree_array(tree, X, options; variable=false) (src/InterfaceDynamicExpressions.jl:118-124)
 * reduced through the loss. */
int srhip_eval_loss_grad(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* prog,
                         const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                         double* out_loss, double* out_grad, uint8_t* out_ok);

/* Per-row derivatives: eval_grad_tree_array(tree, X, options; variable) and eval_diff_tree_array(tree, X,
 * options, direction) (src/InterfaceDynamicExpressions.jl:90-95,118-124; DynamicExpressions v0.16,
 * external) for every tree of prog, forward-mode dual numbers on the device.
 *   wrt = SRHIP_WRT_CONSTANTS: d out / d c for each constant (get_constants order), nconst_t rows per tree
 *   wrt = SRHIP_WRT_FEATURES, direction = 0: d out / d x_f for every feature, nfeatures rows per tree
 *   wrt = SRHIP_WRT_FEATURES, direction = d >= 1: d out / d x_d only, 1 row per tree
 * out_pred: T[ntrees][m] (the evaluator's predictions, as srhip_eval_predict); out_grad: T[sum of rows][m],
 * tree-major, m = n or nidx; out_ok[t] = did_succeed of the evaluation && every derivative finite. */
enum { SRHIP_WRT_CONSTANTS = 0, SRHIP_WRT_FEATURES = 1 };
int srhip_eval_grad_predict(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* prog, int32_t wrt,
                            int32_t direction, const int64_t* idx, int64_t nidx, void* out_pred, void* out_grad,
                            uint8_t* out_ok);

typedef struct srhip_optim_options {
  int32_t iterations;  /* BFGS iterations per start (Optim.Options(iterations=8), src/Options.jl:693) */
  int32_t nrestarts;   /* perturbed restarts c * (1 + randn/2) (optimizer_nrestarts=2, src/Options.jl:432) */
  uint64_t seed;       /* RNG seed of the restart perturbations */
  double g_tol;        /* gradient infinity-norm tolerance (Optim default 1e-8; <= 0 -> 1e-8) */
} srhip_optim_options;

/* optimize_constants for every tree of prog at once (src/ConstantOptimization.jl:11-81): per tree
 * Newton (one constant) or BFGS (several), each with the BackTracking line search, from the current
 * constants and nrestarts perturbed starts; a tree's constants are replaced (in prog) only where the
 * best minimum beats its baseline loss.  out_loss[T]: the loss of the returned trees (eval_loss,
 * regularization=false); out_improved[T]; out_fcalls[T] (nullable): the reference's num_evals per
 * tree -- objective calls of all starts (result.f_calls) + 1 if improved (the re-score), 0 for a tree
 * without constants or with a static did_succeed failure (left unchanged). */
int srhip_optimize_constants(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* prog,
                             const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                             const srhip_optim_options* opt, double* out_loss,
                             uint8_t* out_improved, int64_t* out_fcalls);
/* The same, with the restarts' starting points exchanged with the caller
 * (src/ConstantOptimization.jl:53-68: tmptree = copy(tree); val *= T(1) + T(1//2) * randn(T)):
 *   starts_in  (nullable): [nrestarts][sum nconst] restart points in get_constants order, tree-major,
 *              used instead of the library's own draws (a Float32 program rounds them to Float32);
 *   starts_out (nullable): [nrestarts][sum nconst] the restart points actually used.
 * The library's own draws perturb in the program's type: Float32 programs draw a Float32 normal
 * and compute val * (1f + 0.5f * r) in Float32.  Start 0 is always the tree's current constants;
 * its result is kept unless a restart's minimum is strictly smaller (:65-67), and the kept result
 * replaces the constants only if it beats the baseline (:70-78).  Trees without constants or
 * failing statically report their current constants. */
int srhip_optimize_constants_starts(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* prog,
                                    const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                                    const srhip_optim_options* opt, const double* starts_in,
                                    double* starts_out, double* out_loss, uint8_t* out_improved,
                                    int64_t* out_fcalls);

/* ---- measurement hooks (bench / profiling) --------------------------------------------- */
/* Device time (ms) of the last main kernel on this context -- the interpreter of srhip_eval_loss /
 * srhip_eval_predict, or the dual-number kernel of srhip_eval_loss_grad -- measured with HIP events
 * recorded on the context's stream; < 0 if unavailable (also after srhip_optimize_constants*, whose
 * many small gradient launches go without events). */
double srhip_last_kernel_ms(const srhip_ctx* ctx);
/* Work of the last srhip_eval_loss / srhip_eval_loss_partials / srhip_eval_predict on this context,
 * counted on the device (the rows each tree was actually evaluated on: a tree that failed -- the
 * reference's early return -- stops at the failing tile): out[0] evaluated node-rows (count_nodes x
 * rows), out[1] nominal node-rows (every live tree on every row), out[2] evaluated operator-node
 * rows, out[3] evaluated tree-rows. */
int srhip_last_work(const srhip_ctx* ctx, int64_t out[4]);
/* Per-program work counters: sum over trees of count_nodes / operator nodes. */
int srhip_program_stats(const srhip_program* prog, int64_t* total_nodes, int64_t* total_opnodes,
                        int32_t* max_stack);
/* Derived columns of a program (heavy unary operators on feature leaves computed once per
 * workgroup and shared by every tree): count, and if spec is non-null the first
 * min(count, cap) entries as (device unary op << 16) | (feature - 1).  Set SRHIP_NO_DERIVE=1
 * before srhip_program_create to compile without them. */
int srhip_program_derived(const srhip_program* prog, int32_t* count, uint32_t* spec, int32_t cap);
/* Process-wide counters of the per-tree code cache used by srhip_program_create (any argument may be
 * NULL): trees served from the cache, trees compiled, entries made (a tree gets an entry on its
 * second sighting; SRHIP_CODE_CACHE_EAGER=1: on its first). */
int srhip_code_cache_stats(int64_t* hits, int64_t* misses, int64_t* inserts);

/* ---- Cross-population request coalescer (8(b) "Threading") ----------------
 * The reference scores one tree per mutation from every population task concurrently
 * (score_func in next_generation, src/Mutate.jl:268-274, under Threads.@spawn per population,
 * src/SymbolicRegression.jl:964-987 / src/SearchUtils.jl:121-122).  A batcher uses the caller's
 * context and device dataset; any number of threads submit single-tree score requests and block on
 * their ticket; worker threads (SRHIP_COALESCE_WORKERS, default 2: worker 0 on the caller's context,
 * the others on contexts of their own on the same device, so one compiles and launches while
 * another waits for its kernel) flush the queue as ONE program + ONE srhip_eval_loss launch
 * when max_batch requests are queued, when every registered client is waiting (nclients > 0), or
 * max_wait_us after the oldest request.  Requests with different row subsets (batching `idx`)
 * go to separate launches of the same flush.  Results are exactly those of srhip_eval_loss on
 * the single tree (the kernel's per-tree results do not depend on the batch).  Thread-safe; the
 * context must not be used by other callers while the batcher lives. */
typedef struct srhip_batcher srhip_batcher;
int srhip_batcher_create(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_operators* ops,
                         const srhip_loss* loss, int32_t max_batch, int32_t max_wait_us,
                         srhip_batcher** out);
/* expected number of concurrent clients (0 = unknown: flush on max_batch / max_wait_us only) */
int srhip_batcher_set_clients(srhip_batcher* b, int32_t nclients);
/* one tree (nodes[0] is its root); idx = optional 0-based row subset (copied) */
int srhip_batcher_submit(srhip_batcher* b, const srhip_node* nodes, int64_t nnodes,
                         const int64_t* idx, int64_t nidx, uint64_t* ticket);
/* blocks until the ticket's batch ran; returns that request's status (errors carry the message
 * of the failed compile / launch, readable with srhip_last_error on the waiting thread) */
int srhip_batcher_wait(srhip_batcher* b, uint64_t ticket, double* out_loss, uint8_t* out_ok);
/* submit + wait */
int srhip_batcher_eval(srhip_batcher* b, const srhip_node* nodes, int64_t nnodes,
                       const int64_t* idx, int64_t nidx, double* out_loss, uint8_t* out_ok);
/* requests served, device launches, largest batch */
int srhip_batcher_stats(const srhip_batcher* b, int64_t* nrequests, int64_t* nlaunches,
                        int64_t* max_batch_seen);
/* worker wall time spent inside flushes (compile + upload + launch + wait, ms, summed over the
 * workers) and the summed interpreter-kernel time of their launches (HIP events, ms): kernel_ms /
 * elapsed wall time is the device-busy fraction of a search (bench C1 / C3; concurrent launches of
 * two workers can overlap, so it is an upper bound) */
int srhip_batcher_timing(const srhip_batcher* b, double* busy_ms, double* kernel_ms);
/* drains the queue (pending requests are evaluated), joins the worker */
void srhip_batcher_destroy(srhip_batcher* b);

#ifdef __cplusplus
}
#endif
#endif /* SRHIP_H */
