// srhip_internal.h — library-internal declarations shared by the translation units of libsrhip.so
// (srhip_host.cpp: compiler, datasets, evaluation driver, C ABI; srhip_optim.cpp: constant
// gradients and the batched BFGS constant optimizer).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/srhip.h"
#include "srhip_isa.h"
#include "srhip_kernels.h"

namespace srhip {

// ---------------------------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------------------------
// sets the thread-local message returned by srhip_last_error(); returns code
int fail(int code, const char* fmt, ...);
const char* last_error();

// SRHIP_TRACE=1 in the environment prints every HIP call of the library (before and after) to
// stderr, flushed: a GPU hang then names the call it happened in.
inline bool trace_on() {
  static const int on = [] { const char* e = getenv("SRHIP_TRACE"); return e && *e && *e != '0'; }();
  return on != 0;
}
inline int debug_stop() {
  static const int v = [] { const char* e = getenv("SRHIP_DEBUG_STOP"); return e ? atoi(e) : 0; }();
  return v;
}
// SRHIP_NO_EARLY_EXIT=1: interpreter waves evaluate every row of a failed tree (read per launch, so
// a test can compare both settings in one process)
inline bool early_exit_on() {
  const char* e = getenv("SRHIP_NO_EARLY_EXIT");
  return !(e && *e && *e != '0');
}
#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    if (trace_on()) { fprintf(stderr, "[srhip] %s:%d %s\n", __FILE__, __LINE__, #expr); fflush(stderr); } \
    hipError_t e_ = (expr);                                                                       \
    if (trace_on()) { fprintf(stderr, "[srhip]   -> %d\n", (int)e_); fflush(stderr); }          \
    if (e_ != hipSuccess) return fail(SRHIP_ERR_DEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

inline size_t dtype_size(int dtype) { return dtype == SRHIP_F64 ? 8 : 4; }

// overflow thresholds of an exact sum rounded to T: 2^128 - 2^103 and 2^1024 - 2^970
// (computed once: an ldexpl call per use cost ~1 us per 25 trees in the host decisions)
inline long double ovf_threshold(int dtype) {
  static const long double f64 = ldexpl(1.0L, 1024) - ldexpl(1.0L, 970), f32 = ldexpl(1.0L, 128) - ldexpl(1.0L, 103);
  return dtype == SRHIP_F64 ? f64 : f32;
}

// ---------------------------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------------------------
// A regrown scratch buffer takes half again its old size at least (below 256 MB): per-population
// sizes (live trees, undecided lists) vary from call to call, and every regrowth frees the old
// buffer, which synchronises the device -- a pipelined population queued behind it stalls.
inline size_t grown_size(size_t n, size_t old) {
  const size_t g = old + old / 2;
  const size_t want = (old > 0 && g > n && g <= ((size_t)256 << 20)) ? g : n;
  return want < 256 ? 256 : want;
}
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    const size_t want = grown_size(n, bytes);
    release();
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
  }
};
// Program buffers come from a process-wide cache of device allocations, by power-of-two size class
// and device (srhip_host.cpp devpool_*): hipFree synchronises the whole device, so a host thread
// destroying the previous population's program would wait for whatever the device runs meanwhile
// (the fresh-population pipeline: compile on one thread while another evaluates).  Every use of a
// program's buffers is complete when the program is destroyed (evaluations and uploads are
// synchronous), so a returned block is reusable at once.
void* devpool_get(size_t bytes, size_t* cap);
void devpool_put(void* p, size_t cap, int device);
struct PoolBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int device = -1;
  ~PoolBuf() { release(); }
  void release() {
    if (p) devpool_put(p, bytes, device);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    release();
    size_t cap = 0;
    void* q = devpool_get(n, &cap);
    if (!q) return hipErrorOutOfMemory;
    if (hipGetDevice(&device) != hipSuccess) device = -1;
    p = q;
    bytes = cap;
    return hipSuccess;
  }
};
struct HostBuf {  // pinned staging
  void* p = nullptr;
  size_t bytes = 0;
  ~HostBuf() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t n, unsigned flags = hipHostMallocDefault) {
    if (n <= bytes && p) return hipSuccess;
    const size_t want = grown_size(n, bytes);
    release();
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) bytes = want;
    return e;
  }
};

// A tree's evaluation-time metadata in 32 contiguous bytes (built at compile from its TreeInfo): the
// per-call decisions and work counts read this array, not the TreeInfo vectors (heap data written by
// the compile threads, cold in the evaluating thread's caches: ~50 us per fresh 1024-tree population)
struct TreeDecide {
  double maxc = -1.0;          // max |c| of fill_consts (ignoring NaN), -1 without any
  uint64_t feat_mask = 0;      // feat_checks (features < 64)
  int32_t nnodes = 0, nops = 0;
  uint8_t static_fail = 0, has_op = 0, slow = 0;  // slow: a feature check >= 64 (decide from TreeInfo)
};
struct TreeInfo {
  bool static_fail = false;
  std::vector<double> fill_consts;  // |c| * m >= OVF  => fail
  std::vector<int> feat_checks;     // column checks (0-based features)
  std::vector<uint8_t> op_sumcheck; // per emitted operator node: 1 = isfinite(sum) check, 0 = elementwise only
  int32_t nconst = 0, nnodes = 0, nops = 0, need = 0;
  int32_t code_begin = 0, code_len = 0;
  double cost = 0.0;
  // Float32 evaluation programs: (cM, cF, c0) of the bound on every +/- output (EvalArgs::sbound)
  float sb[3] = {0.0f, 0.0f, 0.0f};
};



}  // namespace srhip

namespace srhip {
// Where an evaluation's per-tree records land: coherent pinned host buffers its reductions write into
// (loss sums, check statistics, rows evaluated, the device precise pass's output), the interpreter's
// timing events and a completion event.  Set 0 serves the synchronous calls; srhip_eval_loss_submit
// tickets take sets 1 .. RESULT_SETS - 1, so several evaluations can be in flight on one stream, each
// with records of its own.
struct ResultSet {
  HostBuf h_loss, h_chk, h_rows, h_pout;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
  bool busy = false;
};
constexpr int RESULT_SETS = 4;
}  // namespace srhip

// the opaque handles of include/srhip.h (global namespace, as declared there)
struct srhip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // the gradient kernels' timing (srhip_optim.cpp)
  // the events srhip_last_kernel_ms reads: ev0 / ev1 above, or the last completed evaluation's set's
  hipEvent_t last_ev0 = nullptr, last_ev1 = nullptr;
  srhip::ResultSet rs[srhip::RESULT_SETS];
  hipEvent_t ev_sync = nullptr;  // stream_wait's completion marker (no timing)
  // new programs' uploads (srhip_program_create).  One per context: a device-wide shared upload stream
  // (four streams for the three-context optimiser split instead of six) made C4 168 ms against 142 on
  // one box (round 6, profiles/r06_c4_upload_stream_ab.txt) -- with three evaluation streams on
  // hardware queues of their own the groups' kernels contend; with six, two of them share a queue
  hipStream_t up_stream = nullptr;
  bool timed = false;
  int num_cu = 256;
  int lds_max = 160 * 1024;  // hipDeviceAttributeMaxSharedMemoryPerBlock of the device
  srhip::DevBuf slab_loss, slab_chk, slab_prec, order_prec;
  srhip::DevBuf vX, vy, vw, vidx, vstats;  // gathered views (batching idx)
  srhip::DevBuf g_chunks, g_slab, g_red;   // constant-gradient launches
  srhip::DevBuf g_xd;                        // their derived view (features + derived columns)
  // what g_xd holds when built from a whole dataset (serial, ld, dtype, column base, spec): reused
  // by the next call over the same dataset and spec
  uint64_t g_xd_serial = 0;
  int64_t g_xd_ld = 0;
  int g_xd_dtype = -1, g_xd_base = -1;
  std::vector<uint32_t> g_xd_spec;
  srhip::HostBuf h_gchunks[2], h_gred[2];   // their pinned staging, per pass (gradient, value-only)
  srhip::HostBuf h_gpatch, h_gspec;         // pinned staging of patched / speculative gradient code
  srhip::HostBuf h_stats, h_prec, h_plist, h_dbg;
  srhip::DevBuf fail_flag;  // [order slots] int32: launch epoch in which the tree was seen to fail
  int32_t epoch = 0;        // interpreter launches so far (MODE_LOSS with early exit)
  // persistent launches: the row-block counter (one int32).  Zeroed once; every launch that drains its
  // claims leaves it at zero (the last claim stores 0).  block_ctr_dirty: a launch was issued and not
  // yet seen to drain (error return in between, or lost blocks) -- the next launch zeroes it first
  srhip::DevBuf block_ctr;
  bool block_ctr_dirty = false;
  srhip::DevBuf slab_rows;  // [row block][order slot] valid rows evaluated
  srhip::DevBuf d_ulist;    // the device's undecided-tree list ([0] = count; reset by its consumer)
  // work of the last srhip_eval_loss / srhip_eval_predict on this context (srhip_last_work):
  // evaluated node-rows, nominal node-rows (every live tree on every row), evaluated operator-node
  // rows, evaluated tree-rows
  int64_t work[4] = {0, 0, 0, 0};
  // a second context on the same device (own stream and buffers), created on first use by the
  // constant optimiser, which runs half of the population on it from a second host thread
  std::vector<srhip_ctx*> aux;
  std::mutex aux_mu;
};

struct srhip_dataset {
  srhip_ctx* ctx = nullptr;
  int device = 0;  // own copy: a dataset may be destroyed after its context
  int dtype = SRHIP_F32;
  int64_t nfeat = 0, n = 0, ld = 0;
  bool has_y = false, weighted = false;
  double sum_w = 0.0;
  srhip::DevBuf X, y, w, stats;
  std::vector<srhip::FeatStat> hstats;  // feature stats over all n rows
  uint64_t serial = 0;                   // process-unique (caches keyed by dataset identity)
};

struct srhip_program {
  srhip_ctx* ctx = nullptr;
  int device = -1;  // own copy (-1: host-only program)
  int dtype = SRHIP_F32;
  int32_t ntrees = 0;
  std::vector<srhip_node> nodes;
  std::vector<int64_t> offsets;
  std::vector<int32_t> binops, unaops;
  std::vector<srhip::TreeInfo> info;
  std::vector<srhip::TreeDecide> dec;  // [ntrees], from info (compile_program)
  std::vector<srhip::Ins> code;
  std::vector<int32_t> prog_off;
  int32_t kmax = 0, max_ops = 0, max_len = 0;
  int64_t total_nodes = 0, total_ops = 0;
  int32_t maxfeat = 0;  // largest feature index any tree reads (the columns a launch stages)
  // device copy of the evaluation program, one buffer and one upload (upload_program):
  // [code | prog_off | dcode | dprog_off | dspec | dmask | sbound], 16-byte aligned sections
  // upload_program(P, sync, defer = true) only builds the image: the next evaluation appends its tree
  // order and uploads both with one copy (the coalescer's per-flush program)
  mutable srhip::PoolBuf d_prog;
  mutable std::vector<uint8_t> blob;  // its host image (alive until the next upload)
  mutable bool upload_pending = false;
  mutable int32_t und_hint = 0;  // trees the last device-listed precise pass saw (list capacity hint)
  mutable size_t blob_off[7] = {0, 0, 0, 0, 0, 0, 0};  // section offsets: off, dcode, doff, dspec, dmask, sbound, end
  mutable const srhip::Ins* code_dev = nullptr;
  mutable const int32_t* off_dev = nullptr;
  // derived-column program (srhip_isa.h): the same trees with U(X[f]) leaves reading LDS columns;
  // used by loss / prediction launches whose staging fits LDS, the plain program otherwise
  std::vector<uint32_t> dspec;  // [nd] (U << 16) | (feature - 1)
  std::vector<uint64_t> dmask;  // [ntrees]
  std::vector<srhip::Ins> dcode;
  std::vector<int32_t> dprog_off;
  std::vector<double> dcost;
  int32_t dkmax = 0, dmax_len = 0;
  mutable const srhip::Ins* dcode_dev = nullptr;
  mutable const int32_t* doff_dev = nullptr;
  mutable const uint32_t* dspec_dev = nullptr;
  mutable const uint64_t* dmask_dev = nullptr;
  // Float32 programs: [ntrees][4] (cM, cF, c0, 0) per tree (TreeInfo::sb; EvalArgs::sbound)
  std::vector<float> sbound;
  mutable const float* sbound_dev = nullptr;
  // launch schedule cache: the cost-sorted tree order of the last plan (groups, tpg, derived),
  // resident on the device; a program evaluated again with the same plan skips the sort and upload
  mutable std::mutex ord_mu;
  mutable int ord_key[3] = {-1, -1, -1};
  mutable std::vector<int32_t> ord_goff;  // group offsets of that plan (appended to d_order)
  mutable std::vector<int32_t> ord_host;  // the uploaded order (kept alive: its copy is asynchronous)
  mutable const void* ord_dev = nullptr;  // where it lives on the device (d_order, or inside d_prog)
  mutable srhip::PoolBuf d_order;
  // gradient program (constants not folded, constant leaves carry their get_constants index);
  // compiled on first use by the constant-gradient path
  bool grad_ready = false;
  // derived columns of the gradient program (constant-gradient launches only): gdspec[j] = u << 16 |
  // feature column, read as column gdbase + j of a derived view; g_derived: the compiled gradient
  // program reads them (compiled so when g_want_derived and gdspec is not empty)
  std::vector<uint32_t> gdspec;
  int32_t gdbase = 0;
  bool gdspec_done = false, g_want_derived = false, g_derived = false;
  std::vector<srhip::Ins> gcode;
  std::vector<int32_t> gprog_off;
  std::vector<srhip::TreeInfo> ginfo;  // did_succeed metadata for the gradient program's constants
  int32_t gkmax = 0, gmax_len = 0, gmax_ops = 0;
  srhip::PoolBuf d_gcode, d_goff;
  // constant-leaf values (node storage order) the gradient program was last compiled with: when only
  // constants change (the optimiser's line search), just the trees whose constants moved recompile
  std::vector<double> gsnap;
  std::vector<int64_t> gsnap_off;  // [ntrees] first snapshot entry of each tree
  // trees whose constants were written since the last gradient compile/patch (set by the optimiser);
  // empty = unknown, scan every tree.  Cleared by every full (re)compile.
  std::vector<int32_t> ghint;
  // Speculative slots of the gradient program (the optimiser's line searches): gspec_alloc copies of
  // "a tree at other constants" after the trees' own code, gspec_stride instructions each, slot s at
  // program index ntrees + s (gprog_off / ginfo).  For trees whose code shape does not depend on the
  // constant values (gspec_ok: every constant leaf is the immediate of exactly one instruction) a
  // slot -- and the in-place patch of the tree's own code -- is the full compile's code (gbase) with
  // the constant immediates rewritten (gci: per tree, (instruction offset, constant index) pairs) and
  // the value-dependent did_succeed metadata recomputed (TreeCompiler::static_info); other trees are
  // recompiled.  gspec_cap is the optimiser's request; a full compile allocates it.
  int32_t gspec_cap = 0, gspec_alloc = 0, gspec_stride = 0;
  int64_t gspec_base = 0;
  std::vector<int32_t> gci_off, gci;
  std::vector<uint8_t> gspec_ok;
  std::vector<srhip::TreeInfo> gbase;
};

namespace srhip {

// ---- evaluation views and launch planning (srhip_host.cpp) ----------------------------------
struct View {
  const void* X;
  const void* y;
  const void* w;
  int64_t ld, m;
  const FeatStat* stats;  // host
  double sum_w;
  // gradient launches over a derived view (X = [the program's feature columns | its derived columns],
  // srhip_optim.cpp derived_view): the feature columns staged per row block; -1: the dataset's
  int32_t nfeat_x = -1;
  int32_t nd_x = 0;  // its derived columns (then as many tangent-zero columns)
};
struct LaunchPlan {
  int rb_rows, nrb, groups, tpg;
  bool xlds;
  size_t lds;
};
int compile_program(srhip_program& P);       // eval program (+ invalidates the gradient program)
extern thread_local double g_patch_scan_s, g_patch_copy_s;  // optimiser timing split (SRHIP_OPTIM_TIMING), per thread
int compile_grad_program(srhip_program& P);  // gradient program, uploaded
void grad_derived_spec(srhip_program& P);     // P.gdspec / gdbase from the trees (once)
// Speculative slot `slot` := tree t at constants c[0 .. nconst) (get_constants order), host side;
// false if the tree cannot be instantiated.  *static_fail: did_succeed is false before any row is
// evaluated (a non-finite constant leaf or constant subtree; no evaluation needed).  [lo, hi) grows by the instructions written.
bool spec_instantiate(srhip_program& P, int32_t slot, int32_t t, const double* c, bool* static_fail, int64_t& lo,
                      int64_t& hi);
// sync = false: the copies stay queued on the context's stream (the caller's next evaluation, which
// synchronises before returning, must follow before P's host code changes again)
// stream: the copy's stream (nullptr: the context's; srhip_program_create uses the context's upload
// stream, so a program built on one host thread does not wait for evaluations queued on another)
int upload_program(srhip_program& P, bool sync = true, bool defer = false, hipStream_t stream = nullptr);
int make_view(srhip_ctx* ctx, const srhip_dataset* ds, const int64_t* idx, int64_t nidx, bool need_y, View& v);
int gathered_weight_sum(srhip_ctx* ctx, const srhip_dataset* ds, int64_t nidx, View& v);
// ncols: feature (+ derived) columns staged; lds_budget: bytes of LDS a workgroup may use
LaunchPlan plan_launch(const srhip_ctx* ctx, int dtype, int64_t ncols, bool weighted, bool with_y, int64_t m,
                       int32_t ntrees, int rows_per_tile, size_t lds_budget = 64 * 1024 - 64, int waves = EVAL_WAVES);
// did_succeed decision of tree t from partials in the srhip_eval_loss_partials layout:
// 0 ok, 1 fail, 2 undecided (only the sums' feature / row-count entries are read)
int decide_tree(const TreeInfo& I, const srhip_program& P, int64_t nfeat, const double* sums, double chk);
// the context's failed-tree marks for one early-exit launch over n trees / chunks: a fresh epoch
// (> 0) that no stale mark can equal; the marks are zeroed on the stream when (re)allocated
int next_fail_epoch(srhip_ctx* ctx, int64_t n, int32_t** flags, int32_t* epoch);
int check_eval_args(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode, const srhip_loss* loss);
int run_eval(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode, const srhip_loss* loss,
             const int64_t* idx, int64_t nidx, double* out_loss, void* out_pred, uint8_t* out_ok);
// The precise did_succeed pass for undecided trees (exact per-operator-node sums over the view), on the
// evaluation program or (grad = true) on the gradient program: out_ok[u] for trees[u].
int precise_decide(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const View& v,
                   const int32_t* trees, int32_t nu, bool grad, uint8_t* out_ok);

// Row-sharded evaluation with caller-supplied exchanges (srhip_comm.cpp: RCCL).  The per-tree partials
// stay in device memory: the evaluation's reduction kernel writes them into the exchange's own device
// buffer, laid out [loss | chk | aux] (ShardLayout), which is all-reduced in place and copied to the
// host once.  Every callback returns an SRHIP status.
struct ShardLayout {
  int dtype = 0;
  size_t nt = 0, naux = 0;
  size_t loss_bytes() const { return nt * 8; }  // f64 sums (Int32 data: int64 sums), SUM
  size_t chk_size() const { return dtype == SRHIP_F64 ? 8 : (dtype == SRHIP_F32 ? 4 : 0); }  // f32 MAX / f64 SUM
  size_t chk_off() const { return loss_bytes(); }
  size_t aux_off() const { return (chk_off() + nt * chk_size() + 7) & ~(size_t)7; }  // f64, SUM
  size_t bytes() const { return aux_off() + naux * 8; }
};
struct ShardIO {
  // the device buffer (>= bytes) the reduction writes [loss | chk] into
  std::function<int(size_t bytes, void** dptr)> buffer;
  // after the evaluation completed: aux (host) copied behind [loss | chk], the three segments all-reduced
  // in place as one group, the whole buffer copied into host memory; *out points at that copy
  std::function<int(const ShardLayout& L, const double* aux, const void** out)> reduce;
  // plain f64 SUM of a host array in place (the precise pass's per-operator sums of undecided trees)
  std::function<int(double* buf, size_t n)> reduce_host;
};
// getenv through a per-thread cache that is dropped whenever the environment changes (srhip_host.cpp)
const char* env_get(const char* name);
// Wait for the context's stream: hipStreamSynchronize, or with SRHIP_SYNC_SPIN=1 a spin on a
// completion event.  The spin measured the same C2 step time and slowed a host thread compiling the
// next population beside the evaluation (fresh compile 0.59 -> 0.80 ms, pipelined population
// 1.63 -> 1.95 ms), so blocking is the default.
int stream_wait(srhip_ctx* ctx);
int run_eval_sharded(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const srhip_loss* loss,
                     const int64_t* idx, int64_t nidx, const ShardIO& io, double* out_loss, uint8_t* out_ok);

}  // namespace srhip
