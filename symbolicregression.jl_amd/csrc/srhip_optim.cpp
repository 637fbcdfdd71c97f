// srhip_optim.cpp — constant gradients and the batched constant optimizer of libsrhip.so.
//
// srhip_eval_loss_grad: loss + exact d loss / d constants for every tree of a program (one launch of
//   the dual-number kernel, srhip_grad.hip, over (tree, constant-chunk) pairs).
// srhip_optimize_constants: optimize_constants / _optimize_constants (src/ConstantOptimization.jl:
//   11-81) for a whole population at once.  dispatch_optimize_constants (:22-41) picks the method
//   per tree: no constants -> untouched; one constant -> Optim.Newton(linesearch=BackTracking());
//   otherwise options.optimizer_algorithm = BFGS(linesearch=BackTracking()) (src/Options.jl:429-431).
//   LineSearches' BackTracking: order 3, c1 = 1e-4, rho in [0.1, 0.5]; `iterations` iterations per
//   start (Optim.Options(iterations = 8), src/Options.jl:691-705) from the current constants and from
//   `nrestarts` perturbed starts x0 .* (1 + randn/2); a tree's constants are replaced only if the best
//   minimum beats its baseline loss (:70-78).  Every tree runs its own state machine and each kernel
//   launch evaluates the one point every still-active tree needs next (bfgs_pipelined).
//   Differences from the reference, by design: exact (dual-number) gradients instead of Optim's
//   finite differences, and Newton's Hessian as a central difference of those exact gradients instead
//   of a second difference of losses -- parity is on the optimised loss, SURVEY.md 8(a) A13.
#include <algorithm>
#include <numeric>
#include <chrono>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "srhip_grad.h"
#include "srhip_internal.h"

using namespace srhip;

namespace {

// Launch geometry of the dual-number kernel: row blocks of a fixed size (SRHIP_GRAD_RB, default 256
// rows = 4 tiles per wave, fewer for smaller datasets), independent of how many chunks a launch
// carries -- a tree's per-block partial sums, and so its loss and gradient bits, depend on the dataset
// alone -- and enough tree groups to fill the chip.  The optimiser's last rounds evaluate a handful
// of trees: small blocks keep those launches short (many workgroups, each a few tiles deep).
LaunchPlan grad_plan(const srhip_ctx* ctx, int64_t m, int32_t nchunks) {
  static const int rb_env = [] { const char* e = getenv("SRHIP_GRAD_RB"); return e ? atoi(e) : 0; }();
  int rb = (rb_env >= 256 && rb_env <= 4096 && (rb_env & (rb_env - 1)) == 0) ? rb_env : 256;
  m = std::max<int64_t>(1, m);
  while (rb > 256 && rb / 2 >= m) rb /= 2;  // >= 256: the value-only pass runs 4 rows per lane
  LaunchPlan L{};
  L.rb_rows = rb;
  L.nrb = (int)((m + rb - 1) / rb);
  L.xlds = false;
  L.lds = 0;
  const int target_blocks = 4 * ctx->num_cu;
  int g = (target_blocks + L.nrb - 1) / L.nrb;
  g = std::max(1, std::min(g, std::max(1, nchunks / (2 * GRAD_WAVES))));
  L.tpg = (std::max(1, nchunks) + g - 1) / g;
  L.groups = (std::max(1, nchunks) + L.tpg - 1) / L.tpg;
  return L;
}

// constant offsets (get_constants order) of every tree: coff[t] .. coff[t+1]
std::vector<int64_t> const_offsets(const srhip_program& P) {
  std::vector<int64_t> c(P.ntrees + 1, 0);
  for (int32_t t = 0; t < P.ntrees; ++t) c[t + 1] = c[t] + P.info[t].nconst;
  return c;
}

void get_consts_rec(const srhip_node* nd, int64_t i, std::vector<double>& out) {
  const srhip_node& n = nd[i];
  if (n.degree == 0) {
    if (n.constant) out.push_back(n.val);
    return;
  }
  get_consts_rec(nd, n.l, out);
  if (n.degree == 2) get_consts_rec(nd, n.r, out);
}
void set_consts_rec(srhip_node* nd, int64_t i, const double*& c) {
  srhip_node& n = nd[i];
  if (n.degree == 0) {
    if (n.constant) n.val = *c++;
    return;
  }
  set_consts_rec(nd, n.l, c);
  if (n.degree == 2) set_consts_rec(nd, n.r, c);
}
std::vector<double> get_all_consts(const srhip_program& P) {
  std::vector<double> out;
  for (int32_t t = 0; t < P.ntrees; ++t) get_consts_rec(P.nodes.data() + P.offsets[t], 0, out);
  return out;
}
void set_all_consts(srhip_program& P, const double* c) {
  for (int32_t t = 0; t < P.ntrees; ++t) set_consts_rec(P.nodes.data() + P.offsets[t], 0, c);
  P.grad_ready = false;
  P.ghint.clear();  // every tree may have changed
}

}  // namespace

// Loss and gradient for `trees` (f[t] = +Inf where did_succeed fails or is undecided); gradients
// land at g[coff[t] ..].  The gradient program must match the program's current constants.
// SRHIP_OPTIM_TIMING=1: host-side time split of the optimiser (compile/patch vs the rest), stderr
static thread_local double g_t_compile = 0.0, g_t_eval = 0.0, g_t_host = 0.0;
static thread_local int64_t g_n_launch = 0;
static thread_local bool g_stats_on = false;
static thread_local bool g_launch_log = false;  // SRHIP_OPTIM_TIMING=3: one stderr line per launch (caller's group)
static thread_local int64_t g_hist[5] = {0, 0, 0, 0, 0}, g_nonfinite_trials = 0;
static thread_local int64_t g_spec_launched = 0, g_spec_used = 0;  // speculative trial points
// (SRHIP_OPTIM_TIMING=2) evaluated items by pass (0 gradient, 1 value-only) and launch size (items
// <= 64 / > 64): [pass][big][all, non-finite f]
static thread_local int64_t g_items[2][2][2] = {};
// integer knob through the environment cache (read per call: tests flip it within one process)
static int env_int_opt(const char* name, int dflt) {
  const char* e = env_get(name);
  return e && *e ? atoi(e) : dflt;
}
static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// One gradient evaluation of the launch: program slot `slot` (a tree, or a speculative slot holding
// tree `tree` at other constants) -> f (+Inf where did_succeed fails), g[0 .. nconst of tree), ok.
struct GradItem {
  int32_t slot, tree;
  double* f;
  double* g;     // unused for value_only items
  uint8_t* ok;   // nullable
  bool value_only = false;  // loss only (a line-search trial point): the cheap KT = 0 kernel
};
// The derived view of constant-gradient launches (GMODE_LOSS: the optimiser and srhip_eval_loss_grad):
// X' = [the program's feature columns | its derived columns U(X[f]) | their tangent-zero columns] in
// the context's g_xd, built once per call (one copy + one launch; reused by the next call over the
// same dataset and spec), so a gradient program reads every heavy operator of a feature as a column
// instead of evaluating it per row, per trial point (C4: ~0.9 per tree, cos / exp of a feature).
// Off below SRHIP_GRAD_DERIVED_MIN_ROWS rows (default 8192), above SRHIP_GRAD_DERIVED_MAX_MB of view
// (default 256) and with SRHIP_GRAD_DERIVED=0.
static int derived_view(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, View& v) {
  P->g_want_derived = false;
  const char* e = env_get("SRHIP_GRAD_DERIVED");
  if (e && *e == '0') return SRHIP_OK;
  if (v.m < env_int_opt("SRHIP_GRAD_DERIVED_MIN_ROWS", 8192)) return SRHIP_OK;
  grad_derived_spec(*P);
  const int nd = (int)P->gdspec.size();
  if (nd == 0 || P->gdbase <= 0) return SRHIP_OK;
  const size_t es = P->dtype == SRHIP_F64 ? 8 : 4;
  const size_t bytes = (size_t)(P->gdbase + 2 * nd) * v.ld * es;
  if (bytes > ((size_t)env_int_opt("SRHIP_GRAD_DERIVED_MAX_MB", 256) << 20)) return SRHIP_OK;  // (a copy per call)
  // a view of the whole dataset (not a gathered batch) with the same spec as the last build: reused
  const bool whole = v.X == ds->X.p;
  const bool same = whole && ctx->g_xd.p && ctx->g_xd_serial == ds->serial && ctx->g_xd_ld == v.ld &&
                    ctx->g_xd_dtype == P->dtype && ctx->g_xd_base == P->gdbase && ctx->g_xd_spec == P->gdspec;
  if (!same) {
    ctx->g_xd_serial = 0;  // (until rebuilt)
    HIP_TRY(ctx->g_xd.ensure(bytes));
    HIP_TRY(hipMemcpyAsync(ctx->g_xd.p, v.X, (size_t)P->gdbase * v.ld * es, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(launch_grad_derive(P->dtype, v.X, (uint8_t*)ctx->g_xd.p + (size_t)P->gdbase * v.ld * es, v.ld,
                               P->gdspec.data(), nd, ctx->stream));
    // the split optimiser's auxiliary contexts read the view from their own streams: it must be
    // complete before this returns (as make_view's is), not merely queued on ctx->stream
    HIP_TRY(hipStreamSynchronize(ctx->stream));  // (C4 unchanged: 141.7-142.5 ms without it, 142.5-144.3 with)
    if (whole) {
      ctx->g_xd_serial = ds->serial;
      ctx->g_xd_ld = v.ld;
      ctx->g_xd_dtype = P->dtype;
      ctx->g_xd_base = P->gdbase;
      ctx->g_xd_spec = P->gdspec;
    }
  }
  v.X = ctx->g_xd.p;
  v.nfeat_x = P->gdbase;
  v.nd_x = nd;
  P->g_want_derived = true;
  return SRHIP_OK;
}

static int eval_grad_items(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss,
                           const View& v, const std::vector<GradItem>& items, bool timed = true);
// Loss and gradient for `trees` at the program's current constants: f[t], g[coff[t] ..], ok[t]
// (nullable; did_succeed -- a tree can succeed with an overflowing loss: f = Inf, ok = 1), plus the
// items in `extra` (speculative slots, already instantiated; their instructions [spec_lo, spec_hi)
// are uploaded with the launch).
static int eval_grad(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss, const View& v,
                     const std::vector<int32_t>& trees, const std::vector<int64_t>& coff, double* f, double* g,
                     uint8_t* ok = nullptr, const std::vector<GradItem>* extra = nullptr, int64_t spec_lo = 0,
                     int64_t spec_hi = -1, const uint8_t* value_only = nullptr, bool timed = true) {
  const double t0 = now_s();
  int rc = compile_grad_program(*P);
  g_t_compile += now_s() - t0;
  g_n_launch += 1;
  if (rc) return rc;
  std::vector<GradItem> items;
  items.reserve(trees.size() + (extra ? extra->size() : 0));
  for (int32_t t : trees)
    items.push_back(GradItem{t, t, f + t, g + coff[t], ok ? ok + t : nullptr, value_only && value_only[t]});
  if (extra) items.insert(items.end(), extra->begin(), extra->end());
  auto body = [&]() -> int {
    if (spec_hi > spec_lo) {  // pinned staging (synchronised with the launch in eval_grad_items)
      const size_t nb = (size_t)(spec_hi - spec_lo) * sizeof(Ins);
      HIP_TRY(ctx->h_gspec.ensure(nb));
      memcpy(ctx->h_gspec.p, P->gcode.data() + spec_lo, nb);
      HIP_TRY(hipMemcpyAsync((Ins*)P->d_gcode.p + spec_lo, ctx->h_gspec.p, nb, hipMemcpyHostToDevice, ctx->stream));
    }
    return eval_grad_items(ctx, ds, P, loss, v, items, timed);
  };
  rc = body();
  // a patched gradient program's upload (compile_grad_program) may still be in flight from P->gcode:
  // on an error return, drain the stream before the caller can destroy or recompile the program
  if (rc) (void)hipStreamSynchronize(ctx->stream);
  return rc;
}
// timed: HIP events around the gradient kernels (srhip_last_kernel_ms).  The optimiser's launches go
// without: two timing events per launch cost C4 ~5 % (149-153 against 141-145 ms on one box).
static int eval_grad_items(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss,
                           const View& v, const std::vector<GradItem>& items, bool timed) {
  const int dtype = P->dtype;
  const bool weighted = ds->weighted;
  const double wsum = weighted ? v.sum_w : (double)v.m;
  // tangent width of the gradient pass: a chunk carries the primal plus kt tangents, so trees with
  // few constants waste most of an 8-wide chunk; estimated cost per chunk ~ (3 + kt) (the primal's
  // transcendentals and derivative factors cost about three tangent updates).  Values and the
  // tangents of each constant do not depend on kt (independent components, same primal code; kt = 0
  // is the value-only pass).
  int64_t cost4 = 0, cost8 = 0;
  for (const GradItem& it : items) {
    if (P->ginfo[it.slot].static_fail || it.value_only) continue;
    const int nc = std::max(P->info[it.tree].nconst, 1);
    cost4 += (int64_t)((nc + 3) / 4) * (3 + 4);
    cost8 += (int64_t)((nc + GRAD_KT - 1) / GRAD_KT) * (3 + GRAD_KT);
  }
  const char* kte = env_get("SRHIP_GRAD_KT");  // tuning / tests: force 4 or 8
  int kt = cost4 < cost8 ? 4 : GRAD_KT;
  if (kte && (atoi(kte) == 4 || atoi(kte) == GRAD_KT)) kt = atoi(kte);
  // two passes on the stream (gradient chunks, then value-only chunks), one synchronisation
  struct Pass {
    int kt;
    std::vector<int32_t> chunks, chunk_item;
    const double* red = nullptr;  // the reduced records, in the context's pinned staging
    LaunchPlan L;
  } pass[2];
  pass[0].kt = kt;
  pass[1].kt = 0;
  for (size_t i = 0; i < items.size(); ++i) {
    const GradItem& it = items[i];
    *it.f = INFINITY;
    if (it.ok) *it.ok = 0;
    const int nc = P->info[it.tree].nconst;
    if (!it.value_only)
      for (int k = 0; k < nc; ++k) it.g[k] = 0.0;
    if (P->ginfo[it.slot].static_fail) continue;
    Pass& ps = pass[it.value_only ? 1 : 0];
    const int span = it.value_only ? 1 : std::max(nc, 1);
    for (int c0 = 0; c0 < span; c0 += std::max(ps.kt, 1)) {
      ps.chunks.push_back(it.slot);
      ps.chunks.push_back(c0);
      ps.chunk_item.push_back((int32_t)i);
    }
  }
  const int nch0 = (int)pass[0].chunks.size() / 2, nch1 = (int)pass[1].chunks.size() / 2;
  if (nch0 + nch1 == 0) {  // a patched gradient program may still be uploading from P->gcode
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SRHIP_OK;
  }
  // buffers sized for both passes before the first launch (no reallocation under a queued kernel)
  size_t slab_n = 0, red_n = 0, chunk_n = 0;
  for (Pass& ps : pass) {
    const int nch = (int)ps.chunks.size() / 2;
    if (nch == 0) continue;
    ps.L = grad_plan(ctx, v.m, nch);
    // launch order: descending estimated cost, dealt round-robin over the tree groups (each group's
    // range stays contiguous), so every group gets the same cost mix and its waves -- which claim
    // chunks dynamically -- start with the longest ones.  Records are read back by position.
    if (nch > 1) {
      std::vector<int32_t> by(nch);
      std::iota(by.begin(), by.end(), 0);
      std::stable_sort(by.begin(), by.end(), [&](int32_t x, int32_t y) {
        return P->ginfo[ps.chunks[2 * x]].cost > P->ginfo[ps.chunks[2 * y]].cost;
      });
      const int G = ps.L.groups, tpg = ps.L.tpg;
      std::vector<int32_t> fill(G, 0), chunks2(ps.chunks.size()), item2(nch);
      int g = 0;
      for (int32_t k : by) {
        while (fill[g] >= std::min(tpg, nch - g * tpg)) g = (g + 1) % G;
        const int pos = g * tpg + fill[g]++;
        chunks2[2 * pos] = ps.chunks[2 * k];
        chunks2[2 * pos + 1] = ps.chunks[2 * k + 1];
        item2[pos] = ps.chunk_item[k];
        g = (g + 1) % G;
      }
      ps.chunks.swap(chunks2);
      ps.chunk_item.swap(item2);
    }
    slab_n = std::max(slab_n, (size_t)nch * ps.L.nrb * (ps.kt + 2));
    red_n = std::max(red_n, (size_t)nch * (ps.kt + 2));
    chunk_n = std::max(chunk_n, ps.chunks.size());
  }
  HIP_TRY(ctx->g_chunks.ensure(chunk_n * sizeof(int32_t)));
  HIP_TRY(ctx->g_slab.ensure(slab_n * sizeof(double)));
  HIP_TRY(ctx->g_red.ensure(red_n * sizeof(double)));
  const int K = P->gkmax <= 2 ? 2 : (P->gkmax <= 4 ? 4 : 8);  // stack slots of the kernel variant
  bool first = true;
  for (int pi = 0; pi < 2; ++pi) {
    Pass& ps = pass[pi];
    const int nch = (int)ps.chunks.size() / 2;
    if (nch == 0) continue;
    // pinned staging both ways (a pageable source or destination makes the runtime stage the copy
    // through its own buffer, synchronously); stream order: this copy follows the previous pass's
    // kernel, which has read its chunk list
    HIP_TRY(ctx->h_gred[pi].ensure((size_t)nch * (ps.kt + 2) * sizeof(double), hipHostMallocCoherent));
    GradArgs a{};
    // SRHIP_GRAD_INLINE_MAX (0: always copy the list), read per pass through the environment cache
    // so a test can compare both forms in one process
    const char* ie = env_get("SRHIP_GRAD_INLINE_MAX");
    const int inline_max = ie && *ie ? std::max(0, std::min(atoi(ie), GRAD_INLINE)) : GRAD_INLINE;
    const bool inl = nch <= inline_max;
    if (inl) {  // in the kernel arguments
      memcpy(a.inl, ps.chunks.data(), ps.chunks.size() * sizeof(int32_t));
    } else {
      HIP_TRY(ctx->h_gchunks[pi].ensure(ps.chunks.size() * sizeof(int32_t)));
      memcpy(ctx->h_gchunks[pi].p, ps.chunks.data(), ps.chunks.size() * sizeof(int32_t));
      HIP_TRY(hipMemcpyAsync(ctx->g_chunks.p, ctx->h_gchunks[pi].p, ps.chunks.size() * sizeof(int32_t),
                             hipMemcpyHostToDevice, ctx->stream));
    }
    a.code = (const Ins*)P->d_gcode.p;
    a.prog_off = (const int32_t*)P->d_goff.p;
    a.chunks = inl ? nullptr : (const int32_t*)ctx->g_chunks.p;
    a.X = v.X;
    a.y = v.y;
    a.w = weighted ? v.w : nullptr;
    a.slab = (double*)ctx->g_slab.p;
    a.ld = v.ld;
    a.nvalid = v.m;
    a.nchunks = nch;
    a.nfeat = v.nfeat_x >= 0 ? v.nfeat_x : (int32_t)ds->nfeat;
    a.gd_nd = v.nd_x;
    a.rb_rows = ps.L.rb_rows;
    a.nrb = ps.L.nrb;
    a.chunks_per_group = ps.L.tpg;
    a.loss_kind = loss->kind;
    a.loss_p0 = loss->p0;
    a.weighted = weighted ? 1 : 0;
    a.max_steps = P->gmax_len;
    if (first && timed) HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));  // srhip_last_kernel_ms: the gradient kernels
    first = false;
    // value-only screening (SRHIP_GRAD_SCREEN = the fewest value-only chunks screened; default 0 =
    // off): row block 0 of every chunk first, in a launch of its own, then the other blocks, where a
    // chunk whose block-0 check statistic is already non-finite is skipped.  Records of evaluated
    // blocks are the same computation as in one launch, so losses and decisions are bit-identical
    // (test_value_only_screening_is_exact).  C4 (~40 % of its trial points overflow), same box:
    // off 173.6-177.9 ms, every pass 190-193, passes of >= 16 chunks 176.8-179.6 -- the extra launch
    // costs what the skipped blocks save at 100k rows.
    const int screen_min = env_int_opt("SRHIP_GRAD_SCREEN", 0);
    if (ps.kt == 0 && screen_min > 0 && nch >= screen_min && ps.L.nrb > 1) {
      GradArgs sa = a;
      const int tpg_s = 2 * GRAD_WAVES;
      sa.chunks_per_group = tpg_s;
      HIP_TRY(launch_grad(dtype, K, 0, sa, dim3(1, (nch + tpg_s - 1) / tpg_s), ctx->stream));
      a.block0 = 1;
      a.screened = 1;
      HIP_TRY(launch_grad(dtype, K, 0, a, dim3(ps.L.nrb - 1, ps.L.groups), ctx->stream));
    } else {
      HIP_TRY(launch_grad(dtype, K, ps.kt, a, dim3(ps.L.nrb, ps.L.groups), ctx->stream));
    }
    // the reduction writes the records straight into coherent pinned host memory (no copy on the stream)
    HIP_TRY(launch_grad_reduce(dtype, ps.kt, (const double*)ctx->g_slab.p, ps.L.nrb, nch, (double*)ctx->h_gred[pi].p,
                               ctx->stream));
    ps.red = (const double*)ctx->h_gred[pi].p;
  }
  if (timed) HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
  ctx->timed = timed;
  ctx->last_ev0 = ctx->ev0;
  ctx->last_ev1 = ctx->ev1;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  // decision inputs in the partials layout: only the feature statistics and the row count are read
  std::vector<double> sums(2 * (size_t)P->ntrees + 2 * ds->nfeat + 1, 0.0);
  for (int64_t fi = 0; fi < ds->nfeat; ++fi) {
    sums[2 * (size_t)P->ntrees + 2 * fi] = v.stats[fi].sum;
    sums[2 * (size_t)P->ntrees + 2 * fi + 1] = (double)v.stats[fi].nonfinite;
  }
  sums.back() = (double)v.m;
  std::vector<int32_t> undecided, undecided_item;
  for (const Pass& ps : pass) {
    const int nch = (int)ps.chunks.size() / 2;
    for (int c = 0; c < nch; ++c) {
      const GradItem& it = items[ps.chunk_item[c]];
      const int32_t c0 = ps.chunks[2 * c + 1];
      const double* r = ps.red + (size_t)c * (ps.kt + 2);
      const int nc = P->info[it.tree].nconst;
      for (int j = 0; j < ps.kt && c0 + j < nc; ++j) it.g[c0 + j] = r[1 + j] / wsum;
      if (c0 == 0) {
        const int st = decide_tree(P->ginfo[it.slot], *P, ds->nfeat, sums.data(), r[ps.kt + 1]);
        *it.f = st == 1 ? INFINITY : r[0] / wsum;
        if (it.ok) *it.ok = st != 1;
        if (st == 2) {
          undecided.push_back(it.slot);
          undecided_item.push_back(ps.chunk_item[c]);
        }
      }
    }
  }
  if (g_stats_on)
    for (const GradItem& it : items) {
      int64_t* c = g_items[it.value_only ? 1 : 0][items.size() > 64 ? 1 : 0];
      c[0] += 1;
      c[1] += !std::isfinite(*it.f);
    }
  // near-overflow sums: the exact per-operator-node pass on the gradient program decides, so the
  // objective is eval_loss's (L(Inf) exactly where did_succeed fails)
  if (!undecided.empty()) {
    std::vector<uint8_t> uok(undecided.size());
    const int rc = precise_decide(ctx, ds, P, v, undecided.data(), (int32_t)undecided.size(), true, uok.data());
    if (rc) return rc;
    for (size_t u = 0; u < undecided.size(); ++u)
      if (!uok[u]) {
        const GradItem& it = items[undecided_item[u]];
        *it.f = INFINITY;
        if (it.ok) *it.ok = 0;
      }
  }
  return SRHIP_OK;
}

namespace {

// LineSearches.jl BackTracking (order 3) state of one tree: a finite-value phase (halve alpha while
// phi(alpha) is not finite, at most iterfinitemax = 52 times), then the sufficient-decrease phase
// (cubic / quadratic interpolation, alpha shrunk into [0.1, 0.5] of its last value, at most
// iterations = 1000 times; a non-finite phi there simply fails the test and is interpolated on).
struct LineSearch {
  double phi0, dphi0, a1, a2, phix0, phix1;
  int iter = 0, iterfinite = 0;
  bool armijo = false;  // the finite-value phase is over
};
constexpr int LS_ITERFINITEMAX = 52, LS_ITERATIONS = 1000;

// next trial step after phi(a2) = phix1 failed the sufficient-decrease test
double backtrack_step(LineSearch& s) {
  const double rho_hi = 0.5, rho_lo = 0.1;
  double a_tmp;
  // LineSearches.jl's expressions with Julia's association (x^2 = x*x, x^3 = x*x*x as literal powers)
  if (s.iter == 1) {
    a_tmp = -(s.dphi0 * (s.a2 * s.a2)) / (2.0 * (s.phix1 - s.phi0 - s.dphi0 * s.a2));
  } else {
    const double a1sq = s.a1 * s.a1, a2sq = s.a2 * s.a2;
    const double div = 1.0 / (a1sq * a2sq * (s.a2 - s.a1));
    const double e1 = s.phix1 - s.phi0 - s.dphi0 * s.a2, e0 = s.phix0 - s.phi0 - s.dphi0 * s.a1;
    const double a = (a1sq * e1 - a2sq * e0) * div;
    const double b = (-(s.a1 * s.a1 * s.a1) * e1 + (s.a2 * s.a2 * s.a2) * e0) * div;
    if (fabs(a) <= 2.220446049250313e-16) a_tmp = s.dphi0 / (2.0 * b);
    else a_tmp = (-b + sqrt(std::max(b * b - 3.0 * a * s.dphi0, 0.0))) / (3.0 * a);
  }
  s.a1 = s.a2;
  a_tmp = std::isnan(a_tmp) ? s.a2 * rho_hi : std::min(a_tmp, s.a2 * rho_hi);  // NaNMath.min
  return std::max(a_tmp, s.a2 * rho_lo);
}

// one BackTracking step on phi(a2): LS_CONTINUE (next trial at the new a2), LS_ACCEPT, or a failure
// that ends the start: LS_FAIL (iterations exhausted, LineSearchException) or LS_FAIL_NEGINF (the
// slope overflowed to -Inf: phi0 + c1 a dphi0 = -Inf for every alpha > 0 the remaining iterations can
// reach, so every further trial fails and BackTracking throws after exactly LS_ITERATIONS of them)
enum { LS_CONTINUE = 0, LS_ACCEPT = 1, LS_FAIL = 2, LS_FAIL_NEGINF = 3 };
int ls_update(LineSearch& L, double phi) {
  L.phix1 = phi;
  if (!L.armijo) {
    if (!std::isfinite(phi) && L.iterfinite < LS_ITERFINITEMAX) {  // hard-coded halving until finite
      L.iterfinite += 1;
      L.a1 = L.a2;
      L.a2 = L.a1 / 2.0;
      return LS_CONTINUE;
    }
    L.armijo = true;
  }
  if (phi > L.phi0 + 1e-4 * L.a2 * L.dphi0) {  // sufficient decrease not met (or phi = Inf)
    if (L.dphi0 == -INFINITY) return LS_FAIL_NEGINF;
    if (++L.iter > LS_ITERATIONS) return LS_FAIL;
    const double a2 = backtrack_step(L);
    L.phix0 = L.phix1;
    L.a2 = a2;
    return LS_CONTINUE;
  }
  return LS_ACCEPT;
}

}  // namespace

// All restarts of all trees as one pipelined batch.  Every tree runs its own state machine
// (initial point -> [Hessian probes] -> line-search trials -> ... -> next restart); each launch
// evaluates the one point every active tree needs next, so a tree never waits for a slower tree's
// line search or restart.  A tree's loss and gradient do not depend on which other trees share the
// launch (fixed row chunks, fixed reduction order), so each tree's trajectory -- and the outcome --
// is the one it would follow optimised alone (tests/test_gpu_optim.py checks this bit for bit).
//
// BFGS (nconst >= 2): Optim's BFGS -- inverse-Hessian approximation from the identity, direction
//   s = -H g (steepest descent if that is not a descent direction), update skipped unless
//   dx'dg > 0.
// Newton (nconst == 1, src/ConstantOptimization.jl:27-31): direction s = -g / |h| (Optim's
//   cholesky!(Positive, H) of a 1x1 Hessian flips a negative curvature and replaces a zero one by
//   1), h = (g(c + e) - g(c - e)) / 2e with e = cbrt(eps) max(1, |c|): two extra gradient launches
//   per iteration ("Hessian probes", not counted as objective calls, as Optim counts h_calls apart).
// Both: BackTracking line search from alpha = 1 (InitialStatic), stop on |g|_inf <= g_tol, on an
//   unchanged objective (f_reltol = x_abstol = 0) or after `iterations` iterations.
//
// Speculative trial points (SRHIP_OPTIM_SPEC slots, default 256, 0 = off): a line search whose last
// trial was non-finite usually keeps failing for many trials (an overflowing direction halves alpha
// ~50 times, then shrinks it in the Armijo phase until x + a s rounds back to x -- hundreds of
// launches for one tree at the pipeline's tail).  While few trees are active, the launch also
// evaluates, in spare program slots (the tree's code with its constant immediates rewritten), the
// next points the tree's BackTracking would try if every pending trial came back non-finite.  After
// the launch they are consumed in order for as long as the line search really asks for exactly that
// alpha (same line search, bitwise-equal alpha), so every consumed result is the one the sequential
// pipeline would have launched for: trajectories, outcomes and objective-call counts are unchanged.
static int bfgs_pipelined(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss,
                          const View& v, const std::vector<int32_t>& trees, const std::vector<int64_t>& coff,
                          int iterations, double g_tol, const std::vector<std::vector<double>>& starts,
                          std::vector<double>& best_x, std::vector<double>& best_f, std::vector<int64_t>& fcalls) {
  enum { INIT = 0, TRIAL = 1, DONE = 2, HESS_P = 3, HESS_M = 4, GRADAT = 5 };
  const int nstarts = (int)starts.size();
  const size_t nall = best_x.size();
  std::vector<double> x(nall), g(nall), s(nall), xe(nall), fe(P->ntrees), ge(nall), f(P->ntrees, INFINITY);
  std::vector<double> hstep(P->ntrees, 0.0), gplus(P->ntrees, 0.0), hcurv(P->ntrees, 1.0);
  std::vector<int64_t> hoff(P->ntrees + 1, 0);
  for (int32_t t = 0; t < P->ntrees; ++t) {
    const int64_t n = coff[t + 1] - coff[t];
    hoff[t + 1] = hoff[t] + n * n;
  }
  std::vector<double> H(hoff.back(), 0.0);
  std::vector<int> phase(P->ntrees, DONE), start(P->ntrees, 0), iter(P->ntrees, 0);
  std::vector<LineSearch> ls(P->ntrees);
  // consecutive non-finite trials of the current line search, and a line-search generation counter
  std::vector<int> nfstreak(P->ntrees, 0);
  std::vector<int64_t> lsgen(P->ntrees, 0);
  // the last two finite trial points (alpha, phi) of the current line search, newest first: the
  // speculation's model of phi along the search direction
  struct Hist {
    int n = 0;
    double a[2], f[2];
  };
  std::vector<Hist> hist(P->ntrees);
  // per-tree speculation depth: doubled while every speculative point of a launch is consumed,
  // cut back to what was consumed (+1) after a misprediction
  std::vector<int> sdepth(P->ntrees, 4);
  // value-only trial points (SRHIP_OPTIM_VALUE_TRIALS, default on): a line search's trials after its
  // first are evaluated without tangents; an accepted one is re-evaluated with its gradient (phase
  // GRADAT, same point, same loss bits, not an objective call)
  const char* vte = getenv("SRHIP_OPTIM_VALUE_TRIALS");
  const bool value_trials = !(vte && *vte == '0');
  std::vector<uint8_t> vonly(P->ntrees, 0);
  std::vector<double> xacc(nall), phiacc(P->ntrees, 0.0);
  for (size_t k = 0; k < nall; ++k) xe[k] = best_x[k];
  auto newton = [&](int32_t t) { return coff[t + 1] - coff[t] == 1; };
  auto gnorm = [&](int32_t t, const std::vector<double>& gg) {
    double m = 0.0;
    for (int64_t k = coff[t]; k < coff[t + 1]; ++k) m = std::max(m, fabs(gg[k]));
    return m;
  };
  auto begin_start = [&](int32_t t) {
    const int64_t n = coff[t + 1] - coff[t], o = coff[t];
    for (int64_t k = o; k < o + n; ++k) x[k] = starts[start[t]][k];
    for (int64_t i = 0; i < n; ++i)
      for (int64_t j = 0; j < n; ++j) H[hoff[t] + i * n + j] = i == j ? 1.0 : 0.0;
    phase[t] = INIT;
  };
  auto finish_start = [&](int32_t t) {
    // the first start is `result` unconditionally (:50); a restart replaces it only if strictly
    // better (:65-67)
    if (start[t] == 0 || f[t] < best_f[t]) {
      best_f[t] = f[t];
      for (int64_t k = coff[t]; k < coff[t + 1]; ++k) best_x[k] = x[k];
    }
    if (++start[t] < nstarts) begin_start(t);
    else phase[t] = DONE;
  };
  // Newton: probe the gradient at c + e and c - e for the curvature at the current point
  auto begin_hess = [&](int32_t t) {
    hstep[t] = 6.055454452393343e-06 * std::max(1.0, fabs(x[coff[t]]));  // cbrt(eps(Float64))
    phase[t] = HESS_P;
  };
  // next iteration of t from (x, f, g): search direction and a fresh line search
  auto begin_iter = [&](int32_t t) {
    if (iter[t] >= iterations) {
      finish_start(t);
      return;
    }
    const int64_t n = coff[t + 1] - coff[t], o = coff[t];
    double dphi = 0.0;
    if (newton(t)) {
      s[o] = -g[o] / hcurv[t];
      dphi = g[o] * s[o];
    } else {
      for (int64_t i = 0; i < n; ++i) {
        double acc = 0.0;
        for (int64_t j = 0; j < n; ++j) acc += H[hoff[t] + i * n + j] * g[o + j];
        s[o + i] = -acc;
        dphi += g[o + i] * s[o + i];
      }
      if (!(dphi < 0.0)) {
        dphi = 0.0;
        for (int64_t i = 0; i < n; ++i) {
          for (int64_t j = 0; j < n; ++j) H[hoff[t] + i * n + j] = i == j ? 1.0 : 0.0;
          s[o + i] = -g[o + i];
          dphi -= g[o + i] * g[o + i];
        }
      }
    }
    LineSearch& L = ls[t];
    L = LineSearch();
    L.phi0 = f[t];
    L.dphi0 = dphi;
    L.a1 = L.a2 = 1.0;  // InitialStatic: alpha = 1
    L.phix0 = L.phix1 = f[t];
    phase[t] = TRIAL;
    nfstreak[t] = 0;
    lsgen[t] += 1;
    hist[t] = Hist();
  };
  auto next_iter = [&](int32_t t) {  // after an accepted step
    iter[t] += 1;
    if (newton(t) && iter[t] < iterations) begin_hess(t);
    else begin_iter(t);
  };
  const char* tre = getenv("SRHIP_OPTIM_TRACE");
  const int trace_tree = tre && *tre ? atoi(tre) : -1;
  // one evaluation result of tree t at the point xv: loss phi, gradient gv
  // an accepted step to (xv, phi) with gradient gv there: BFGS update, then converge or iterate
  auto accept = [&](int32_t t, double phi, const double* gv, const double* xv) {
    const int64_t o = coff[t], n = coff[t + 1] - coff[t];
    const LineSearch& L = ls[t];
    if (!newton(t)) {
      std::vector<double> dx(n), dg(n), u(n);
      double dxdg = 0.0;
      for (int64_t i = 0; i < n; ++i) {
        dx[i] = L.a2 * s[o + i];
        dg[i] = gv[i] - g[o + i];
        dxdg += dx[i] * dg[i];
      }
      if (dxdg > 0.0) {
        double dgu = 0.0;
        for (int64_t i = 0; i < n; ++i) {
          double acc = 0.0;
          for (int64_t j = 0; j < n; ++j) acc += H[hoff[t] + i * n + j] * dg[j];
          u[i] = acc;
          dgu += dg[i] * acc;
        }
        const double c1 = (dxdg + dgu) / (dxdg * dxdg), c2 = 1.0 / dxdg;
        for (int64_t i = 0; i < n; ++i)
          for (int64_t j = 0; j < n; ++j)
            H[hoff[t] + i * n + j] += c1 * dx[i] * dx[j] - c2 * (u[i] * dx[j] + dx[i] * u[j]);
      }
    }
    const double fold = f[t];
    for (int64_t k = 0; k < n; ++k) {
      x[o + k] = xv[k];
      g[o + k] = gv[k];
    }
    f[t] = phi;
    if (phi == fold || gnorm(t, g) <= g_tol) finish_start(t);  // converged
    else next_iter(t);
  };
  // one evaluation result of tree t at the point xv: loss phi, gradient gv (nullptr: value only)
  auto consume = [&](int32_t t, double phi, const double* gv, const double* xv) {
    const int64_t o = coff[t], n = coff[t + 1] - coff[t];
    if (t == trace_tree) {  // SRHIP_OPTIM_TRACE=<tree>: every evaluation of one tree, stderr
      fprintf(stderr, "[srhip optim] tree %d start %d iter %d phase %d a %.17g f %.17g x", t, start[t], iter[t],
              phase[t], phase[t] == TRIAL ? ls[t].a2 : 0.0, phi);
      for (int64_t k = 0; k < n; ++k) fprintf(stderr, " %.17g", xv[k]);
      fprintf(stderr, " g");
      for (int64_t k = 0; k < n; ++k) fprintf(stderr, gv ? " %.17g" : " -", gv ? gv[k] : 0.0);
      fprintf(stderr, "\n");
    }
    if (phase[t] == GRADAT) {  // the gradient at an accepted value-only trial point
      accept(t, phiacc[t], gv, xacc.data() + o);
      return;
    }
    if (phase[t] == HESS_P) {
      gplus[t] = std::isfinite(phi) ? gv[0] : NAN;
      phase[t] = HESS_M;
      return;
    }
    if (phase[t] == HESS_M) {
      const double h = std::isfinite(phi) ? (gplus[t] - gv[0]) / (2.0 * hstep[t]) : NAN;
      hcurv[t] = (std::isfinite(h) && h != 0.0) ? fabs(h) : 1.0;  // cholesky!(Positive, [h])
      begin_iter(t);
      return;
    }
    fcalls[t] += 1;
    if (phase[t] == INIT) {
      f[t] = phi;
      for (int64_t k = 0; k < n; ++k) g[o + k] = gv[k];
      iter[t] = 0;
      if (!std::isfinite(f[t]) || gnorm(t, g) <= g_tol) finish_start(t);
      else if (newton(t) && iterations > 0) begin_hess(t);
      else begin_iter(t);
      return;
    }
    if (g_stats_on && !std::isfinite(phi)) g_nonfinite_trials += 1;
    LineSearch& L = ls[t];
    if (std::isfinite(phi)) {
      Hist& h = hist[t];
      h.a[1] = h.a[0];
      h.f[1] = h.f[0];
      h.a[0] = L.a2;
      h.f[0] = phi;
      h.n = std::min(h.n + 1, 2);
    }
    switch (ls_update(L, phi)) {
      case LS_CONTINUE: nfstreak[t] = std::isfinite(phi) ? 0 : nfstreak[t] + 1; return;
      case LS_FAIL_NEGINF: fcalls[t] += LS_ITERATIONS - L.iter; finish_start(t); return;  // counted, not launched
      case LS_FAIL: finish_start(t); return;  // LineSearchException: the start ends at its last accepted point
      default: break;
    }
    if (!gv) {  // accepted without a gradient: fetch it at this point next launch
      for (int64_t k = 0; k < n; ++k) xacc[o + k] = xv[k];
      phiacc[t] = phi;
      phase[t] = GRADAT;
      return;
    }
    accept(t, phi, gv, xv);
  };
  for (int32_t t : trees) begin_start(t);
  const char* spe = getenv("SRHIP_OPTIM_SPEC");
  // default 32 slots: a launch of a few trees is latency-bound (one tree x 100k rows fills ~5 % of
  // the wave slots), so a few dozen extra points cost little; more only adds mispredicted work
  const int spec_cap = spe && *spe ? std::max(0, std::min(atoi(spe), 4096)) : 32;
  // speculate only in the pipeline's tail (SRHIP_OPTIM_SPEC_ACTIVE, default 64 active trees), at most
  // SRHIP_OPTIM_SPEC_DEPTH (default 64) points per tree and launch
  const size_t SPEC_MAX_ACTIVE = (size_t)std::max(0, env_int_opt("SRHIP_OPTIM_SPEC_ACTIVE", 64));
  const int SPEC_MAX_DEPTH = std::max(1, env_int_opt("SRHIP_OPTIM_SPEC_DEPTH", 64));
  if (P->gspec_cap != spec_cap) {
    P->gspec_cap = spec_cap;  // the next gradient compile allocates the slots (a full compile)
    P->grad_ready = false;
  }
  struct Spec {
    int32_t t, slot;
    int64_t gen;
    double alpha;
    int64_t off;  // into sx / sg
  };
  std::vector<Spec> spec;
  std::vector<double> sx, sg, sf;
  std::vector<GradItem> sitems;
  std::vector<int32_t> act;
  for (;;) {
    act.clear();
    for (int32_t t : trees) {
      if (phase[t] == DONE) continue;
      act.push_back(t);
      const int64_t o = coff[t], e = coff[t + 1];
      switch (phase[t]) {
        case INIT: for (int64_t k = o; k < e; ++k) xe[k] = x[k]; break;
        case TRIAL: for (int64_t k = o; k < e; ++k) xe[k] = x[k] + ls[t].a2 * s[k]; break;
        case HESS_P: xe[o] = x[o] + hstep[t]; break;
        case HESS_M: xe[o] = x[o] - hstep[t]; break;
        case GRADAT: for (int64_t k = o; k < e; ++k) xe[k] = xacc[k]; break;
        default: break;
      }
      // trials after a line search's first: loss only
      vonly[t] = value_trials && phase[t] == TRIAL && ls[t].iter + ls[t].iterfinite >= 1;
    }
    if (act.empty()) break;
    const double t0 = now_s();
    for (int32_t t : act) {  // only the active trees' constants change (get_constants order per tree)
      const double* c = xe.data() + coff[t];
      set_consts_rec(P->nodes.data() + P->offsets[t], 0, c);
    }
    // the patch scans just the trees whose constants moved (a union if an earlier hint is pending;
    // no hint at all -- an unknown change -- keeps the full scan)
    if (P->grad_ready) P->ghint = act;
    else if (!P->ghint.empty()) P->ghint.insert(P->ghint.end(), act.begin(), act.end());
    P->grad_ready = false;
    // speculative points of trees in a non-finite streak (instantiated after the compile / patch:
    // a full compile resets the slot region)
    spec.clear();
    sitems.clear();
    int64_t spec_lo = INT64_MAX, spec_hi = -1;
    if (spec_cap > 0 && act.size() <= SPEC_MAX_ACTIVE) {
      // a line search that has already failed twice is likely to keep backtracking
      auto candidate = [&](int32_t t) {
        return phase[t] == TRIAL && ls[t].iter + ls[t].iterfinite >= 2;
      };
      int ncand = 0;
      for (int32_t t : act) ncand += candidate(t);
      if (ncand > 0) {
        const double tc = now_s();
        int rc = compile_grad_program(*P);
        g_t_compile += now_s() - tc;
        if (rc) return rc;
        int slot = 0;
        int64_t off = 0;
        for (int32_t t : act) {
          const int depth = std::min(std::min(sdepth[t], SPEC_MAX_DEPTH), P->gspec_alloc - slot);
          if (depth < 1 || !candidate(t)) continue;
          // the line search run ahead on predicted values: non-finite again after a non-finite
          // trial; otherwise phi(a) = phi0 + d (a / a_k)^q through the last two finite points (q = 2
          // from one).  Only the alphas matter, and BackTracking's steps are mostly its clamps
          // (0.5 or 0.1 of the last alpha), which a rough model reproduces bit for bit.
          const Hist& h = hist[t];
          const double phi0 = ls[t].phi0;
          double q = 2.0;
          if (h.n == 2 && h.f[0] > phi0 && h.f[1] > phi0 && h.a[0] != h.a[1] && h.a[0] > 0.0 && h.a[1] > 0.0)
            q = log((h.f[1] - phi0) / (h.f[0] - phi0)) / log(h.a[1] / h.a[0]);
          const bool model = nfstreak[t] == 0 && h.n > 0 && h.f[0] > phi0 && h.a[0] > 0.0 && std::isfinite(q);
          if (nfstreak[t] == 0 && !model) continue;
          LineSearch Ls = ls[t];
          for (int j = 0; j < depth; ++j) {
            const double phi_pred = model ? phi0 + (h.f[0] - phi0) * pow(Ls.a2 / h.a[0], q) : INFINITY;
            if (ls_update(Ls, phi_pred) != LS_CONTINUE) break;
            spec.push_back(Spec{t, slot++, lsgen[t], Ls.a2, off});
            off += coff[t + 1] - coff[t];
          }
        }
        sx.resize(off);
        sg.resize(off);
        sf.resize(spec.size());
        size_t keep = 0;
        int32_t dead = -1;  // a tree whose chain broke (slot instantiation refused): drop its rest
        for (size_t i = 0; i < spec.size(); ++i) {
          const Spec& q = spec[i];
          if (q.t == dead) continue;
          const int64_t o = coff[q.t], n = coff[q.t + 1] - o;
          for (int64_t k = 0; k < n; ++k) sx[q.off + k] = x[o + k] + q.alpha * s[o + k];
          bool sfail = false;
          if (!spec_instantiate(*P, q.slot, q.t, sx.data() + q.off, &sfail, spec_lo, spec_hi)) {
            dead = q.t;
            continue;
          }
          spec[keep++] = q;
        }
        spec.resize(keep);
        for (size_t i = 0; i < spec.size(); ++i)
          sitems.push_back(GradItem{P->ntrees + spec[i].slot, spec[i].t, &sf[i], sg.data() + spec[i].off, nullptr,
                                    value_trials});
        g_spec_launched += (int64_t)spec.size();
      }
    }
    const double t1 = now_s();
    int rc = eval_grad(ctx, ds, P, loss, v, act, coff, fe.data(), ge.data(), nullptr, &sitems, spec_lo, spec_hi,
                       vonly.data(), /*timed=*/false);
    if (rc) return rc;
    if (g_stats_on)  // SRHIP_OPTIM_TIMING=2: launch-size histogram
      g_hist[act.size() <= 1 ? 0 : act.size() <= 4 ? 1 : act.size() <= 16 ? 2 : act.size() <= 64 ? 3 : 4] += 1;
    const double t2 = now_s();
    g_t_host += t1 - t0;
    g_t_eval += t2 - t1;
    size_t si = 0;
    int64_t used_all = 0;
    for (int32_t t : act) {
      const int64_t o = coff[t];
      consume(t, fe[t], vonly[t] ? nullptr : ge.data() + o, xe.data() + o);
      // then t's speculative points, in order, while its line search asks for exactly them
      int launched = 0, used = 0;
      bool hit = true;
      for (; si < spec.size() && spec[si].t == t; ++si) {
        const Spec& q = spec[si];
        launched += 1;
        hit = hit && phase[t] == TRIAL && lsgen[t] == q.gen && memcmp(&ls[t].a2, &q.alpha, sizeof(double)) == 0;
        if (!hit) continue;
        consume(t, sf[si], value_trials ? nullptr : sg.data() + q.off, sx.data() + q.off);
        used += 1;
      }
      used_all += used;
      if (launched > 0) {
        g_spec_used += used;
        // all used and still searching: go deeper; else keep what would have been used (+1)
        sdepth[t] = used == launched && phase[t] == TRIAL ? std::min(2 * sdepth[t], SPEC_MAX_DEPTH)
                                                          : std::max(1, std::min(sdepth[t], used + 1));
      }
    }
    if (g_launch_log) {
      int nv = 0, ntrial = 0;
      for (int32_t t : act) {
        nv += vonly[t];
        ntrial += phase[t] == TRIAL;
      }
      fprintf(stderr, "srhip launch: t %.3f act %zu trial %d vonly %d spec %zu used %lld host %.3f eval %.3f ms\n",
              1e3 * t2, act.size(), ntrial, nv, spec.size(), (long long)used_all, 1e3 * (t1 - t0), 1e3 * (t2 - t1));
    }
  }
  if (g_stats_on) {  // the trees with the most objective calls (the pipeline's tail)
    std::vector<int32_t> by(trees);
    std::sort(by.begin(), by.end(), [&](int32_t a, int32_t b) { return fcalls[a] > fcalls[b]; });
    for (size_t i = 0; i < by.size() && i < 4; ++i)
      fprintf(stderr, "srhip optim: tree %d: %lld objective calls, %d constants\n", by[i], (long long)fcalls[by[i]],
              (int)(coff[by[i] + 1] - coff[by[i]]));
  }
  return SRHIP_OK;
}

extern "C" {

int srhip_eval_loss_grad(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss,
                         const int64_t* idx, int64_t nidx, double* out_loss, double* out_grad, uint8_t* out_ok) {
  if (!out_loss || !out_grad || !out_ok) return fail(SRHIP_ERR_INVALID, "null output");
  int rc = check_eval_args(ctx, ds, P, MODE_LOSS, loss);
  if (rc) return rc;
  if (P->dtype == SRHIP_I32) return fail(SRHIP_ERR_UNSUPPORTED, "constant gradients need Float32 / Float64");
  HIP_TRY(hipSetDevice(ctx->device));
  View v;
  rc = make_view(ctx, ds, idx, nidx, true, v);
  if (rc) return rc;
  if (idx && ds->weighted) {
    rc = gathered_weight_sum(ctx, ds, nidx, v);
    if (rc) return rc;
  }
  rc = derived_view(ctx, ds, P, v);
  if (rc) return rc;
  const std::vector<int64_t> coff = const_offsets(*P);
  std::vector<int32_t> all(P->ntrees);
  for (int32_t t = 0; t < P->ntrees; ++t) all[t] = t;
  // (diagnostic, scripts/grad_bench.py: SRHIP_GRAD_VALUE_ONLY=1 runs the line search's value-only pass
  // over every tree -- losses only, the gradients are left zero)
  const char* vo = env_get("SRHIP_GRAD_VALUE_ONLY");
  std::vector<uint8_t> value_only;
  if (vo && atoi(vo) == 1) value_only.assign(P->ntrees, 1);
  rc = eval_grad(ctx, ds, P, loss, v, all, coff, out_loss, out_grad, out_ok, nullptr, 0, -1,
                 value_only.empty() ? nullptr : value_only.data());
  if (rc) return rc;
  return SRHIP_OK;
}

int srhip_eval_grad_predict(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, int32_t wrt, int32_t direction,
                            const int64_t* idx, int64_t nidx, void* out_pred, void* out_grad, uint8_t* out_ok) {
  if (!out_pred || !out_grad || !out_ok) return fail(SRHIP_ERR_INVALID, "null output");
  if (wrt != SRHIP_WRT_CONSTANTS && wrt != SRHIP_WRT_FEATURES) return fail(SRHIP_ERR_INVALID, "wrt %d", wrt);
  int rc = check_eval_args(ctx, ds, P, MODE_PRED, nullptr);
  if (rc) return rc;
  if (P->dtype == SRHIP_I32) return fail(SRHIP_ERR_UNSUPPORTED, "derivatives need Float32 / Float64");
  if (direction < 0 || (direction > 0 && (wrt != SRHIP_WRT_FEATURES || direction > ds->nfeat)))
    return fail(SRHIP_ERR_INVALID, "direction %d (wrt %d, %lld features)", direction, wrt, (long long)ds->nfeat);
  // values and did_succeed: the evaluator itself (eval_tree_array semantics, bit-identical predictions)
  rc = run_eval(ctx, ds, P, MODE_PRED, nullptr, idx, nidx, nullptr, out_pred, out_ok);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  View v;
  rc = make_view(ctx, ds, idx, nidx, false, v);
  if (rc) return rc;
  P->g_want_derived = false;  // per-row derivatives (features: the operators' own) -- no derived columns
  rc = compile_grad_program(*P);
  if (rc) return rc;
  const int32_t nt = P->ntrees;
  const int64_t m = v.m;
  const size_t es = dtype_size(P->dtype);
  // derivative rows of each tree: nconst (constants), nfeatures, or 1 (one direction)
  std::vector<int64_t> row0(nt + 1, 0);
  for (int32_t t = 0; t < nt; ++t)
    row0[t + 1] = row0[t] + (wrt == SRHIP_WRT_CONSTANTS ? P->info[t].nconst : (direction > 0 ? 1 : ds->nfeat));
  const int64_t nrows_out = row0[nt];
  if (nrows_out == 0) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));  // a patched gradient program may still be uploading
    return SRHIP_OK;
  }
  std::vector<int32_t> chunks;
  for (int32_t t = 0; t < nt; ++t) {
    if (P->ginfo[t].static_fail) continue;
    const int64_t nc = row0[t + 1] - row0[t];
    const int32_t first = direction > 0 ? direction - 1 : 0, end = direction > 0 ? direction : (int32_t)nc;
    for (int32_t c0 = first; c0 < end; c0 += GRAD_ROW_KT) {
      chunks.push_back(t);
      chunks.push_back(c0);
      chunks.push_back(end);
      chunks.push_back((int32_t)(row0[t] + c0 - first));
    }
  }
  auto body = [&]() -> int {
    const int nch = (int)chunks.size() / 4;
    DevBuf der;
    HIP_TRY(der.ensure((size_t)nrows_out * m * es));
    if (nch > 0) {
      const LaunchPlan L = grad_plan(ctx, m, nch);
      HIP_TRY(ctx->g_chunks.ensure(chunks.size() * sizeof(int32_t)));
      HIP_TRY(hipMemcpyAsync(ctx->g_chunks.p, chunks.data(), chunks.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                             ctx->stream));
      GradArgs a{};
      a.code = (const Ins*)P->d_gcode.p;
      a.prog_off = (const int32_t*)P->d_goff.p;
      a.chunks = (const int32_t*)ctx->g_chunks.p;
      a.X = v.X;
      a.ld = v.ld;
      a.nvalid = m;
      a.nchunks = nch;
      a.nfeat = (int32_t)ds->nfeat;
      a.rb_rows = L.rb_rows;
      a.nrb = L.nrb;
      a.chunks_per_group = L.tpg;
      a.max_steps = P->gmax_len;
      a.out_der = der.p;
      HIP_TRY(launch_grad_rows(P->dtype, P->gkmax <= 4 ? 4 : 8, wrt == SRHIP_WRT_CONSTANTS ? GMODE_ROWC : GMODE_ROWF, a,
                               dim3(L.nrb, L.groups), ctx->stream));
    }
    HIP_TRY(hipMemcpyAsync(out_grad, der.p, (size_t)nrows_out * m * es, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SRHIP_OK;
  };
  rc = body();
  if (rc) {
    (void)hipStreamSynchronize(ctx->stream);
    return rc;
  }
  // complete = did_succeed of the evaluation and every derivative finite; a static failure's rows NaN
  for (int32_t t = 0; t < nt; ++t) {
    const int64_t n = (row0[t + 1] - row0[t]) * m;
    if (P->ginfo[t].static_fail || P->info[t].static_fail) {
      for (int64_t i = 0; i < n; ++i) {
        if (es == 8) ((double*)out_grad)[row0[t] * m + i] = NAN;
        else ((float*)out_grad)[row0[t] * m + i] = NAN;
      }
      out_ok[t] = 0;
      continue;
    }
    bool fin = true;
    for (int64_t i = 0; i < n && fin; ++i)
      fin = es == 8 ? std::isfinite(((const double*)out_grad)[row0[t] * m + i])
                    : std::isfinite(((const float*)out_grad)[row0[t] * m + i]);
    if (!fin) out_ok[t] = 0;
  }
  return SRHIP_OK;
}

}  // extern "C"

namespace {

// the context's first n auxiliary contexts (created on first use), or fewer if creation fails
std::vector<srhip_ctx*> aux_ctxs(srhip_ctx* ctx, int n) {
  std::lock_guard<std::mutex> g(ctx->aux_mu);
  while ((int)ctx->aux.size() < n) {
    srhip_ctx* a = nullptr;
    if (srhip_ctx_create(ctx->device, &a) != SRHIP_OK) break;
    ctx->aux.push_back(a);
  }
  return std::vector<srhip_ctx*>(ctx->aux.begin(), ctx->aux.begin() + std::min<size_t>(n, ctx->aux.size()));
}

// bfgs_pipelined over G groups of the trees at once (G = SRHIP_OPTIM_SPLIT, default 3; 1 = off;
// populations of fewer than 64 trees are not split): tree i goes to group i % G; group 0 runs on the
// caller's thread and context, group g > 0 as a program of its own on the context's auxiliary
// context g - 1 (own stream and buffers) from a host thread of its own.  Each launch's host
// turnaround (decisions, constant patches, synchronisation) then overlaps the other groups' kernels.
// A tree's trajectory does not depend on the trees that share its launches (fixed row blocks, fixed
// reduction order), so the outcome is the one bfgs_pipelined gives over all trees at once.
int optimize_split(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss, const View& v,
                   const std::vector<int32_t>& trees, const std::vector<int64_t>& coff, int iterations, double g_tol,
                   const std::vector<std::vector<double>>& starts, std::vector<double>& best_x,
                   std::vector<double>& best_f, std::vector<int64_t>& fcalls) {
  const char* se = getenv("SRHIP_OPTIM_SPLIT");
  int G = se && *se ? std::max(1, std::min(atoi(se), 8)) : 3;
  if (trees.size() < 64) G = 1;
  const std::vector<srhip_ctx*> aux = G > 1 ? aux_ctxs(ctx, G - 1) : std::vector<srhip_ctx*>();
  G = 1 + (int)aux.size();
  if (G == 1) return bfgs_pipelined(ctx, ds, P, loss, v, trees, coff, iterations, g_tol, starts, best_x, best_f, fcalls);
  std::vector<std::vector<int32_t>> grp(G);
  for (size_t i = 0; i < trees.size(); ++i) grp[i % G].push_back(trees[i]);
  const srhip_operators ops{(int32_t)P->binops.size(), (int32_t)P->unaops.size(), P->binops.data(),
                            P->unaops.data()};
  struct Part {
    srhip_program* P = nullptr;
    std::vector<int64_t> coff;
    std::vector<std::vector<double>> starts;
    std::vector<double> bx, bf;
    std::vector<int64_t> fc;
    std::vector<int32_t> all;
    int rc = SRHIP_OK;
    std::string err;
    Part() = default;
    Part(const Part&) = delete;  // owns P
    Part& operator=(const Part&) = delete;
    ~Part() { srhip_program_destroy(P); }
  };
  std::vector<Part> part(G);
  for (int gi = 1; gi < G; ++gi) {
    Part& q = part[gi];
    const std::vector<int32_t>& tb = grp[gi];
    std::vector<srhip_node> nodes2;
    std::vector<int64_t> offs2(1, 0);
    for (int32_t t : tb) {
      nodes2.insert(nodes2.end(), P->nodes.begin() + P->offsets[t], P->nodes.begin() + P->offsets[t + 1]);
      offs2.push_back((int64_t)nodes2.size());
    }
    const int32_t n2 = (int32_t)tb.size();
    const int rc = srhip_program_create(aux[gi - 1], P->dtype, nodes2.data(), offs2.data(), n2, &ops, &q.P);
    if (rc) return rc;
    // the caller's derived view serves every group: the same column numbering
    q.P->gdspec = P->gdspec;
    q.P->gdbase = P->gdbase;
    q.P->gdspec_done = P->gdspec_done;
    q.P->g_want_derived = P->g_want_derived;
    q.coff = const_offsets(*q.P);
    q.starts.assign(starts.size(), std::vector<double>(q.coff.back()));
    q.bx.resize(q.coff.back());
    q.bf.resize(n2);
    q.fc.resize(n2);
    q.all.resize(n2);
    for (int32_t j = 0; j < n2; ++j) {
      const int32_t t = tb[j];
      for (int64_t k = 0; k < q.coff[j + 1] - q.coff[j]; ++k) {
        for (size_t s = 0; s < starts.size(); ++s) q.starts[s][q.coff[j] + k] = starts[s][coff[t] + k];
        q.bx[q.coff[j] + k] = best_x[coff[t] + k];
      }
      q.bf[j] = best_f[t];
      q.fc[j] = fcalls[t];
      q.all[j] = j;
    }
  }
  std::vector<std::thread> th;
  for (int gi = 1; gi < G; ++gi)
    th.emplace_back([&, gi] {
      Part& q = part[gi];
      srhip_ctx* c = aux[gi - 1];
      (void)hipSetDevice(c->device);
      q.rc = bfgs_pipelined(c, ds, q.P, loss, v, q.all, q.coff, iterations, g_tol, q.starts, q.bx, q.bf, q.fc);
      if (q.rc) q.err = last_error();
    });
  const int rc = bfgs_pipelined(ctx, ds, P, loss, v, grp[0], coff, iterations, g_tol, starts, best_x, best_f, fcalls);
  for (std::thread& t : th) t.join();
  if (rc) return rc;
  for (int gi = 1; gi < G; ++gi) {
    Part& q = part[gi];
    if (q.rc) return fail(q.rc, "%s", q.err.c_str());
    for (int32_t j = 0; j < (int32_t)grp[gi].size(); ++j) {
      const int32_t t = grp[gi][j];
      for (int64_t k = 0; k < q.coff[j + 1] - q.coff[j]; ++k) best_x[coff[t] + k] = q.bx[q.coff[j] + k];
      best_f[t] = q.bf[j];
      fcalls[t] = q.fc[j];
    }
  }
  return SRHIP_OK;
}

}  // namespace

extern "C" {

int srhip_optimize_constants_starts(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P,
                                    const srhip_loss* loss, const int64_t* idx, int64_t nidx,
                                    const srhip_optim_options* opt, const double* starts_in, double* starts_out,
                                    double* out_loss, uint8_t* out_improved, int64_t* out_fcalls) {
  if (!opt || !out_loss || !out_improved) return fail(SRHIP_ERR_INVALID, "null argument");
  if (opt->iterations < 0 || opt->nrestarts < 0) return fail(SRHIP_ERR_INVALID, "negative iterations / restarts");
  int rc = check_eval_args(ctx, ds, P, MODE_LOSS, loss);
  if (rc) return rc;
  if (P->dtype == SRHIP_I32) return fail(SRHIP_ERR_UNSUPPORTED, "constant optimisation needs Float32 / Float64");
  HIP_TRY(hipSetDevice(ctx->device));
  const int32_t nt = P->ntrees;
  // baseline = f(tree) with the evaluator itself (src/ConstantOptimization.jl:49)
  std::vector<double> base(nt);
  std::vector<uint8_t> base_ok(nt);
  rc = run_eval(ctx, ds, P, MODE_LOSS, loss, idx, nidx, base.data(), nullptr, base_ok.data());
  if (rc) return rc;
  View v;
  rc = make_view(ctx, ds, idx, nidx, true, v);
  if (rc) return rc;
  if (idx && ds->weighted) {
    rc = gathered_weight_sum(ctx, ds, nidx, v);
    if (rc) return rc;
  }
  rc = derived_view(ctx, ds, P, v);
  if (rc) return rc;
  const std::vector<int64_t> coff = const_offsets(*P);
  const std::vector<double> x0 = get_all_consts(*P);
  std::vector<int32_t> trees;  // trees with constants (nconst == 0: nothing to optimise, :35)
  for (int32_t t = 0; t < nt; ++t)
    if (P->info[t].nconst > 0 && !P->info[t].static_fail) trees.push_back(t);
  std::vector<double> best_x = x0, best_f(nt, INFINITY);
  std::vector<int64_t> fcalls(nt, 0);
  std::mt19937_64 rng(opt->seed);
  std::normal_distribution<double> randn(0.0, 1.0);
  const double g_tol = opt->g_tol > 0 ? opt->g_tol : 1e-8;
  if (!trees.empty()) {
    // the starting points: x0, then nrestarts perturbed copies drawn start-major, then tree, then
    // constant (src/ConstantOptimization.jl:53-60: c * (1 + randn/2))
    // Float32 trees perturb in T as the reference does (node.val * (T(1) + T(1//2) * randn(T))):
    // a Float32 normal draw and Float32 arithmetic, the start rounded like the constant it replaces.
    // Caller-supplied starts (starts_in, [nrestarts][sum nconst]) replace the draws; a Float32
    // program rounds them to Float32.  Trees without constants or failing statically keep x0.
    std::vector<std::vector<double>> starts(opt->nrestarts + 1, x0);
    const bool f32 = P->dtype == SRHIP_F32;
    const int64_t nall = (int64_t)x0.size();
    for (int start = 1; start <= opt->nrestarts; ++start)
      for (int32_t t : trees)
        for (int64_t k = coff[t]; k < coff[t + 1]; ++k) {
          double xs;
          if (starts_in) {
            xs = starts_in[(int64_t)(start - 1) * nall + k];
          } else if (f32) {
            const float r = (float)randn(rng);
            xs = (double)((float)x0[k] * (1.0f + 0.5f * r));
          } else {
            xs = x0[k] * (1.0 + 0.5 * randn(rng));
          }
          starts[start][k] = f32 ? (double)(float)xs : xs;
        }
    if (starts_out)
      for (int start = 1; start <= opt->nrestarts; ++start)
        std::copy(starts[start].begin(), starts[start].end(), starts_out + (int64_t)(start - 1) * nall);
    const double tb = now_s();
    g_t_compile = g_t_eval = g_t_host = 0.0;
    g_patch_scan_s = g_patch_copy_s = 0.0;
    g_n_launch = 0;
    const char* te = getenv("SRHIP_OPTIM_TIMING");
    g_stats_on = te && (*te == '2' || *te == '3');
    g_launch_log = te && *te == '3';
    for (int64_t& h : g_hist) h = 0;
    g_nonfinite_trials = 0;
    g_spec_launched = g_spec_used = 0;
    for (auto& a : g_items)
      for (auto& b : a) b[0] = b[1] = 0;
    rc = optimize_split(ctx, ds, P, loss, v, trees, coff, opt->iterations, g_tol, starts, best_x, best_f, fcalls);
    if (g_stats_on)
      fprintf(stderr, "srhip optim (the caller's group: 1 of SRHIP_OPTIM_SPLIT groups): launches by active trees: "
              "1: %lld, 2-4: %lld, 5-16: %lld, 17-64: %lld, >64: %lld; "
              "non-finite trial points %lld; speculative points %lld evaluated, %lld used\n", (long long)g_hist[0],
              (long long)g_hist[1], (long long)g_hist[2], (long long)g_hist[3], (long long)g_hist[4],
              (long long)g_nonfinite_trials, (long long)g_spec_launched, (long long)g_spec_used);
    if (g_stats_on)
      fprintf(stderr, "srhip optim: items (all / non-finite f): gradient small %lld/%lld big %lld/%lld; value-only "
              "small %lld/%lld big %lld/%lld\n", (long long)g_items[0][0][0], (long long)g_items[0][0][1],
              (long long)g_items[0][1][0], (long long)g_items[0][1][1], (long long)g_items[1][0][0],
              (long long)g_items[1][0][1], (long long)g_items[1][1][0], (long long)g_items[1][1][1]);
    if (te && (*te == '1' || *te == '2' || *te == '3'))
      fprintf(stderr,
              "srhip optim: %.1f ms total (all groups), caller's group: %lld launches, eval_grad %.1f ms (compile/patch "
              "%.1f ms: scan+recompile %.1f, "
              "snapshot+upload %.1f), set_consts %.1f ms\n",
              1e3 * (now_s() - tb), (long long)g_n_launch, 1e3 * g_t_eval, 1e3 * g_t_compile, 1e3 * g_patch_scan_s,
              1e3 * g_patch_copy_s, 1e3 * g_t_host);
    if (rc) {
      set_all_consts(*P, x0.data());
      compile_program(*P);
      upload_program(*P);
      return rc;
    }
  } else if (starts_out) {
    for (int start = 1; start <= opt->nrestarts; ++start)
      std::copy(x0.begin(), x0.end(), starts_out + (int64_t)(start - 1) * (int64_t)x0.size());
  }
  // accept where the best minimum beats the baseline (:70-78)
  std::vector<double> final_x = x0;
  for (int32_t t = 0; t < nt; ++t) {
    const bool better = best_f[t] < base[t];
    out_improved[t] = better ? 1 : 0;
    if (better)
      for (int64_t k = coff[t]; k < coff[t + 1]; ++k) final_x[k] = best_x[k];
  }
  set_all_consts(*P, final_x.data());
  rc = compile_program(*P);
  if (rc) return rc;
  rc = upload_program(*P);
  if (rc) return rc;
  // the loss of the returned trees, by the evaluator (the reference re-scores accepted members)
  std::vector<uint8_t> ok(nt);
  rc = run_eval(ctx, ds, P, MODE_LOSS, loss, idx, nidx, out_loss, nullptr, ok.data());
  if (rc) return rc;
  // num_evals bookkeeping (src/ConstantOptimization.jl:51,65,79): the objective calls of every start
  // (result.f_calls), plus one for the re-score of an accepted tree; 0 for a tree left alone
  if (out_fcalls)
    for (int32_t t = 0; t < nt; ++t) out_fcalls[t] = fcalls[t] + out_improved[t];
  return SRHIP_OK;
}

int srhip_optimize_constants(srhip_ctx* ctx, const srhip_dataset* ds, srhip_program* P, const srhip_loss* loss,
                             const int64_t* idx, int64_t nidx, const srhip_optim_options* opt, double* out_loss,
                             uint8_t* out_improved, int64_t* out_fcalls) {
  return srhip_optimize_constants_starts(ctx, ds, P, loss, idx, nidx, opt, nullptr, nullptr, out_loss, out_improved,
                                         out_fcalls);
}

}  // extern "C"
