// srhip_host.cpp — host side of libsrhip.so: the tree compiler (Node{T} -> bytecode), device
// datasets, and the C ABI declared in include/srhip.h.
//
// The compiler restates, per tree, the host-decidable half of DynamicExpressions v0.16's
// eval_tree_array (external dependency; behaviour pinned by the reference's
// test/test_evaluation.jl, test/test_nan_detection.jl):
//   * constant subtrees are evaluated once as scalars (_eval_constant_tree): any non-finite
//     operator output => did_succeed = false; the folded value c is then a fill(c, n) array whose
//     isfinite(sum) is checked by its parent (or by the final root check);
//   * a non-finite constant leaf under a non-constant parent fails (@return_on_check);
//   * a feature leaf evaluated as a child array (child of a non-fused unary node, or the root)
//     gets its column's isfinite(sum) checked;
//   * every remaining operator node is emitted as bytecode; the device checks its outputs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sys/resource.h>
#include <sys/syscall.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/srhip.h"
#include "srhip_internal.h"
#include "srhip_isa.h"
#include "srhip_kernels.h"
#include "srhip_ops.h"

using namespace srhip;

static bool env_flag(const char* name);
static int env_int(const char* name, int dflt);

// ---------------------------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------------------------
static thread_local std::string g_err;

int srhip::fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
const char* srhip::last_error() { return g_err.c_str(); }

// Environment switches read per call (tests and the bench toggle them inside one process) through a
// per-thread cache: a getenv scans the whole environment (~1 us each, ~10 per evaluation); the cache
// is dropped whenever the environment's entry pointers change (every setenv / putenv / unsetenv
// replaces, adds or removes one), which a walk over those pointers detects in ~50 ns.
// (diagnostic) SRHIP_HOST_TIMING=1 timestamps: run_eval's wait and the end of eval_partials' tail
static thread_local std::chrono::steady_clock::time_point g_wait_begin, g_wait_done, g_tail_done;
extern "C" char** environ;
const char* srhip::env_get(const char* name) {
  struct Ent {
    const char* name;
    const char* val;
  };
  static thread_local uint64_t sig = 0;
  static thread_local std::vector<Ent> cache;
  uint64_t h = 1469598103934665603ull ^ (uint64_t)(uintptr_t)environ;
  for (char** e = environ; e && *e; ++e) h = (h ^ (uint64_t)(uintptr_t)*e) * 1099511628211ull;
  if (h != sig) {
    cache.clear();
    sig = h;
  }
  for (const Ent& c : cache)
    if (c.name == name || strcmp(c.name, name) == 0) return c.val;
  const char* v = getenv(name);
  cache.push_back(Ent{name, v});
  return v;
}

#ifndef SRHIP_COS_NC
// cos / sin of an operator output without their check fold (srhip_isa.h UN_NC_FLAG; 0: the checked form;
// C2 same box: 1.263 against 1.267 ms, profiles/r05_c2_scratch_g23/)
#define SRHIP_COS_NC 1
#endif

// ---------------------------------------------------------------------------------------------
// tree compiler
// ---------------------------------------------------------------------------------------------
namespace {

template <typename T> struct HostVal {
  static T from(double v) { return (T)v; }
  static uint64_t bits(T v) {
    if constexpr (sizeof(T) == 8) {
      uint64_t b;
      memcpy(&b, &v, 8);
      return b;
    } else {
      uint32_t b;
      memcpy(&b, &v, 4);
      return b;
    }
  }
};

static double op_cost(uint32_t h) {
  if (h == H_END) return 0.0;
  if (h < H_BIN0) return 1.0;
  if (h < H_HEAVY0) {
    const int sb = (h - H_BIN0) / SPEC_STRIDE;
    return sb == SB_DIV ? 10.0 : 2.0;
  }
  if (h < H_UN0) return 120.0;
  const int u = h - H_UN0;
  switch (u) {
    case UN_NEG: case UN_SQUARE: case UN_CUBE: case UN_ABS: case UN_RELU: case UN_SIGN:
    case UN_ROUND: case UN_FLOOR: case UN_CEIL:
      return 2.0;
    case UN_EXP: case UN_EXP2: case UN_SQRT: case UN_LOG: case UN_LOG2: case UN_LOG10:
      return 14.0;
    case UN_COS: case UN_SIN:
      return 30.0;
    default:
      return 60.0;
  }
}

template <typename T> class TreeCompiler {
 public:
  // grad = true: the constant-gradient program: constant subtrees are NOT folded (their
  // constants need tangents) and every constant leaf carries its get_constants index (0-based,
  // depth-first left-to-right) in the instruction's operand field.
  TreeCompiler(const srhip_node* nodes, int64_t nn, const srhip_program& prog, int nfeat_hint, bool grad = false)
      : nd_(nodes), nn_(nn), prog_(prog), nfeat_hint_(nfeat_hint), grad_(grad) {}
  // point a compiler (and its scratch vectors' capacity) at another tree
  void rebind(const srhip_node* nodes, int64_t nn) {
    nd_ = nodes;
    nn_ = nn;
    dmask_ = 0;
  }

  // returns SRHIP_OK or an error (g_err set); fills info and appends to code
  int compile(TreeInfo& info, std::vector<Ins>& code) { return compile_pair(info, code, nullptr, nullptr); }
  // The program of the tree (derived columns as set by set_derived) and, when dinfo is given, its
  // derived program too (derived columns dspec at dbase, set_derived's meaning) from the same
  // analysis: validation, counts, constant numbering and the host-decided checks do not depend on the
  // derived columns, so they run once.  Only code_begin / code_len / need / cost / static_fail of
  // *dinfo are filled (what a population's derived program keeps).
  int compile_pair(TreeInfo& info, std::vector<Ins>& code, TreeInfo* dinfo, std::vector<Ins>* dcode,
                   const std::vector<uint32_t>* dspec = nullptr, int dbase = 0) {
    info = TreeInfo();
    if (nn_ <= 0) return fail(SRHIP_ERR_INVALID, "empty tree");
    memo_const_.assign(nn_, -1);
    state_.assign(nn_, 0);
    int rc = validate(0, 0);
    if (rc) return rc;
    cidx_.assign(nn_, -1);
    tally(0, info);
    // host-decided checks (reference semantics, see header comment)
    static_checks(0, -1, info);
    if (std::is_same<T, float>::value && !grad_ && !info.static_fail) skip_bounds(info);
    rc = emit_program(info, code);
    if (rc || !dinfo) return rc;
    if (!grad_ && !reads_derived(dspec)) {
      // no U(X[f]) node of this tree is a derived column: the derived program is the plain one, byte
      // for byte (every emit decision is the same without a derived column), copied instead of emitted
      dinfo->static_fail = info.static_fail;
      dinfo->need = info.need;
      dinfo->cost = info.cost;
      dinfo->code_begin = (int32_t)dcode->size();
      dinfo->code_len = info.code_len;
      dcode->insert(dcode->end(), code.begin() + info.code_begin, code.begin() + info.code_begin + info.code_len);
      return SRHIP_OK;
    }
    const std::vector<uint32_t>* ds0 = dspec_;
    const int db0 = dbase_;
    set_derived(dspec, dbase);
    scratch_.op_sumcheck.clear();
    scratch_.static_fail = info.static_fail;
    scratch_.need = 0;
    scratch_.cost = 0.0;
    rc = emit_program(scratch_, *dcode);
    set_derived(ds0, db0);
    dinfo->static_fail = scratch_.static_fail;
    dinfo->need = scratch_.need;
    dinfo->cost = scratch_.cost;
    dinfo->code_begin = scratch_.code_begin;
    dinfo->code_len = scratch_.code_len;
    return rc;
  }

 private:
  const srhip_node* nd_;
  int64_t nn_;
  const srhip_program& prog_;
  int nfeat_hint_;
  bool grad_;
  std::vector<int32_t> cidx_;
  std::vector<int8_t> memo_const_;
  std::vector<int16_t> memo_need_;
  std::vector<int32_t> dcolv_;  // derived column per node, or -1
  std::vector<uint8_t> state_;
  std::vector<Ins>* code_ = nullptr;
  TreeInfo* info_ = nullptr;
  const std::vector<uint32_t>* dspec_ = nullptr;  // derived columns (nullptr: plain program)
  int dbase_ = 0;                                 // LDS column of derived column 0
  uint64_t dmask_ = 0;

 public:
  // compile U(X[f]) nodes listed in dspec as reads of LDS column dbase + d (srhip_isa.h)
  void set_derived(const std::vector<uint32_t>* dspec, int dbase) {
    dspec_ = dspec;
    dbase_ = dbase;
  }
  uint64_t dmask() const { return dmask_; }
  // does some U(X[f]) node of the tree read one of the derived columns dspec lists
  bool reads_derived(const std::vector<uint32_t>* dspec) const {
    if (!dspec || dspec->empty()) return false;
    for (int64_t i = 0; i < nn_; ++i) {
      const srhip_node& n = nd_[i];
      if (n.degree != 1 || !leaf_is_feature(n.l)) continue;
      const uint32_t key = ((uint32_t)classify_unop(unaop(i)) << 16) | (uint32_t)(nd_[n.l].feature - 1);
      for (uint32_t k : *dspec)
        if (k == key) return true;
    }
    return false;
  }
  // the value-dependent did_succeed metadata alone (static_fail, fill_consts, feat_checks) of a tree
  // compiled before with other constant values: the gradient program's code does not depend on them
  void static_info(TreeInfo& info) {
    info = TreeInfo();
    memo_const_.assign(nn_, -1);
    static_checks(0, -1, info);
  }

 private:
  TreeInfo scratch_;  // compile_pair's derived-program info (its op_sumcheck's capacity reused)

  // code for the analysed tree (validate, tally and static_checks done) under the current derived
  // columns, appended to code; fills info's need, cost, code_begin and code_len
  int emit_program(TreeInfo& info, std::vector<Ins>& code) {
    dcolv_.assign(dspec_ && !grad_ ? nn_ : 0, -1);
    for (int64_t i = 0; i < (int64_t)dcolv_.size(); ++i) {
      const srhip_node& n = nd_[i];
      if (n.degree != 1 || !leaf_is_feature(n.l)) continue;
      const uint32_t key = ((uint32_t)classify_unop(unaop(i)) << 16) | (uint32_t)(nd_[n.l].feature - 1);
      for (size_t d = 0; d < dspec_->size(); ++d)
        if ((*dspec_)[d] == key) dcolv_[i] = (int32_t)d;
    }
    memo_need_.assign(nn_, -1);
    info.code_begin = (int32_t)code.size();
    if (!info.static_fail) {
      info.need = need(0);
      if (info.need > K_MAX)
        return fail(SRHIP_ERR_UNSUPPORTED, "tree needs %d stack slots (> %d)", info.need, K_MAX);
      code_ = &code;
      info_ = &info;
      emit(0, 0, -1);
      if (super_ && (!grad_ || SRHIP_GRAD_SUPER_LEVEL >= 1)) fuse_push_loads(code, info.code_begin);
      Ins end{H_END, 0, 0};
      code.push_back(end);
      for (int64_t i = info.code_begin; i < (int64_t)code.size(); ++i) info.cost += op_cost(code[i].h);
    } else {
      Ins end{H_END, 0, 0};
      code.push_back(end);
    }
    info.code_len = (int32_t)code.size() - info.code_begin;
    return SRHIP_OK;
  }

  // one depth-first pass: node, operator-node and constant counts (count_nodes walks, shared
  // subtrees counted per use) and the get_constants numbering of the constant leaves
  void tally(int64_t i, TreeInfo& info) {
    const srhip_node& n = nd_[i];
    ++info.nnodes;
    if (n.degree == 0) {
      if (n.constant) cidx_[i] = info.nconst++;
      return;
    }
    ++info.nops;
    tally(n.l, info);
    if (n.degree == 2) tally(n.r, info);
  }

  int validate(int64_t i, int depth) {
    if (i < 0 || i >= nn_) return fail(SRHIP_ERR_INVALID, "child index %lld out of range", (long long)i);
    if (depth > 100000) return fail(SRHIP_ERR_INVALID, "tree too deep");
    if (state_[i] == 1) return fail(SRHIP_ERR_INVALID, "cycle in tree at node %lld", (long long)i);
    if (state_[i] == 2) return SRHIP_OK;  // shared subtree (GraphNode) already validated
    state_[i] = 1;
    const srhip_node& n = nd_[i];
    int rc = SRHIP_OK;
    if (n.degree == 0) {
      if (!n.constant) {
        if (n.feature < 1) rc = fail(SRHIP_ERR_INVALID, "feature index %d < 1", (int)n.feature);
        else if (nfeat_hint_ > 0 && n.feature > nfeat_hint_)
          rc = fail(SRHIP_ERR_INVALID, "feature index %d > nfeatures %d", (int)n.feature, nfeat_hint_);
      }
    } else if (n.degree == 1) {
      if (n.op < 1 || n.op > prog_.unaops.size())
        rc = fail(SRHIP_ERR_INVALID, "unary op index %d out of range", (int)n.op);
      else if (std::is_same<T, int32_t>::value && !int_unop_ok(unaop(i)))
        rc = fail(SRHIP_ERR_UNSUPPORTED, "unary op code %d is not defined for Int32", unaop(i));
      else rc = validate(n.l, depth + 1);
    } else if (n.degree == 2) {
      if (n.op < 1 || n.op > prog_.binops.size())
        rc = fail(SRHIP_ERR_INVALID, "binary op index %d out of range", (int)n.op);
      else if (std::is_same<T, int32_t>::value && !int_binop_ok(binop(i)))
        rc = fail(SRHIP_ERR_UNSUPPORTED, "binary op code %d is not defined for Int32", binop(i));
      else {
        rc = validate(n.l, depth + 1);
        if (!rc) rc = validate(n.r, depth + 1);
      }
    } else {
      rc = fail(SRHIP_ERR_INVALID, "bad degree %d", (int)n.degree);
    }
    state_[i] = 2;
    return rc;
  }

  bool is_const(int64_t i) {
    if (memo_const_[i] >= 0) return memo_const_[i];
    const srhip_node& n = nd_[i];
    bool c;
    if (n.degree == 0) c = n.constant;
    else if (n.degree == 1) c = is_const(n.l);
    else c = is_const(n.l) && is_const(n.r);
    memo_const_[i] = c;
    return c;
  }
  // Float32 evaluation programs fold no check statistic for + and -, nor for * by a constant
  // (srhip_eval_impl.h bin_rows_chk).  skip_bounds sets info.sb = (cM, cF, c0) with every such output
  // of the tree within cM M + cF F + c0,
  // M the tree's statistic of the folded values and F the features' max |x|: a folded operator output
  // is within M (a division the in-range path leaves unfolded is within 2^80: + 2^80), a cos / sin
  // within 1, a feature within F, a constant (subtree) its |value|, a +/- within the sum of its
  // operands' bounds and c * x within |c| times x's -- the reduction raises the statistic to that
  // bound, which only ever moves a tree
  // from decided to undecided (the precise pass then decides it exactly); never rounded down
  struct SkipB {
    double m = 0.0, f = 0.0, k = 0.0;
  };
  SkipB skip_bound(int64_t i, SkipB& mx) {
    SkipB b;
    const srhip_node& n = nd_[i];
    if (is_const(i)) {
      T v{};
      if (n.degree == 0) v = HostVal<T>::from(n.val);
      else eval_const(i, &v);
      const double a = fabs((double)v);
      b.k = a == a && a < INFINITY ? a : INFINITY;
      return b;
    }
    if (n.degree == 0) {
      b.f = 1.0;
      return b;
    }
    if (n.degree == 1) {
      (void)skip_bound(n.l, mx);
      const int u = classify_unop(unaop(i));
      if (u == UN_COS || u == UN_SIN) b.k = 1.0;
      else b.m = 1.0;
      return b;
    }
    const SkipB l = skip_bound(n.l, mx), r = skip_bound(n.r, mx);
    int sb, hb;
    classify_binop(binop(i), &sb, &hb);
    if (sb == SB_ADD || sb == SB_SUB) {
      b.m = l.m + r.m;
      b.f = l.f + r.f;
      b.k = l.k + r.k;
      mx.m = std::max(mx.m, b.m);
      mx.f = std::max(mx.f, b.f);
      mx.k = std::max(mx.k, b.k);
      return b;
    }
    if (sb == SB_MUL && (is_const(n.l) || is_const(n.r))) {
      // a product with a constant (the AC / CA / FC / CF forms): |c| times the other operand's bound,
      // never a zero factor -- 0 * Inf is NaN: an operand bound that is infinite (a non-finite feature)
      // must leave the product's bound infinite
      const SkipB& o = is_const(n.l) ? r : l;
      const double a = std::max(is_const(n.l) ? l.k : r.k, 0x1p-126);
      b.m = a * o.m;
      b.f = a * o.f;
      b.k = a * o.k;
      mx.m = std::max(mx.m, b.m);
      mx.f = std::max(mx.f, b.f);
      mx.k = std::max(mx.k, b.k);
      return b;
    }
    b.m = 1.0;
    if (sb == SB_DIV) b.k = 0x1p80;
    return b;
  }
  static float round_up_f(double x) {
    const float f = (float)x;
    return (double)f >= x ? f : std::nextafter(f, INFINITY);
  }
  void skip_bounds(TreeInfo& info) {
    SkipB mx;
    (void)skip_bound(0, mx);
    info.sb[0] = round_up_f(mx.m);
    info.sb[1] = round_up_f(mx.f);
    info.sb[2] = round_up_f(mx.k);
  }
  bool is_leaf(int64_t i) const { return nd_[i].degree == 0; }
  bool leafish(int64_t i) { return is_leaf(i) || (!grad_ && is_const(i)) || dcol(i) >= 0; }
  // derived column of node i (a listed U applied to a feature leaf), or -1
  int dcol(int64_t i) const { return dcolv_.empty() ? -1 : dcolv_[i]; }
  // column a leaf-like operand is read from (feature or derived), or -1 for constants
  int leaf_col(int64_t i) {
    if (leaf_is_feature(i)) return nd_[i].feature - 1;
    const int d = dcol(i);
    if (d < 0) return -1;
    dmask_ |= 1ull << d;
    return dbase_ + d;
  }
  // operand field of an instruction that consumes constant leaf i (gradient program only)
  uint32_t cop(int64_t i) const { return grad_ && cidx_[i] >= 0 ? (uint32_t)cidx_[i] : 0u; }
  int binop(int64_t i) const { return prog_.binops[nd_[i].op - 1]; }
  int unaop(int64_t i) const { return prog_.unaops[nd_[i].op - 1]; }

  // scalar semantics for constant folding (DynamicExpressions _eval_constant_tree)
  static T apply_bin(int code, T a, T b) {
    if constexpr (std::is_same<T, int32_t>::value) {
      switch (code) {
        case SRHIP_OP_ADD: return IOps::add(a, b);
        case SRHIP_OP_SUB: return IOps::sub(a, b);
        case SRHIP_OP_MUL: return IOps::mul(a, b);
        case SRHIP_OP_GREATER: return IOps::greater(a, b);
        case SRHIP_OP_COND: return IOps::cond(a, b);
        case SRHIP_OP_LOGICAL_OR: return IOps::logical_or(a, b);
        case SRHIP_OP_LOGICAL_AND: return IOps::logical_and(a, b);
        case SRHIP_OP_MAX: return IOps::max(a, b);
        case SRHIP_OP_MIN: return IOps::min(a, b);
        default: return 0;
      }
    } else {
      using O = FOps<T>;
      switch (code) {
#define X_(NAME, FN) case SRHIP_OP_##NAME: return O::FN(a, b);
        SRHIP_SPEC_BINOPS(X_)
        SRHIP_HEAVY_BINOPS(X_)
#undef X_
        default: return FP<T>::nan();
      }
    }
  }
  static T apply_un(int code, T a) {
    if constexpr (std::is_same<T, int32_t>::value) {
      switch (code) {
        case SRHIP_OP_NEG: return IOps::neg(a);
        case SRHIP_OP_SQUARE: return IOps::square(a);
        case SRHIP_OP_CUBE: return IOps::cube(a);
        case SRHIP_OP_ABS: return IOps::abs(a);
        case SRHIP_OP_RELU: return IOps::relu(a);
        case SRHIP_OP_SIGN: return IOps::sign(a);
        default: return 0;
      }
    } else {
      using O = FOps<T>;
      switch (code) {
#define X_(NAME, FN) case SRHIP_OP_##NAME: return O::FN(a);
        SRHIP_UNOPS(X_)
#undef X_
        default: return FP<T>::nan();
      }
    }
  }
  // returns ok; value in *v
  bool eval_const(int64_t i, T* v) {
    const srhip_node& n = nd_[i];
    if (n.degree == 0) {  // deg0_eval_constant: no check on the leaf itself
      *v = HostVal<T>::from(n.val);
      return true;
    }
    if (n.degree == 1) {
      T a;
      if (!eval_const(n.l, &a)) return false;
      *v = apply_un(unaop(i), a);
      return m_isfinite(*v);
    }
    T a, b;
    if (!eval_const(n.l, &a)) return false;
    if (!eval_const(n.r, &b)) return false;
    *v = apply_bin(binop(i), a, b);
    return m_isfinite(*v);
  }

  // Reference fusion: node C is evaluated inline (per element, no isfinite(sum)) by its deg-1
  // parent in DynamicExpressions' deg1_l2_ll0_lr0 / deg1_l1_ll0 kernels.
  bool fused_inner(int64_t c, int64_t parent) const {
    if (parent < 0 || nd_[parent].degree != 1) return false;
    const srhip_node& n = nd_[c];
    if (n.degree == 2) return is_leaf(n.l) && is_leaf(n.r);
    if (n.degree == 1) return is_leaf(n.l);
    return false;
  }

  void static_checks(int64_t i, int64_t parent, TreeInfo& info) {
    const srhip_node& n = nd_[i];
    const bool root = parent < 0;
    if (is_const(i)) {
      // constant subtree (or constant leaf): scalar path, fill(c, n) array then checked
      if (n.degree == 0) {
        if (root) info.fill_consts.push_back(n.val);
        else if (!m_isfinite(HostVal<T>::from(n.val))) info.static_fail = true;  // @return_on_check
        return;
      }
      T v;
      if (!eval_const(i, &v)) {
        info.static_fail = true;
        return;
      }
      info.fill_consts.push_back((double)v);
      return;
    }
    if (n.degree == 0) {  // feature leaf
      if (root) info.feat_checks.push_back(n.feature - 1);
      return;
    }
    if (n.degree == 1) {
      const int64_t c = n.l;
      // a feature leaf under a non-fused unary node is evaluated as an array and checked
      if (is_leaf(c) && !nd_[c].constant && !fused_inner(i, parent)) info.feat_checks.push_back(nd_[c].feature - 1);
      static_checks(c, i, info);
      return;
    }
    static_checks(n.l, i, info);
    static_checks(n.r, i, info);
  }

  int need(int64_t i) {
    if (memo_need_[i] < 0) memo_need_[i] = (int16_t)need_(i);
    return memo_need_[i];
  }
  int need_(int64_t i) {
    if (leafish(i)) return 0;
    const srhip_node& n = nd_[i];
    if (n.degree == 1) return need(n.l);
    const bool ll = leafish(n.l), rl = leafish(n.r);
    int sb, hb;
    classify_binop(binop(i), &sb, &hb);
    const int leaf_slot = hb >= 0 ? 1 : 0;  // a heavy op's leaf operand is loaded into a slot
    if (ll && rl) return leaf_slot;
    if (rl) return std::max(need(n.l), leaf_slot);
    if (ll) return std::max(need(n.r), leaf_slot);
    const int a = need(n.l), b = need(n.r);
    return a == b ? a + 1 : std::max(a, b);
  }

  void push_ins(uint32_t h, uint32_t a, uint64_t imm) { code_->push_back(Ins{h, a, imm}); }
  // operator instruction: a = (op ordinal + 1) << 16 | operand -- or, in a gradient program's
  // leaf-constant superinstructions (FC / CF), hi = the constant's index in the upper half (the
  // interpreter's precise pass counts operator ordinals in execution order: srhip_eval_impl.h
  // precise_hook; only a derived-column load needs its ordinal field, to mark it an operator)
  void push_op(uint32_t h, uint32_t operand, uint64_t imm, int64_t node, int64_t parent, int64_t hi = -1) {
    // the gradient program evaluates constant subtrees per row (their constants need tangents); the
    // reference evaluates them as scalars (_eval_constant_tree): finiteness only, no isfinite(sum)
    const bool scalar = grad_ && is_const(node);
    info_->op_sumcheck.push_back((!scalar && (parent < 0 || !fused_inner(node, parent))) ? 1 : 0);
    const uint32_t ord = (uint32_t)info_->op_sumcheck.size();
    push_ins(h, ((hi >= 0 ? (uint32_t)hi : ord) << 16) | (operand & 0xffff), imm);
  }
  uint64_t leaf_imm(int64_t i) {
    if (nd_[i].degree == 0) return HostVal<T>::bits(HostVal<T>::from(nd_[i].val));
    T v;
    eval_const(i, &v);  // folded constant subtree (ok: checked in static_checks)
    return HostVal<T>::bits(v);
  }
  bool leaf_is_feature(int64_t i) const { return nd_[i].degree == 0 && !nd_[i].constant; }

  // Superinstructions (SRHIP_NO_SUPER=1 turns them off; gradient programs as far as the build's
  // SRHIP_GRAD_SUPER_LEVEL allows -- none by default -- and SRHIP_GRAD_NO_SUPER=1 turns those off): the
  // leaf-leaf operand forms (emit) and a push fused with the leaf load that
  // follows it: one dispatch instead of two.  In a gradient program a leaf-constant form carries the
  // constant's index in its upper half (push_op's hi) and a push fuses with a plain feature or constant
  // load only (a derived-column load is an operator of its own).
  const bool super_ = grad_ ? grad_super_env() : super_env();

 public:
  static bool super_env() {
    const char* e = env_get("SRHIP_NO_SUPER");
    return !(e && *e && *e != '0');
  }
  static bool grad_super_env() {
    const char* e = env_get("SRHIP_GRAD_NO_SUPER");
    return super_env() && !(e && *e && *e != '0');
  }
  static bool grad_uniform_env() {
    const char* e = env_get("SRHIP_GRAD_UNIFORM");
    return !(e && *e == '0');
  }

 private:
  static void fuse_push_loads(std::vector<Ins>& code, int32_t begin) {
    size_t w = (size_t)begin;
    for (size_t r = (size_t)begin; r < code.size(); ++r) {
      const Ins& a = code[r];
      if (a.h >= H_PUSH0 && a.h < H_PUSH0 + K_MAX && r + 1 < code.size() &&
          ((code[r + 1].h == H_LOADF && (code[r + 1].a >> 16) == 0) || code[r + 1].h == H_LOADC)) {
        const Ins& b = code[r + 1];
        const uint32_t k = a.h - H_PUSH0;
        code[w++] = Ins{(b.h == H_LOADF ? H_PUSHLF0 : H_PUSHLC0) + k, b.a, b.imm};
        ++r;
        continue;
      }
      code[w++] = a;
    }
    code.resize(w);
  }

  void emit_leaf(int64_t i) {
    const int col = leaf_col(i);
    if (col >= 0) push_ins(H_LOADF, (uint32_t)col, 0);
    else push_ins(H_LOADC, cop(i), leaf_imm(i));
  }

  void emit(int64_t i, int base, int64_t parent) {
    if (leafish(i)) {
      emit_leaf(i);
      return;
    }
    const srhip_node& n = nd_[i];
    if (n.degree == 1) {
      if (grad_ && prog_.g_want_derived && leaf_is_feature(n.l)) {
        // a heavy operator of a feature in a constant-gradient program: its derived column (the
        // operator's value, no tangent), loaded with the operator's own ordinal -- its check fold and
        // precise sum stay where the operator's were
        const int u = classify_unop(unaop(i));
        const uint32_t key = (uint32_t)u << 16 | (uint32_t)leaf_col(n.l);
        for (size_t j = 0; j < prog_.gdspec.size(); ++j)
          if (prog_.gdspec[j] == key) {
            push_op(H_LOADF, (uint32_t)(prog_.gdbase + (int)j), 0, i, parent);
            return;
          }
      }
      emit(n.l, base, i);
      const int u = classify_unop(unaop(i));
      // cos / sin of an operator output need no check fold of their own (srhip_isa.h UN_NC_FLAG); the
      // gradient program keeps every fold
      const bool nc = SRHIP_COS_NC && !grad_ && !leafish(n.l) && (u == UN_COS || u == UN_SIN);
      // gradient programs: an operator of a constant subtree (one value on every row) is evaluated
      // once per lane (SRHIP_GRAD_UNIFORM=0: per row)
      const bool uni = grad_ && is_const(n.l) && grad_uniform_env();
      push_op(h_un(u), (nc ? UN_NC_FLAG : 0) | (uni ? UN_UNIFORM_FLAG : 0), 0, i, parent);
      return;
    }
    int sb, hb;
    classify_binop(binop(i), &sb, &hb);
    const int64_t L = n.l, Rr = n.r;
    const bool ll = leafish(L), rl = leafish(Rr);
    if (sb >= 0) {
      // (a gradient program's two constant leaves keep the uniform constant form below)
      if (ll && rl && super_ && (!grad_ || SRHIP_GRAD_SUPER_LEVEL >= 2) && (leaf_col(L) >= 0 || leaf_col(Rr) >= 0)) {
        // deg2_l0_r0: both operands leaves (feature, derived column or constant) in one instruction
        const int cl = leaf_col(L), cr = leaf_col(Rr);
        if (cl >= 0 && cr >= 0) push_op(h_spec(sb, SPEC_FF), cl, (uint64_t)cr, i, parent);
        else if (cl >= 0) push_op(h_spec(sb, SPEC_FC), cl, leaf_imm(Rr), i, parent, grad_ ? (int64_t)cop(Rr) : -1);
        else push_op(h_spec(sb, SPEC_CF), cr, leaf_imm(L), i, parent, grad_ ? (int64_t)cop(L) : -1);
        return;
      }
      // gradient programs: an operator of two constant subtrees (one value on every row) is evaluated
      // once per lane (the forms whose operand field is a constant index or unused)
      const uint32_t uni = grad_ && is_const(i) && grad_uniform_env() ? UN_UNIFORM_FLAG : 0u;
      if (rl) {
        emit(L, base, i);
        if (leaf_col(Rr) >= 0) push_op(h_spec(sb, SPEC_AF), leaf_col(Rr), 0, i, parent);
        else push_op(h_spec(sb, SPEC_AC), cop(Rr) | uni, leaf_imm(Rr), i, parent);
      } else if (ll) {
        emit(Rr, base, i);
        if (leaf_col(L) >= 0) push_op(h_spec(sb, SPEC_FA), leaf_col(L), 0, i, parent);
        else push_op(h_spec(sb, SPEC_CA), cop(L) | uni, leaf_imm(L), i, parent);
      } else if (need(L) >= need(Rr)) {
        emit(L, base, i);
        push_ins(H_PUSH0 + base, 0, 0);
        emit(Rr, base + 1, i);
        push_op(h_spec(sb, SPEC_SA0 + base), uni, 0, i, parent);
      } else {
        emit(Rr, base, i);
        push_ins(H_PUSH0 + base, 0, 0);
        emit(L, base + 1, i);
        push_op(h_spec(sb, SPEC_AS0 + base), uni, 0, i, parent);
      }
      return;
    }
    // heavy binary op (pow, mod, atan2): the second operand lives in stack slot `base`
    if (rl) {
      emit(L, base, i);
      if (leaf_col(Rr) >= 0) push_ins(H_SLOADF0 + base, leaf_col(Rr), 0);
      else push_ins(H_SLOADC0 + base, cop(Rr), leaf_imm(Rr));
      push_op(h_heavy(hb, HEAVY_AS0 + base), 0, 0, i, parent);  // A = A op S[base]
    } else if (ll) {
      emit(Rr, base, i);
      if (leaf_col(L) >= 0) push_ins(H_SLOADF0 + base, leaf_col(L), 0);
      else push_ins(H_SLOADC0 + base, cop(L), leaf_imm(L));
      push_op(h_heavy(hb, HEAVY_SA0 + base), 0, 0, i, parent);  // A = S[base] op A
    } else if (need(L) >= need(Rr)) {
      emit(L, base, i);
      push_ins(H_PUSH0 + base, 0, 0);
      emit(Rr, base + 1, i);
      push_op(h_heavy(hb, HEAVY_SA0 + base), 0, 0, i, parent);  // A = S op A
    } else {
      emit(Rr, base, i);
      push_ins(H_PUSH0 + base, 0, 0);
      emit(L, base + 1, i);
      push_op(h_heavy(hb, HEAVY_AS0 + base), 0, 0, i, parent);  // A = A op S
    }
  }
};

// Host worker threads for the compiler: created once per process (a fork child makes its own) and
// parked on a condition variable between jobs, so a population compile pays no thread start-up.
// One job at a time; a caller that finds the pool busy (concurrent coalescer flushes) runs its items
// itself.  The process's pool is never destroyed: detached workers parked at exit are simply ended.
// Work items are claimed from one 64-bit counter holding (job generation << 32 | next index): a
// worker snapshots (generation, fn, n) under the mutex when it wakes, and a claim succeeds only by a
// compare-exchange on its own generation, so a worker delayed past the end of its job can never run
// an item of the next one (nor count it done).
class HostPool {
 public:
  static HostPool& get() {
    // lock-free, so that a fork taken while another thread is here cannot leave a held mutex behind;
    // the loser of a creation race shuts its own pool down (joins its threads) and deletes it
    static std::atomic<HostPool*> pool{nullptr};
    HostPool* p = pool.load();
    if (!p || p->pid_ != getpid()) {
      HostPool* q = new HostPool();
      if (pool.compare_exchange_strong(p, q)) {
        p = q;
      } else {
        q->shutdown();
        delete q;
      }
    }
    return *p;
  }
  int threads() const { return (int)nthr_ + 1; }
  // fn(0) .. fn(n - 1) on the pool's threads and the caller; false (nothing run) if busy
  bool run(int n, const std::function<void(int)>& fn) {
    std::unique_lock<std::mutex> busy(busy_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    uint32_t g;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      done_ = 0;
      g = ++gen_;
      next_.store((uint64_t)g << 32);
    }
    cv_.notify_all();
    work(g, &fn, n);
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [&] { return done_ == n_; });
    fn_ = nullptr;
    return true;
  }

 private:
  HostPool() : pid_(getpid()) {
    // up to 15 workers + the caller: the CPU share a GPU process gets on the MI355X boxes (16);
    // hardware_concurrency there reports the whole machine
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    nthr_ = std::min(15u, hw - 1);
    // SRHIP_POOL_NICE = n > 0: the workers run at nice n, so a thread that is waiting for the device
    // (an evaluation beside a pipelined compile) gets its core back first when the device finishes
    const char* ne = getenv("SRHIP_POOL_NICE");
    const int nice_v = ne && *ne ? atoi(ne) : 0;
    for (unsigned i = 0; i < nthr_; ++i)
      threads_.emplace_back([this, nice_v] {
        if (nice_v > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice_v);
        loop();
      });
  }
  ~HostPool() {
    for (std::thread& t : threads_)
      if (t.joinable()) t.detach();
  }
  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (std::thread& t : threads_)
      if (t.joinable()) t.join();
  }
  void loop() {
    uint32_t seen = 0;
    for (;;) {
      uint32_t g;
      const std::function<void(int)>* fn;
      int n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = g = gen_;
        fn = fn_;
        n = n_;
      }
      if (fn) work(g, fn, n);
    }
  }
  void work(uint32_t g, const std::function<void(int)>* fn, int n) {
    for (;;) {
      uint64_t v = next_.load();
      if ((uint32_t)(v >> 32) != g || (int)(uint32_t)v >= n) return;
      if (!next_.compare_exchange_weak(v, v + 1)) continue;
      (*fn)((int)(uint32_t)v);
      std::lock_guard<std::mutex> lk(mu_);
      if (++done_ == n_) cv_done_.notify_all();
    }
  }
  const pid_t pid_;
  unsigned nthr_ = 0;
  std::vector<std::thread> threads_;
  std::mutex busy_mu_, mu_;
  std::condition_variable cv_, cv_done_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, done_ = 0;
  bool stop_ = false;
  std::atomic<uint64_t> next_{0};
  uint32_t gen_ = 0;
};

// Per-tree code cache: a tree's compiled code and metadata depend only on its node table (constant
// values included: folded constants are immediates), the operator tables and the element type, and
// its derived-program code also on which derived column each of its U(X[f]) nodes reads and where the
// derived columns start (the population's feature count).  Entries are keyed by a hash of the node
// bytes and operator tables and confirmed by comparing them in full, so a hit returns exactly the
// bytes a compile would produce.  Sharded by hash; a shard that grows past its share of
// CODE_CACHE_ENTRIES is emptied (the cache holds recent trees: the search's survivors, migrants and
// re-scored members).  SRHIP_NO_CODE_CACHE=1 bypasses it (read per compile).
// Entries are made on a tree's SECOND sighting: the first only records its hash in a lossy
// direct-mapped table of the shard (one 8-byte store), so a population of new trees -- every tree
// of a fresh population misses -- does not pay for copying ~10 vectors per tree into entries it will
// never hit (C2's 1024-tree compile, one thread: 7.6 -> ~4.6 ms).  A tree that recurs (survivors,
// migrants, re-scored members) is cached from its second compile and hits from its third.
// SRHIP_CODE_CACHE_EAGER=1 makes entries on the first sighting (read per compile).
constexpr int CODE_CACHE_SHARDS = 64;
constexpr size_t CODE_CACHE_ENTRIES = 1 << 15;
constexpr size_t CODE_CACHE_SEEN = 1 << 12;  // first-sighting hashes per shard
std::atomic<int64_t> g_cache_hits{0}, g_cache_misses{0}, g_cache_inserts{0};

inline uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}
inline uint64_t hash_words(const void* p, size_t bytes, uint64_t h) {
  const unsigned char* c = (const unsigned char*)p;
  size_t i = 0;
  for (; i + 8 <= bytes; i += 8) {
    uint64_t w;
    memcpy(&w, c + i, 8);
    h = mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
  }
  for (; i < bytes; ++i) h = mix64(h ^ c[i]);
  return h;
}
inline uint64_t ops_hash(const srhip_program& P) {
  uint64_t h = hash_words(P.binops.data(), P.binops.size() * 4, 0x5eed ^ P.binops.size());
  return hash_words(P.unaops.data(), P.unaops.size() * 4, h ^ (P.unaops.size() << 20));
}

template <typename T> class CodeCache {
 public:
  struct Derived {
    int32_t dbase = -1;
    std::vector<int32_t> dsig;  // derived column of each U(X[f]) node, in node order (-1: none)
    std::vector<Ins> code;
    TreeInfo info;              // need, cost, code_len, static_fail
    uint64_t dmask = 0;
  };
  static CodeCache& get() {
    static CodeCache* c = new CodeCache();  // never destroyed (worker threads may outlive statics)
    return *c;
  }
  static bool enabled() {
    const char* e = env_get("SRHIP_NO_CODE_CACHE");
    return !(e && *e && *e != '0');
  }
  // derived column per U(X[f]) node of a valid tree (as TreeCompiler::emit_program assigns them)
  static void derived_sig(const srhip_node* nd, int64_t nn, const srhip_program& P, std::vector<int32_t>& sig) {
    sig.clear();
    for (int64_t i = 0; i < nn; ++i) {
      const srhip_node& n = nd[i];
      if (n.degree != 1 || nd[n.l].degree != 0 || nd[n.l].constant) continue;
      const uint32_t key = ((uint32_t)classify_unop(P.unaops[n.op - 1]) << 16) | (uint32_t)(nd[n.l].feature - 1);
      int32_t d = -1;
      for (size_t k = 0; k < P.dspec.size(); ++k)
        if (P.dspec[k] == key) d = (int32_t)k;
      sig.push_back(d);
    }
  }
  // On a hit, appends the plain code to code (and, with dcode, the derived code to dcode) exactly as
  // TreeCompiler::compile / compile_pair would, fills info / *dinfo / *dmask and returns true.
  // Returns LOOKUP_HIT (filled), LOOKUP_SEEN (a miss whose hash was seen before: compile and insert)
  // or LOOKUP_NEW (a first sighting, now recorded: compile, do not insert unless eager).
  enum { LOOKUP_NEW = 0, LOOKUP_HIT = 1, LOOKUP_SEEN = 2 };
  int lookup(uint64_t h, const srhip_node* nd, int64_t nn, const srhip_program& P, bool sup, TreeInfo& info,
             std::vector<Ins>& code, TreeInfo* dinfo, std::vector<Ins>* dcode, uint64_t* dmask,
             std::vector<int32_t>& sig) {
    Shard& s = shards_[h % CODE_CACHE_SHARDS];
    std::lock_guard<std::mutex> lk(s.mu);
    auto it = s.map.find(h);
    if (it == s.map.end()) {
      const uint64_t hk = h ? h : 1;  // 0 marks an empty slot
      uint64_t& slot = s.seen[(h / CODE_CACHE_SHARDS) % CODE_CACHE_SEEN];
      if (slot == hk) return LOOKUP_SEEN;
      slot = hk;
      return LOOKUP_NEW;
    }
    const Entry& e = it->second;
    if (!same(e, nd, nn, P, sup)) return LOOKUP_SEEN;  // a hash collision with a cached tree
    if (dinfo) {
      derived_sig(nd, nn, P, sig);
      if (!e.d || e.d->dbase != P.maxfeat || e.d->dsig != sig) return LOOKUP_SEEN;
      dinfo->static_fail = e.d->info.static_fail;
      dinfo->need = e.d->info.need;
      dinfo->cost = e.d->info.cost;
      dinfo->code_len = e.d->info.code_len;
      dinfo->code_begin = (int32_t)dcode->size();
      dcode->insert(dcode->end(), e.d->code.begin(), e.d->code.end());
      *dmask = e.d->dmask;
    }
    info = e.info;
    info.code_begin = (int32_t)code.size();
    code.insert(code.end(), e.code.begin(), e.code.end());
    return LOOKUP_HIT;
  }
  void insert(uint64_t h, const srhip_node* nd, int64_t nn, const srhip_program& P, bool sup, const TreeInfo& info,
              const Ins* code, const TreeInfo* dinfo, const Ins* dcode, uint64_t dmask) {
    Entry e;
    e.nodes.assign(nd, nd + nn);
    e.binops = P.binops;
    e.unaops = P.unaops;
    e.super = sup;
    e.info = info;
    e.code.assign(code, code + info.code_len);
    if (dinfo) {
      e.d.reset(new Derived());
      e.d->dbase = P.maxfeat;
      derived_sig(nd, nn, P, e.d->dsig);
      e.d->info.static_fail = dinfo->static_fail;
      e.d->info.need = dinfo->need;
      e.d->info.cost = dinfo->cost;
      e.d->info.code_len = dinfo->code_len;
      e.d->code.assign(dcode, dcode + dinfo->code_len);
      e.d->dmask = dmask;
    }
    Shard& s = shards_[h % CODE_CACHE_SHARDS];
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.map.size() >= CODE_CACHE_ENTRIES / CODE_CACHE_SHARDS) s.map.clear();
    s.map[h] = std::move(e);
  }

 private:
  struct Entry {
    std::vector<srhip_node> nodes;
    std::vector<int32_t> binops, unaops;
    bool super = true;  // compiled with superinstructions (SRHIP_NO_SUPER unset)
    TreeInfo info;
    std::vector<Ins> code;
    std::unique_ptr<Derived> d;
  };
  struct Shard {
    std::mutex mu;
    std::unordered_map<uint64_t, Entry> map;
    std::vector<uint64_t> seen = std::vector<uint64_t>(CODE_CACHE_SEEN, 0);
  };
  static bool same(const Entry& e, const srhip_node* nd, int64_t nn, const srhip_program& P, bool sup) {
    return e.super == sup && (int64_t)e.nodes.size() == nn && memcmp(e.nodes.data(), nd, (size_t)nn * sizeof(srhip_node)) == 0 &&
           e.binops == P.binops && e.unaops == P.unaops;
  }
  Shard shards_[CODE_CACHE_SHARDS];
};

// The population's programs in one pass over the trees: the plain program and, when the population
// has derived columns (srhip_isa.h), the derived program, compiled tree by tree on the host pool
// (contiguous tree ranges; per-range code vectors concatenated in tree order: the same bytes as one
// sequential pass).  Derived columns: the heavy U(X[f]) nodes of the population's trees are counted
// first, the pairs used at least DERIVE_MIN_USES times kept (most used first, at most DERIVE_MAX).
// SRHIP_NO_DERIVE=1 disables them.
template <typename T>
void choose_derived_t(srhip_program& P) {
  P.dspec.clear();
  const char* env = env_get("SRHIP_NO_DERIVE");
  const bool off = env && *env && *env != '0';
  if (std::is_same<T, int32_t>::value || off) return;
  std::vector<std::pair<uint32_t, int>> cnt;  // (key, uses), in order of first use
  // uses counted in a dense (unary class, feature) table when it is small, else by search in cnt
  const int64_t nf = std::max<int32_t>(P.maxfeat, 1);
  const bool dense = (int64_t)NUM_UNOP * nf <= (1 << 16);
  std::vector<int32_t> slot(dense ? (size_t)(NUM_UNOP * nf) : 0, -1);  // index into cnt
  for (int32_t t = 0; t < P.ntrees; ++t) {
    // node tables are per tree with tree-relative child indices
    const int64_t b = P.offsets[t], e = P.offsets[t + 1];
    for (int64_t i = b; i < e; ++i) {
      const srhip_node& n = P.nodes[i];
      if (n.degree != 1) continue;
      // (this pass runs before the trees are validated: a malformed child or operator index is
      // skipped here and rejected by the compiler's validation with SRHIP_ERR_INVALID)
      if (n.l < 0 || n.l >= e - b) continue;
      if (n.op < 1 || (size_t)n.op > P.unaops.size()) continue;
      const srhip_node& c = P.nodes[b + n.l];
      if (c.degree != 0 || c.constant || c.feature < 1) continue;
      const int u = classify_unop(P.unaops[n.op - 1]);
      if (!un_derivable(u)) continue;
      const uint32_t key = ((uint32_t)u << 16) | (uint32_t)(c.feature - 1);
      int32_t* sl = dense && c.feature <= nf ? &slot[(size_t)u * nf + (c.feature - 1)] : nullptr;
      int32_t k = sl ? *sl : -1;
      if (!sl) {
        auto it = std::find_if(cnt.begin(), cnt.end(), [&](const std::pair<uint32_t, int>& q) { return q.first == key; });
        if (it != cnt.end()) k = (int32_t)(it - cnt.begin());
      }
      if (k < 0) {
        k = (int32_t)cnt.size();
        cnt.emplace_back(key, 0);
        if (sl) *sl = k;
      }
      ++cnt[k].second;
    }
  }
  std::stable_sort(cnt.begin(), cnt.end(), [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) {
    return a.second > b.second;
  });
  static const int dmax_env = [] { const char* e = getenv("SRHIP_DERIVE_MAX"); return e ? atoi(e) : -1; }();
  const int dmax = dmax_env >= 0 ? std::min(dmax_env, DERIVE_MAX) : DERIVE_MAX;
  for (const auto& e : cnt)
    if (e.second >= DERIVE_MIN_USES && (int)P.dspec.size() < dmax) P.dspec.push_back(e.first);
}

static TreeDecide make_decide(const TreeInfo& I) {
  TreeDecide d;
  for (double c : I.fill_consts)
    if (!std::isnan(c)) d.maxc = std::max(d.maxc, fabs(c));
  for (int f : I.feat_checks) {
    if (f >= 0 && f < 64) d.feat_mask |= (uint64_t)1 << f;
    else d.slow = 1;
  }
  d.nnodes = I.nnodes;
  d.nops = I.nops;
  d.static_fail = I.static_fail;
  d.has_op = !I.op_sumcheck.empty();
  return d;
}
template <typename T>
int compile_program_t(srhip_program& P) {
  const int32_t n = P.ntrees;
  P.code.clear();
  P.prog_off.assign(n, 0);
  P.info.assign(n, TreeInfo());
  P.kmax = 0;
  P.max_ops = 0;
  P.max_len = 0;
  P.total_nodes = 0;
  P.total_ops = 0;
  P.dmask.assign(n, 0);
  P.dcode.clear();
  P.dprog_off.assign(n, 0);
  P.dcost.assign(n, 0.0);
  P.dec.assign(n, TreeDecide());
  P.sbound.clear();
  P.dkmax = P.dmax_len = 0;
  // operator-node count and the largest feature index, from the node tables
  P.maxfeat = 0;
  for (const srhip_node& nd : P.nodes) {
    P.total_ops += nd.degree > 0;
    if (nd.degree == 0 && !nd.constant) P.maxfeat = std::max<int32_t>(P.maxfeat, nd.feature);
  }
  choose_derived_t<T>(P);
  const bool der = !P.dspec.empty();
  std::vector<TreeInfo> dinfo(der ? n : 0);
  HostPool& pool = HostPool::get();
  // SRHIP_COMPILE_THREADS caps the threads one compile uses (read per compile; default: the pool)
  const int cap_env = env_int("SRHIP_COMPILE_THREADS", 0);
  const int wmax = cap_env > 0 ? std::min(cap_env, pool.threads()) : pool.threads();
  const int W = (int)std::max<int64_t>(1, std::min<int64_t>(wmax, (int64_t)n / 64));
  std::vector<std::vector<Ins>> part(W), dpart(W);
  std::vector<std::string> errs(W);
  std::vector<int> rcs(W, SRHIP_OK);
  CodeCache<T>* cache = CodeCache<T>::enabled() ? &CodeCache<T>::get() : nullptr;
  const bool sup = TreeCompiler<T>::super_env();
  const uint64_t oph = cache ? ops_hash(P) ^ (sup ? 0x5u : 0u) : 0;
  const bool eager = env_flag("SRHIP_CODE_CACHE_EAGER");
  const std::function<void(int)> range = [&](int w) {
    const int32_t t0 = (int32_t)((int64_t)n * w / W), t1 = (int32_t)((int64_t)n * (w + 1) / W);
    TreeCompiler<T> tc(nullptr, 0, P, 0);
    std::vector<int32_t> sig;
    int64_t nhit = 0, nmiss = 0, nins = 0;
    struct Count {  // the range's cache counters, added once at its end
      int64_t &a, &b, &c;
      ~Count() {
        g_cache_hits += a;
        g_cache_misses += b;
        g_cache_inserts += c;
      }
    } count{nhit, nmiss, nins};
    for (int32_t t = t0; t < t1 && !rcs[w]; ++t) {
      const int64_t b = P.offsets[t], e = P.offsets[t + 1];
      const srhip_node* tn = P.nodes.data() + b;
      uint64_t h = 0;
      bool keep = false;  // make a cache entry of this compile
      if (cache) {
        h = hash_words(tn, (size_t)(e - b) * sizeof(srhip_node), oph ^ (uint64_t)(e - b));
        const int lk = cache->lookup(h, tn, e - b, P, sup, P.info[t], part[w], der ? &dinfo[t] : nullptr,
                                     der ? &dpart[w] : nullptr, &P.dmask[t], sig);
        if (lk == CodeCache<T>::LOOKUP_HIT) {
          ++nhit;
          continue;
        }
        ++nmiss;
        keep = eager || lk == CodeCache<T>::LOOKUP_SEEN;
      }
      tc.rebind(tn, e - b);
      const int rc = der ? tc.compile_pair(P.info[t], part[w], &dinfo[t], &dpart[w], &P.dspec, P.maxfeat)
                         : tc.compile(P.info[t], part[w]);
      if (!rc && der) P.dmask[t] = tc.dmask();
      if (!rc && keep && cache) {
        ++nins;
        cache->insert(h, tn, e - b, P, sup, P.info[t], part[w].data() + P.info[t].code_begin, der ? &dinfo[t] : nullptr,
                      der ? dpart[w].data() + dinfo[t].code_begin : nullptr, P.dmask[t]);
      }
      if (rc) {
        errs[w] = "tree " + std::to_string(t) + ": " + g_err;
        rcs[w] = rc;
      }
    }
  };
  if (W == 1 || !pool.run(W, range))
    for (int w = 0; w < W; ++w) range(w);
  for (int w = 0; w < W; ++w)
    if (rcs[w]) return fail(rcs[w], "%s", errs[w].c_str());
  for (int w = 0; w < W; ++w) {
    const int32_t t0 = (int32_t)((int64_t)n * w / W), t1 = (int32_t)((int64_t)n * (w + 1) / W);
    const int32_t base = (int32_t)P.code.size(), dbase = (int32_t)P.dcode.size();
    for (int32_t t = t0; t < t1; ++t) {
      P.info[t].code_begin += base;
      if (der) dinfo[t].code_begin += dbase;
    }
    P.code.insert(P.code.end(), part[w].begin(), part[w].end());
    if (der) P.dcode.insert(P.dcode.end(), dpart[w].begin(), dpart[w].end());
  }
  for (int32_t t = 0; t < n; ++t) {
    P.prog_off[t] = P.info[t].code_begin;
    P.kmax = std::max(P.kmax, P.info[t].need);
    P.max_ops = std::max(P.max_ops, (int32_t)P.info[t].op_sumcheck.size());
    P.max_len = std::max(P.max_len, P.info[t].code_len);
    P.total_nodes += P.info[t].nnodes;
    P.dec[t] = make_decide(P.info[t]);
    if (std::is_same<T, float>::value) P.sbound.insert(P.sbound.end(), {P.info[t].sb[0], P.info[t].sb[1], P.info[t].sb[2], 0.0f});
    if (der) {
      const TreeInfo& ti = dinfo[t];
      P.dprog_off[t] = ti.code_begin;
      P.dcost[t] = ti.cost;
      P.dkmax = std::max(P.dkmax, ti.need);
      P.dmax_len = std::max(P.dmax_len, ti.code_len);
    }
  }
  // (diagnostic) SRHIP_DUMP_CODE=path: the derived (or plain) program's instructions as int32 (h, a,
  // imm low, imm high) records with a (-1, static_fail, need, cost) separator per tree, for
  // instruction-mix studies (scripts/code_stats.py) and the code-cache test; with derived columns the
  // plain program's go to path.plain
  if (const char* dump = env_get("SRHIP_DUMP_CODE")) {
    for (int pass = 0; pass < (der ? 2 : 1); ++pass) {
      const bool dd = der && pass == 0;
      FILE* f = fopen(pass ? (std::string(dump) + ".plain").c_str() : dump, "wb");
      if (!f) break;
      const std::vector<Ins>& code = dd ? P.dcode : P.code;
      for (int32_t t = 0; t < n; ++t) {
        const TreeInfo& ti = dd ? dinfo[t] : P.info[t];
        for (int32_t i = 0; i < ti.code_len; ++i) {
          const Ins& ins = code[(size_t)ti.code_begin + i];
          const int32_t rec[4] = {(int32_t)ins.h, (int32_t)ins.a, (int32_t)(uint32_t)ins.imm,
                                  (int32_t)(uint32_t)(ins.imm >> 32)};
          fwrite(rec, sizeof rec, 1, f);
        }
        const int32_t sep[4] = {-1, ti.static_fail ? 1 : 0, ti.need, (int32_t)ti.cost};
        fwrite(sep, sizeof sep, 1, f);
      }
      fclose(f);
    }
  }
  return SRHIP_OK;
}

template <typename T>
int compile_grad_t(srhip_program& P) {
  P.g_derived = P.g_want_derived && !P.gdspec.empty();
  if (!P.g_derived) P.g_want_derived = false;
  P.gcode.clear();
  P.gprog_off.assign(P.ntrees, 0);
  P.ginfo.assign(P.ntrees, TreeInfo());
  P.gkmax = 0;
  P.gmax_len = 0;
  P.gmax_ops = 0;
  for (int32_t t = 0; t < P.ntrees; ++t) {
    const int64_t b = P.offsets[t], e = P.offsets[t + 1];
    TreeCompiler<T> tc(P.nodes.data() + b, e - b, P, 0, true);
    TreeInfo& gi = P.ginfo[t];
    int rc = tc.compile(gi, P.gcode);
    if (rc) return fail(rc, "tree %d (gradient program): %s", (int)t, g_err.c_str());
    P.gprog_off[t] = gi.code_begin;
    P.gkmax = std::max(P.gkmax, gi.need);
    P.gmax_len = std::max(P.gmax_len, gi.code_len);
    P.gmax_ops = std::max(P.gmax_ops, (int32_t)gi.op_sumcheck.size());
  }
  // speculative slots: the constant-carrying instructions of every tree, and the region itself
  P.gci_off.assign(P.ntrees + 1, 0);
  P.gci.clear();
  P.gspec_ok.assign(P.ntrees, 0);
  P.gbase.assign(P.ntrees, TreeInfo());
  for (int32_t t = 0; t < P.ntrees; ++t) {
    const TreeInfo& gi = P.ginfo[t];
    if (!gi.static_fail) {
      int32_t nc = 0;
      for (int32_t i = 0; i < gi.code_len; ++i) {
        const Ins& ins = P.gcode[(size_t)gi.code_begin + i];
        bool carries = ins.h == H_LOADC || (ins.h >= H_SLOADC0 && ins.h < H_SLOADC0 + K_MAX) ||
                       (ins.h >= H_PUSHLC0 && ins.h < H_PUSHLC0 + K_MAX);
        bool hi = false;  // the constant index in the upper half (leaf-constant superinstructions)
        if (ins.h >= H_BIN0 && ins.h < H_HEAVY0) {
          const uint32_t form = (ins.h - H_BIN0) % SPEC_STRIDE;
          carries = form == SPEC_AC || form == SPEC_CA || form == SPEC_FC || form == SPEC_CF;
          hi = form == SPEC_FC || form == SPEC_CF;
        }
        if (!carries) continue;
        P.gci.push_back(i);
        P.gci.push_back((int32_t)(hi ? ins.a >> 16 : ins.a & 0xffff & ~UN_UNIFORM_FLAG));  // (the constant index)
        ++nc;
      }
      // every constant leaf is consumed by exactly one such instruction
      P.gspec_ok[t] = nc == gi.nconst;
      if (P.gspec_ok[t]) P.gbase[t] = gi;
      else P.gci.resize(P.gci_off[t]);
    }
    P.gci_off[t + 1] = (int32_t)P.gci.size();
  }
  P.gspec_alloc = P.gspec_cap;
  P.gspec_stride = std::max<int32_t>(1, P.gmax_len);
  P.gspec_base = (int64_t)P.gcode.size();
  P.gcode.resize(P.gcode.size() + (size_t)P.gspec_alloc * P.gspec_stride, Ins{H_END, 0, 0});
  for (int32_t sl = 0; sl < P.gspec_alloc; ++sl) {
    P.gprog_off.push_back((int32_t)(P.gspec_base + (int64_t)sl * P.gspec_stride));
    TreeInfo si;
    si.static_fail = true;
    si.code_begin = P.gprog_off.back();
    si.code_len = 1;
    P.ginfo.push_back(si);
  }
  return SRHIP_OK;
}

template <typename T>
bool spec_instantiate_t(srhip_program& P, int32_t slot, int32_t t, const double* c, bool* static_fail, int64_t& lo,
                        int64_t& hi) {
  if (slot < 0 || slot >= P.gspec_alloc || t < 0 || t >= P.ntrees || P.gspec_ok.size() != (size_t)P.ntrees)
    return false;
  TreeInfo& si = P.ginfo[(size_t)P.ntrees + slot];
  const int64_t dst = P.gspec_base + (int64_t)slot * P.gspec_stride;
  // the tree's nodes at the constants c (get_constants order = pre-order over constant leaves)
  const int64_t b = P.offsets[t], e = P.offsets[t + 1];
  std::vector<srhip_node> nd(P.nodes.begin() + b, P.nodes.begin() + e);
  struct Rec {
    static void set(std::vector<srhip_node>& v, int64_t i, const double*& c) {
      srhip_node& n = v[(size_t)i];
      if (n.degree == 0) {
        if (n.constant) n.val = *c++;
        return;
      }
      set(v, n.l, c);
      if (n.degree == 2) set(v, n.r, c);
    }
  };
  const double* cp = c;
  Rec::set(nd, 0, cp);
  TreeCompiler<T> tc(nd.data(), e - b, P, 0, true);
  if (!P.gspec_ok[t]) {  // the code's shape is not known to be value-independent: compile it
    std::vector<Ins> scratch;
    TreeInfo gi;
    if (tc.compile(gi, scratch)) return false;
    *static_fail = gi.static_fail;
    if (!gi.static_fail) {
      if (gi.code_len > P.gspec_stride || (size_t)gi.code_len != scratch.size()) return false;
      std::copy(scratch.begin(), scratch.end(), P.gcode.begin() + dst);
      lo = std::min<int64_t>(lo, dst);
      hi = std::max<int64_t>(hi, dst + gi.code_len);
    }
    si = std::move(gi);
    si.code_begin = (int32_t)dst;
    if (si.static_fail) si.code_len = 1;
    return true;
  }
  // the base code with the constant immediates rewritten; metadata recomputed from the values
  const TreeInfo& base = P.gbase[t];
  if (base.code_len > P.gspec_stride) return false;
  TreeInfo meta;
  tc.static_info(meta);
  *static_fail = meta.static_fail;
  if (meta.static_fail) {  // @return_on_check: did_succeed = false, nothing to evaluate
    si = TreeInfo();
    si.static_fail = true;
    si.code_begin = (int32_t)dst;
    si.code_len = 1;
    return true;
  }
  std::copy(P.gcode.begin() + base.code_begin, P.gcode.begin() + base.code_begin + base.code_len, P.gcode.begin() + dst);
  for (int32_t j = P.gci_off[t]; j < P.gci_off[t + 1]; j += 2)
    P.gcode[(size_t)dst + P.gci[j]].imm = HostVal<T>::bits(HostVal<T>::from(c[P.gci[j + 1]]));
  si = base;
  si.fill_consts = std::move(meta.fill_consts);
  si.code_begin = (int32_t)dst;
  lo = std::min<int64_t>(lo, dst);
  hi = std::max<int64_t>(hi, dst + base.code_len);
  return true;
}

void grad_snapshot(srhip_program& P) {
  P.gsnap.clear();
  P.gsnap_off.assign(P.ntrees + 1, 0);
  for (int32_t t = 0; t < P.ntrees; ++t) {
    for (int64_t i = P.offsets[t]; i < P.offsets[t + 1]; ++i)
      if (P.nodes[(size_t)i].degree == 0 && P.nodes[(size_t)i].constant) P.gsnap.push_back(P.nodes[(size_t)i].val);
    P.gsnap_off[t + 1] = (int64_t)P.gsnap.size();
  }
}

// Recompile in place only the trees whose constant values differ (bitwise) from the snapshot the
// gradient program was compiled with.  A tree's code depends on its own nodes only and is
// position-independent, so an unchanged length means the new code drops into the old slot; any
// other outcome (length change, no snapshot) returns patched = false and the caller recompiles all.
// a tree's constant values in get_constants order (pre-order over constant leaves)
void gather_consts_preorder(const srhip_node* nd, int64_t i, std::vector<double>& out) {
  const srhip_node& n = nd[i];
  if (n.degree == 0) {
    if (n.constant) out.push_back(n.val);
    return;
  }
  gather_consts_preorder(nd, n.l, out);
  if (n.degree == 2) gather_consts_preorder(nd, n.r, out);
}

template <typename T>
int patch_grad_t(srhip_program& P, bool& patched, int64_t& lo, int64_t& hi) {
  patched = false;
  lo = INT64_MAX;
  hi = -1;
  const size_t nslots = (size_t)P.ntrees + P.gspec_alloc;
  if (P.gsnap.empty() || P.gprog_off.size() != nslots || P.ginfo.size() != nslots ||
      P.gsnap_off.size() != (size_t)P.ntrees + 1 || (size_t)P.gsnap_off[P.ntrees] != P.gsnap.size() ||
      P.gspec_cap != P.gspec_alloc || P.gspec_ok.size() != (size_t)P.ntrees || P.gci_off.size() != (size_t)P.ntrees + 1)
    return SRHIP_OK;
  std::vector<Ins> scratch;
  std::vector<double> cvals;
  // the trees the optimiser wrote constants of (P.ghint), or all of them
  std::vector<int32_t> all;
  if (P.ghint.empty()) {
    all.resize(P.ntrees);
    for (int32_t t = 0; t < P.ntrees; ++t) all[t] = t;
  }
  const std::vector<int32_t>& scan = P.ghint.empty() ? all : P.ghint;
  for (int32_t t : scan) {
    if (t < 0 || t >= P.ntrees) return SRHIP_OK;
    const int64_t b = P.offsets[t], e = P.offsets[t + 1];
    bool dirty = false;
    int64_t k = P.gsnap_off[t];
    for (int64_t i = b; i < e; ++i) {
      const srhip_node& n = P.nodes[(size_t)i];
      if (n.degree != 0 || !n.constant) continue;
      if (k >= P.gsnap_off[t + 1]) return SRHIP_OK;
      dirty |= memcmp(&n.val, &P.gsnap[k], sizeof(double)) != 0;
      P.gsnap[k++] = n.val;  // the snapshot follows the patch (this tree recompiles below if dirty)
    }
    if (!dirty) continue;
    if ((size_t)t < P.gspec_ok.size() && P.gspec_ok[t]) {
      // the code is the full compile's with new constant immediates; the did_succeed metadata is
      // recomputed from the new values (constant leaves' finiteness, constant subtrees folded)
      cvals.clear();
      gather_consts_preorder(P.nodes.data() + b, 0, cvals);
      TreeInfo meta;
      TreeCompiler<T>(P.nodes.data() + b, e - b, P, 0, true).static_info(meta);
      TreeInfo& cur = P.ginfo[t];
      const TreeInfo& base = P.gbase[t];
      cur = base;
      cur.static_fail = meta.static_fail;
      cur.fill_consts = std::move(meta.fill_consts);
      if (cur.static_fail) continue;  // skipped by the evaluation; the slot keeps its code
      for (int32_t j = P.gci_off[t]; j < P.gci_off[t + 1]; j += 2)
        P.gcode[(size_t)base.code_begin + P.gci[j]].imm = HostVal<T>::bits(HostVal<T>::from(cvals[P.gci[j + 1]]));
      lo = std::min<int64_t>(lo, base.code_begin);
      hi = std::max<int64_t>(hi, (int64_t)base.code_begin + base.code_len);
      continue;
    }
    scratch.clear();
    TreeCompiler<T> tc(P.nodes.data() + b, e - b, P, 0, true);
    TreeInfo gi;
    int rc = tc.compile(gi, scratch);
    if (rc) return fail(rc, "tree %d (gradient program): %s", (int)t, g_err.c_str());
    TreeInfo& old = P.ginfo[t];
    if (gi.static_fail) {
      // a non-finite constant: eval_grad skips the tree, so its slot keeps the last code (and
      // length) and a later finite point patches into the same slot instead of forcing a full
      // recompile of the whole population (trial points of the line search do overflow)
      gi.code_begin = old.code_begin;
      gi.code_len = old.code_len;
      old = std::move(gi);
      continue;
    }
    if (gi.code_len != old.code_len) return SRHIP_OK;
    std::copy(scratch.begin(), scratch.end(), P.gcode.begin() + old.code_begin);
    lo = std::min<int64_t>(lo, old.code_begin);
    hi = std::max<int64_t>(hi, (int64_t)old.code_begin + old.code_len);
    gi.code_begin = old.code_begin;
    old = std::move(gi);
  }
  P.gkmax = 0;
  P.gmax_len = 0;
  P.gmax_ops = 0;
  for (const TreeInfo& gi : P.ginfo) {
    P.gkmax = std::max(P.gkmax, gi.need);
    P.gmax_len = std::max(P.gmax_len, gi.code_len);
    P.gmax_ops = std::max(P.gmax_ops, (int32_t)gi.op_sumcheck.size());
  }
  patched = true;
  return SRHIP_OK;
}

}  // namespace

thread_local double srhip::g_patch_scan_s = 0.0, srhip::g_patch_copy_s = 0.0;
static double host_now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool srhip::spec_instantiate(srhip_program& P, int32_t slot, int32_t t, const double* c, bool* static_fail,
                             int64_t& lo, int64_t& hi) {
  switch (P.dtype) {
    case SRHIP_F32: return spec_instantiate_t<float>(P, slot, t, c, static_fail, lo, hi);
    case SRHIP_F64: return spec_instantiate_t<double>(P, slot, t, c, static_fail, lo, hi);
    default: return false;
  }
}

// the derived columns a constant-gradient program can read: every heavy unary operator applied to a
// feature leaf, distinct (operator, column) pairs in order of first appearance, at most GD_MAX
constexpr size_t GD_MAX = 32;
void srhip::grad_derived_spec(srhip_program& P) {
  if (P.gdspec_done) return;
  P.gdspec_done = true;
  P.gdspec.clear();
  P.gdbase = P.maxfeat;
  for (int32_t t = 0; t < P.ntrees; ++t) {
    const int64_t b = P.offsets[t], e = P.offsets[t + 1];
    for (int64_t i = b; i < e; ++i) {
      const srhip_node& n = P.nodes[i];
      if (n.degree != 1 || n.l < 0 || b + n.l >= e) continue;
      const srhip_node& c = P.nodes[b + n.l];
      if (c.degree != 0 || c.constant || n.op < 1 || n.op > (int)P.unaops.size()) continue;
      const int u = classify_unop(P.unaops[n.op - 1]);
      if (u < 0 || un_grad_inline(u)) continue;
      const uint32_t key = (uint32_t)u << 16 | (uint32_t)(c.feature - 1);
      if (std::find(P.gdspec.begin(), P.gdspec.end(), key) == P.gdspec.end() && P.gdspec.size() < GD_MAX)
        P.gdspec.push_back(key);
    }
  }
}

int srhip::compile_grad_program(srhip_program& P) {
  // a program compiled for the other form (derived columns or not) is compiled again in full
  if (P.grad_ready && P.g_derived != (P.g_want_derived && !P.gdspec.empty())) P.grad_ready = false;
  if (P.grad_ready) return SRHIP_OK;
  const bool same_form = P.g_derived == (P.g_want_derived && !P.gdspec.empty());
  static const bool no_patch = [] { const char* e = getenv("SRHIP_NO_GRAD_PATCH"); return e && *e && *e != '0'; }();
  int rc;
  bool patched = false;
  int64_t lo = 0, hi = -1;  // patched instruction range
  const double t_patch0 = host_now_s();
  if (!no_patch && same_form && P.ctx && P.d_gcode.p) {  // a previous full compile is on the device
    switch (P.dtype) {
      case SRHIP_F32: rc = patch_grad_t<float>(P, patched, lo, hi); break;
      case SRHIP_F64: rc = patch_grad_t<double>(P, patched, lo, hi); break;
      default: rc = SRHIP_OK; break;
    }
    g_patch_scan_s += host_now_s() - t_patch0;
    if (rc) return rc;
  }
  P.ghint.clear();
  if (patched) {  // the device copy differs only in [lo, hi); the snapshot was updated by the patch
    const double t_copy0 = host_now_s();
    HIP_TRY(hipSetDevice(P.ctx->device));
    if (hi > lo) {  // through pinned staging: a pageable source makes the runtime stage it synchronously
      const size_t nb = (size_t)(hi - lo) * sizeof(Ins);
      HIP_TRY(P.ctx->h_gpatch.ensure(nb));
      memcpy(P.ctx->h_gpatch.p, P.gcode.data() + lo, nb);
      HIP_TRY(hipMemcpyAsync((Ins*)P.d_gcode.p + lo, P.ctx->h_gpatch.p, nb, hipMemcpyHostToDevice, P.ctx->stream));
    }
    // no synchronisation here: the gradient launch follows on the same stream, and eval_grad
    // synchronises before it returns, so the staging is not touched while this copy is in flight
    g_patch_copy_s += host_now_s() - t_copy0;
    P.grad_ready = true;
    return SRHIP_OK;
  }
  switch (P.dtype) {
    case SRHIP_F32: rc = compile_grad_t<float>(P); break;
    case SRHIP_F64: rc = compile_grad_t<double>(P); break;
    default: return fail(SRHIP_ERR_UNSUPPORTED, "constant gradients need a Float32 or Float64 program");
  }
  if (rc) return rc;
  if (!P.ctx) return fail(SRHIP_ERR_INVALID, "host-only program");
  grad_snapshot(P);
  HIP_TRY(hipSetDevice(P.ctx->device));
  HIP_TRY(P.d_gcode.ensure(P.gcode.size() * sizeof(Ins)));
  HIP_TRY(P.d_goff.ensure(std::max<size_t>(1, P.gprog_off.size()) * sizeof(int32_t)));
  HIP_TRY(hipMemcpyAsync(P.d_gcode.p, P.gcode.data(), P.gcode.size() * sizeof(Ins), hipMemcpyHostToDevice, P.ctx->stream));
  if (!P.gprog_off.empty())
    HIP_TRY(hipMemcpyAsync(P.d_goff.p, P.gprog_off.data(), P.gprog_off.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                           P.ctx->stream));
  HIP_TRY(hipStreamSynchronize(P.ctx->stream));
  P.grad_ready = true;
  return SRHIP_OK;
}

int srhip::compile_program(srhip_program& P) {
  P.grad_ready = false;
  P.ghint.clear();
  {
    std::lock_guard<std::mutex> g(P.ord_mu);  // costs and live trees change: new schedule
    P.ord_key[0] = P.ord_key[1] = P.ord_key[2] = -1;
    P.ord_goff.clear();
  }
  switch (P.dtype) {
    case SRHIP_F32: return compile_program_t<float>(P);
    case SRHIP_F64: return compile_program_t<double>(P);
    case SRHIP_I32: return compile_program_t<int32_t>(P);
    default: return fail(SRHIP_ERR_INVALID, "bad dtype %d", P.dtype);
  }
}

// device pointers of the program's sections inside d_prog (blob_off layout)
static void set_prog_pointers(const srhip_program& P) {
  const uint8_t* d = (const uint8_t*)P.d_prog.p;
  const bool der = !P.dspec.empty();
  P.code_dev = (const Ins*)d;
  P.off_dev = (const int32_t*)(d + P.blob_off[0]);
  P.dcode_dev = der ? (const Ins*)(d + P.blob_off[1]) : nullptr;
  P.doff_dev = der ? (const int32_t*)(d + P.blob_off[2]) : nullptr;
  P.dspec_dev = der ? (const uint32_t*)(d + P.blob_off[3]) : nullptr;
  P.dmask_dev = der ? (const uint64_t*)(d + P.blob_off[4]) : nullptr;
  P.sbound_dev = P.sbound.empty() ? nullptr : (const float*)(d + P.blob_off[5]);
}

int srhip::upload_program(srhip_program& P, bool sync, bool defer, hipStream_t stream) {
  HIP_TRY(hipSetDevice(P.ctx->device));
  // one host image and one copy (each hipMemcpyAsync costs a few us of API time and a blit on the
  // stream: the coalescer uploads a small program per flush)
  auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const bool der = !P.dspec.empty();
  const size_t n_code = P.code.size() * sizeof(Ins), n_off = P.prog_off.size() * sizeof(int32_t);
  const size_t n_dcode = der ? P.dcode.size() * sizeof(Ins) : 0, n_doff = der ? P.dprog_off.size() * sizeof(int32_t) : 0;
  const size_t n_dspec = der ? P.dspec.size() * sizeof(uint32_t) : 0, n_dmask = der ? P.dmask.size() * sizeof(uint64_t) : 0;
  const size_t o_off = al(n_code), o_dcode = o_off + al(n_off), o_doff = o_dcode + al(n_dcode);
  const size_t n_sb = P.sbound.size() * sizeof(float);
  const size_t o_dspec = o_doff + al(n_doff), o_dmask = o_dspec + al(n_dspec), o_sb = o_dmask + al(n_dmask);
  const size_t total = std::max<size_t>(16, o_sb + al(n_sb));
  P.blob.assign(total, 0);
  uint8_t* h = P.blob.data();
  if (n_code) memcpy(h, P.code.data(), n_code);
  if (n_off) memcpy(h + o_off, P.prog_off.data(), n_off);
  if (n_dcode) memcpy(h + o_dcode, P.dcode.data(), n_dcode);
  if (n_doff) memcpy(h + o_doff, P.dprog_off.data(), n_doff);
  if (n_dspec) memcpy(h + o_dspec, P.dspec.data(), n_dspec);
  if (n_dmask) memcpy(h + o_dmask, P.dmask.data(), n_dmask);
  if (n_sb) memcpy(h + o_sb, P.sbound.data(), n_sb);
  const size_t offs[7] = {o_off, o_dcode, o_doff, o_dspec, o_dmask, o_sb, total};
  memcpy(P.blob_off, offs, sizeof(offs));
  if (defer) {
    P.upload_pending = true;
    return SRHIP_OK;
  }
  P.upload_pending = false;
  // a launch order planned at creation (plan_persistent_order) travels in the same copy
  const bool with_order = !P.ord_host.empty() && P.ord_key[0] > 0;
  const size_t nbytes = with_order ? total + P.ord_host.size() * sizeof(int32_t) : total;
  if (with_order) {
    P.blob.resize(nbytes);
    memcpy(P.blob.data() + total, P.ord_host.data(), P.ord_host.size() * sizeof(int32_t));
    h = P.blob.data();
  }
  HIP_TRY(P.d_prog.ensure(nbytes));
  hipStream_t st = stream ? stream : P.ctx->stream;
  HIP_TRY(hipMemcpyAsync(P.d_prog.p, h, nbytes, hipMemcpyHostToDevice, st));
  set_prog_pointers(P);
  if (with_order) P.ord_dev = (const uint8_t*)P.d_prog.p + total;
  if (sync) HIP_TRY(hipStreamSynchronize(st));
  return SRHIP_OK;
}


// ---------------------------------------------------------------------------------------------
// evaluation driver
// ---------------------------------------------------------------------------------------------
namespace {

}  // namespace

int srhip::make_view(srhip_ctx* ctx, const srhip_dataset* ds, const int64_t* idx, int64_t nidx, bool need_y, View& v) {
  if (need_y && !ds->has_y) return fail(SRHIP_ERR_INVALID, "dataset has no y");
  if (!idx) {
    v.X = ds->X.p;
    v.y = ds->y.p;
    v.w = ds->weighted ? ds->w.p : nullptr;
    v.ld = ds->ld;
    v.m = ds->n;
    v.stats = ds->hstats.data();
    v.sum_w = ds->sum_w;
    return SRHIP_OK;
  }
  if (nidx <= 0) return fail(SRHIP_ERR_INVALID, "empty idx");
  for (int64_t i = 0; i < nidx; ++i)
    if (idx[i] < 0 || idx[i] >= ds->n) return fail(SRHIP_ERR_INVALID, "idx[%lld] = %lld out of range", (long long)i, (long long)idx[i]);
  const size_t es = dtype_size(ds->dtype);
  const int64_t ld = (nidx + ROW_ALIGN - 1) / ROW_ALIGN * ROW_ALIGN;
  HIP_TRY(ctx->vX.ensure((size_t)std::max<int64_t>(1, ds->nfeat) * ld * es));
  HIP_TRY(ctx->vy.ensure((size_t)ld * es));
  HIP_TRY(ctx->vw.ensure((size_t)ld * es));
  HIP_TRY(ctx->vidx.ensure((size_t)nidx * sizeof(int64_t)));
  HIP_TRY(ctx->vstats.ensure(feature_stats_scratch(ds->nfeat) * sizeof(FeatStat)));
  HIP_TRY(ctx->h_stats.ensure((size_t)std::max<int64_t>(1, ds->nfeat) * sizeof(FeatStat)));
  HIP_TRY(hipMemcpyAsync(ctx->vidx.p, idx, (size_t)nidx * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(launch_gather(ds->dtype, ds->X.p, ds->has_y ? ds->y.p : nullptr, ds->weighted ? ds->w.p : nullptr, ds->ld,
                        (int)ds->nfeat, (const int64_t*)ctx->vidx.p, nidx, ld, ctx->vX.p,
                        ds->has_y ? ctx->vy.p : nullptr, ds->weighted ? ctx->vw.p : nullptr, ctx->stream));
  HIP_TRY(launch_feature_stats(ds->dtype, ctx->vX.p, ld, nidx, (int)ds->nfeat, (FeatStat*)ctx->vstats.p, ctx->stream));
  if (ds->dtype != SRHIP_I32 && ds->nfeat > 0)
    HIP_TRY(hipMemcpyAsync(ctx->h_stats.p, ctx->vstats.p, (size_t)ds->nfeat * sizeof(FeatStat), hipMemcpyDeviceToHost,
                           ctx->stream));
  double sw = 0.0;
  if (ds->weighted) {
    // sum of gathered weights, from the host copy kept at upload
    // (computed below by the caller from the device buffer would need a sync; weights are small)
  }
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  v.X = ctx->vX.p;
  v.y = ds->has_y ? ctx->vy.p : nullptr;
  v.w = ds->weighted ? ctx->vw.p : nullptr;
  v.ld = ld;
  v.m = nidx;
  v.stats = (const FeatStat*)ctx->h_stats.p;
  v.sum_w = sw;
  return SRHIP_OK;
}

LaunchPlan srhip::plan_launch(const srhip_ctx* ctx, int dtype, int64_t nxcols, bool weighted, bool with_y, int64_t m,
                              int32_t ntrees, int tile, size_t budget, int waves) {
  LaunchPlan L;
  ntrees = std::max<int32_t>(1, ntrees);  // every tree may have failed statically
  m = std::max<int64_t>(1, m);
  const size_t es = dtype_size(dtype);
  const int ncols = (int)nxcols + (with_y ? 1 : 0) + (weighted ? 1 : 0);
  const int lo = std::max(tile, loss_chunk(dtype));  // row blocks are whole tiles and loss chunks
  int rb = ROW_ALIGN;
  while (rb > lo && (size_t)ncols * rb * es > budget) rb /= 2;
  // do not make blocks much larger than the data
  while (rb > lo && rb / 2 >= m) rb /= 2;
  // diagnostic override (tuning runs): SRHIP_RB_ROWS = rows per workgroup, a power of two >= tile
  static const int rb_env = [] { const char* e = getenv("SRHIP_RB_ROWS"); return e ? atoi(e) : 0; }();
  if (rb_env >= lo && rb_env <= ROW_ALIGN && (rb_env & (rb_env - 1)) == 0 && rb_env < rb) rb = rb_env;
  L.rb_rows = rb;
  L.xlds = (size_t)ncols * rb * es <= budget;
  L.lds = (L.xlds ? (size_t)ncols * rb * es : 0) + 16;
  L.nrb = (int)((m + rb - 1) / rb);
  const int target_blocks = 4 * ctx->num_cu;
  int g = (target_blocks + L.nrb - 1) / L.nrb;
  const int max_g = std::max(1, ntrees / (2 * waves));
  g = std::max(1, std::min(g, max_g));
  L.groups = g;
  L.tpg = (ntrees + g - 1) / g;
  L.groups = (ntrees + L.tpg - 1) / L.tpg;
  return L;
}

namespace {

// Tree groups of a launch (grid.y), as offsets into the order: the plan's uniform groups, or —
// when the launch spans several waves of workgroups over the chip's 2-per-CU slots — the bulk in
// g equal groups plus ~1/32 of the trees in halving tail groups (..., 32, 16, <=16).  Workgroups
// dispatch group by group, so the small ones come last and fill the slots the bulk leaves idle:
// identical workgroups over 977 row tiles x 2 groups use <= 95 % of 512 slots.  Measured on C2
// (scripts/tail_sweep.sh): uniform 2.13 ms, tail 1/32 2.04-2.06 ms, 1/16 2.10, 1/8 2.18 (every
// extra workgroup restages its rows and derived columns, so bigger tails or more bulk groups lose).
// SRHIP_NO_TAIL=1: uniform groups.
std::vector<int32_t> shape_groups(const LaunchPlan& L, int32_t ntrees, int num_cu) {
  static const bool no_tail = [] { const char* e = getenv("SRHIP_NO_TAIL"); return e && *e && *e != '0'; }();
  std::vector<int32_t> off(1, 0);
  const bool tail = !no_tail && ntrees >= 128 && (int64_t)L.groups * L.nrb > 2 * (int64_t)num_cu;
  if (!tail) {
    for (int g = 0; g < L.groups; ++g) off.push_back(std::min(ntrees, off.back() + L.tpg));
    return off;
  }
  // tuning hooks: SRHIP_TAIL_DIV (tail = trees / DIV, default 32), SRHIP_BULK_GROUPS (default: the
  // plan's), SRHIP_TAIL_MIN (smallest tail group, default 16)
  static const int tail_div = [] { const char* e = getenv("SRHIP_TAIL_DIV"); return e && atoi(e) >= 2 ? atoi(e) : 32; }();
  static const int bulk_g = [] { const char* e = getenv("SRHIP_BULK_GROUPS"); return e ? atoi(e) : 0; }();
  const int32_t tl = std::max<int32_t>(16, ntrees / tail_div), bulk = ntrees - tl;
  const int groups = bulk_g > 0 ? std::min<int>(bulk_g, std::max(1, bulk / 16)) : L.groups;
  const int32_t tpg = (bulk + groups - 1) / groups;
  while (off.back() < bulk) off.push_back(std::min(bulk, off.back() + tpg));
  static const int tail_min = [] { const char* e = getenv("SRHIP_TAIL_MIN"); return e && atoi(e) > 0 ? atoi(e) : 16; }();
  int32_t t = tl;
  while (t > tail_min) {
    const int32_t h = t / 2;
    off.push_back(off.back() + h);
    t -= h;
  }
  if (t > 0) off.push_back(off.back() + t);
  return off;
}

// trees sorted by estimated cost (desc), dealt to the groups in proportion to their sizes (each
// tree to the group with the largest free fraction), so every group gets the same cost mix;
// returns order [ntrees], group g's trees at [goff[g], goff[g+1])
std::vector<int32_t> make_order(const srhip_program& P, const std::vector<int32_t>& trees,
                                const std::vector<int32_t>& goff, bool derived) {
  std::vector<int32_t> s(trees);
  auto cost = [&](int32_t t) { return derived ? P.dcost[t] : P.info[t].cost; };
  std::stable_sort(s.begin(), s.end(), [&](int32_t a, int32_t b) { return cost(a) > cost(b); });
  const int groups = (int)goff.size() - 1;
  std::vector<int32_t> order(s.size());
  std::vector<int> fill(groups, 0);
  for (int32_t t : s) {
    int best = -1;
    double bf = -1.0;
    for (int g = 0; g < groups; ++g) {
      const int cap = goff[g + 1] - goff[g];
      if (fill[g] >= cap) continue;
      const double f = (double)(cap - fill[g]) / cap;
      if (f > bf) {
        bf = f;
        best = g;
      }
    }
    order[(size_t)goff[best] + fill[best]++] = t;
  }
  return order;
}

// ---- the did_succeed decision, from (possibly all-reduced) partials ----------------------------
// Partials layout (the C ABI's srhip_eval_loss_partials): sums[2t] = sum of (w *) l over the rows,
// sums[2t+1] = sum of w (unweighted: the row count); sums[2T + 2f] = feature f column sum (Float64
// data: sum of x * 2^-64), sums[2T + 2f + 1] = its non-finite count; sums[2T + 2F] = rows.  Every
// entry combines across row shards by addition; chk[t] (the operator-output check statistic)
// combines by max for Float32 (max |v|) and by addition for Float64 (sum of |v| 2^-512).
static size_t sums_len(int32_t ntrees, int64_t nfeat) { return 2 * (size_t)ntrees + 2 * (size_t)nfeat + 1; }

// Returns 0 ok, 1 fail, 2 undecided (needs the precise pass).
static int decide_info(const TreeInfo& I, int dtype, int32_t T, int64_t nfeat, const double* sums, double chk) {
  if (I.static_fail) return 1;
  if (dtype == SRHIP_I32) return 0;
  const long double m = (long double)sums[2 * (size_t)T + 2 * (size_t)nfeat];
  const long double ovf = ovf_threshold(dtype);
  for (double c : I.fill_consts)
    if ((long double)fabs(c) * m >= ovf) return 1;
  for (int f : I.feat_checks) {
    const double fsum = sums[2 * (size_t)T + 2 * (size_t)f], fbad = sums[2 * (size_t)T + 2 * (size_t)f + 1];
    if (fbad > 0) return 1;
    const long double sum = dtype == SRHIP_F64 ? (long double)fsum * 0x1p64L : (long double)fsum;
    if (!isfinite(fsum) || fabsl(sum) >= ovf) return 1;
  }
  if (I.op_sumcheck.empty()) return 0;
  if (!isfinite(chk)) return 1;  // a NaN / Inf operator output
  long double bound;
  if (dtype == SRHIP_F64) bound = (long double)chk * 0x1p512L;  // sum |v|
  else bound = (long double)chk * m;                              // m * max |v|
  if (bound * 2.0L >= ovf) return 2;
  return 0;
}

// decide_info on the compact record: the same answer (fill constants: |c| m >= OVF is monotone in
// |c|, so the largest decides; NaN never fails; the feature checks in any order)
static int decide_fast(const srhip_program& P, int32_t t, int64_t nfeat, const double* sums, double chk) {
  const TreeDecide& d = P.dec[t];
  if (d.slow) return decide_info(P.info[t], P.dtype, P.ntrees, nfeat, sums, chk);
  if (d.static_fail) return 1;
  const int dtype = P.dtype;
  if (dtype == SRHIP_I32) return 0;
  const int32_t T = P.ntrees;
  const long double m = (long double)sums[2 * (size_t)T + 2 * (size_t)nfeat];
  const long double ovf = ovf_threshold(dtype);
  if (d.maxc >= 0.0 && (long double)d.maxc * m >= ovf) return 1;
  for (uint64_t fm = d.feat_mask; fm; fm &= fm - 1) {
    const int f = __builtin_ctzll(fm);
    const double fsum = sums[2 * (size_t)T + 2 * (size_t)f], fbad = sums[2 * (size_t)T + 2 * (size_t)f + 1];
    if (fbad > 0) return 1;
    const long double sum = dtype == SRHIP_F64 ? (long double)fsum * 0x1p64L : (long double)fsum;
    if (!isfinite(fsum) || fabsl(sum) >= ovf) return 1;
  }
  if (!d.has_op) return 0;
  if (!isfinite(chk)) return 1;
  long double bound;
  if (dtype == SRHIP_F64) bound = (long double)chk * 0x1p512L;
  else bound = (long double)chk * m;
  if (bound * 2.0L >= ovf) return 2;
  return 0;
}

static void finalize(const srhip_program& P, int64_t nfeat, const double* sums, const double* chk, double* out_loss,
                     uint8_t* out_ok, uint8_t* out_status) {
  const bool fast = P.dec.size() == (size_t)P.ntrees && !env_flag("SRHIP_DECIDE_SLOW");
  for (int32_t t = 0; t < P.ntrees; ++t) {
    const double c = chk ? chk[t] : 0.0;
    const int st = fast ? decide_fast(P, t, nfeat, sums, c) : decide_info(P.info[t], P.dtype, P.ntrees, nfeat, sums, c);
    if (out_status) out_status[t] = (uint8_t)st;
    if (out_ok) out_ok[t] = st == 0 ? 1 : 0;
    if (out_loss) out_loss[t] = st == 0 ? sums[2 * (size_t)t] / sums[2 * (size_t)t + 1] : INFINITY;
  }
}

// opsums[u][k]: exact-ish (f64) sum over all rows of operator output k of tree trees[u]
static void finalize_precise(const srhip_program& P, const int32_t* trees, int32_t nsel, const double* opsums,
                             uint8_t* out_ok, bool grad = false) {
  const int stride = std::max(1, grad ? P.gmax_ops : P.max_ops);
  const long double ovf = ovf_threshold(P.dtype);
  for (int u = 0; u < nsel; ++u) {
    const TreeInfo& I = grad ? P.ginfo[trees[u]] : P.info[trees[u]];
    int st = I.static_fail ? 1 : 0;
    for (size_t k = 0; k < I.op_sumcheck.size() && !st; ++k) {
      const double s = opsums[(size_t)u * stride + k];
      if (!isfinite(s)) st = 1;
      else if (I.op_sumcheck[k]) {
        const long double S = P.dtype == SRHIP_F64 ? (long double)s * 0x1p64L : (long double)s;
        if (fabsl(S) >= ovf) st = 1;
      }
    }
    out_ok[u] = st == 0 ? 1 : 0;
  }
}

}  // namespace

// ---- the device-allocation cache behind PoolBuf ----------------------------------------------
namespace {
struct DevPool {
  std::mutex mu;
  std::map<std::pair<int, size_t>, std::vector<void*>> free;  // (device, size class) -> blocks
  size_t cached = 0;
};
DevPool& devpool() {
  static DevPool* P = new DevPool();  // never destroyed: blocks outlive static destruction order
  return *P;
}
constexpr size_t DEVPOOL_MAX_CACHED = (size_t)512 << 20;
size_t devpool_class(size_t n) {
  size_t c = 4096;
  while (c < n) c <<= 1;
  return c;
}
}  // namespace

void* srhip::devpool_get(size_t bytes, size_t* cap) {
  const size_t c = devpool_class(bytes);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  {
    DevPool& P = devpool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.free.find({dev, c});
    if (it != P.free.end() && !it->second.empty()) {
      void* q = it->second.back();
      it->second.pop_back();
      P.cached -= c;
      *cap = c;
      return q;
    }
  }
  void* q = nullptr;
  if (hipMalloc(&q, c) != hipSuccess) return nullptr;
  *cap = c;
  return q;
}

void srhip::devpool_put(void* p, size_t cap, int device) {
  if (!p) return;
  DevPool& P = devpool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (device >= 0 && P.cached + cap <= DEVPOOL_MAX_CACHED) {
      P.free[{device, cap}].push_back(p);
      P.cached += cap;
      return;
    }
  }
  (void)hipFree(p);
}

int srhip::next_fail_epoch(srhip_ctx* ctx, int64_t n, int32_t** flags, int32_t* epoch) {
  const size_t need = (size_t)std::max<int64_t>(n, 1) * sizeof(int32_t);
  const bool fresh = !ctx->fail_flag.p || ctx->fail_flag.bytes < need;  // (a new buffer may reuse an address)
  HIP_TRY(ctx->fail_flag.ensure(need));
  if (fresh || ctx->epoch == INT32_MAX) {  // fresh buffer (or wrap): no stale epochs
    HIP_TRY(hipMemsetAsync(ctx->fail_flag.p, 0, ctx->fail_flag.bytes, ctx->stream));
    ctx->epoch = 0;
  }
  *flags = (int32_t*)ctx->fail_flag.p;
  *epoch = ++ctx->epoch;
  return SRHIP_OK;
}

int srhip::decide_tree(const TreeInfo& I, const srhip_program& P, int64_t nfeat, const double* sums, double chk) {
  return decide_info(I, P.dtype, P.ntrees, nfeat, sums, chk);
}

int srhip::check_eval_args(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode,
                           const srhip_loss* loss) {
  if (!ctx || !ds || !P) return fail(SRHIP_ERR_INVALID, "null handle");
  if (!P->ctx) return fail(SRHIP_ERR_INVALID, "host-only program (created without a context) cannot be evaluated");
  if (ds->dtype != P->dtype) return fail(SRHIP_ERR_INVALID, "dataset dtype %d != program dtype %d", ds->dtype, P->dtype);
  // a dataset is read-only device memory after its (synchronised) upload: any context on its device
  // may evaluate over it (the coalescer's worker contexts share the caller's dataset)
  if (P->ctx != ctx) return fail(SRHIP_ERR_INVALID, "program belongs to a different context");
  if (ds->ctx != ctx && ds->device != ctx->device) return fail(SRHIP_ERR_INVALID, "dataset is on another device");
  if (P->maxfeat > ds->nfeat)
    return fail(SRHIP_ERR_INVALID, "tree uses feature %d but dataset has %lld features", (int)P->maxfeat, (long long)ds->nfeat);
  if (mode == MODE_LOSS) {
    if (!loss) return fail(SRHIP_ERR_INVALID, "null loss");
    if (P->dtype == SRHIP_I32 && loss->kind != SRHIP_LOSS_L2 && loss->kind != SRHIP_LOSS_L1)
      return fail(SRHIP_ERR_UNSUPPORTED, "Int32 datasets support L2/L1 losses only");
    if (loss->kind < SRHIP_LOSS_L2 || loss->kind > SRHIP_LOSS_DWD_MARGIN)
      return fail(SRHIP_ERR_UNSUPPORTED, "loss kind %d", loss->kind);
  }
  return SRHIP_OK;
}

static bool env_flag(const char* name) {
  const char* e = env_get(name);
  return e && *e && *e != '0';
}
static int env_int(const char* name, int dflt) {
  const char* e = env_get(name);
  return e && *e ? atoi(e) : dflt;
}

// run_eval's device-decided precise pass: the reduction lists the trees whose overflow bound needs
// the precise pass, and the precise launch + its reduction follow on the stream before the one host
// synchronisation (no host round trip between the main launch and the precise pass)
constexpr int32_t DEV_PRECISE_MAX = 64;
// h_pout = [count, list (DEV_PRECISE_MAX) | pad to 8 bytes | per-operator sums (double)]: the sums start on
// an 8-byte boundary (they followed the 65 ints directly, at byte 260: misaligned double stores on the
// device and loads on the host -- UBSan's report from tools/host_stress, round 6)
constexpr size_t PREC_SUMS_OFF = ((size_t)(1 + DEV_PRECISE_MAX) * sizeof(int32_t) + 7) & ~(size_t)7;
struct DevPrecise {
  bool used = false;
  int32_t count = 0;             // trees the device listed (may exceed DEV_PRECISE_MAX)
  int stride = 1;
  std::vector<int32_t> list;     // the first min(count, DEV_PRECISE_MAX) of them
  std::vector<double> opsums;    // [list.size()][stride]
};

// Device stage: one interpreter launch over the view + the per-tree reduction.  Fills the partials
// (sums layout above; chk[T]) and, in MODE_PRED, out_pred.  dp (nullable): also the device-decided
// precise pass (multi-block launches; single-block launches finish inside the interpreter and leave
// the precise pass to the caller).
// Row shards (run_eval_sharded): the reduction writes each tree's loss sum and check statistic into the
// exchange's device buffer instead of host memory (sums[2t] / chk stay to be filled from the all-reduced
// buffer); the rows each tree was evaluated on come back for the caller's lost-block check.
struct ShardDev {
  void* d_loss = nullptr;
  void* d_chk = nullptr;
  size_t zero_bytes = 0;  // [loss | chk] cleared before the launch (static-fail trees are never written)
};

// The device-listed precise pass, enqueued on the context's stream: the plain program over the trees
// of the device list ulist ([count, trees ...], count read by the launch, at most cap of them):
// one-tile row blocks and one-wave workgroups, G workgroups per row block, workgroup g taking the
// listed slots g, g + G, ... (G from the program's last count: an unused workgroup still costs its
// dispatch, and a count past G costs one launch longer, not another host round trip) -- K_MAX,
// global reads; then the double-double reduction of the per-block operator sums into the context's
// coherent h_pout ([count, list ..., sums]), which also clears the list.
// The precise pass's scratch (the per-block operator sums of the listed trees, their reduction's host
// output), ensured before the evaluation's main launch: a regrowth frees the old buffer, which
// synchronises the device -- after the launch that would wait for the whole evaluation.  Sized for
// a power-of-two operator count (32 at least: one size for every population of trees up to 33
// nodes) and at most 64 MB of per-block sums: the list's capacity (*cap, <= DEV_PRECISE_MAX) shrinks
// for very long row ranges (4 at least); trees past it take the host-written list.
constexpr size_t PRECISE_SLAB_MAX = (size_t)64 << 20;
constexpr int PRECISE_GRID_X = 2048;
static size_t precise_per_tree(const srhip_program* P, const View& v, int* sa_out = nullptr) {
  int sa = 32;
  while (sa < P->max_ops) sa <<= 1;
  if (sa_out) *sa_out = sa;
  const int rows = 64 * pick_rows_per_lane(P->dtype, K_MAX, MODE_PRECISE, v.m);
  const int64_t nrb = std::max<int64_t>(1, (v.m + rows - 1) / rows);
  return (size_t)sa * nrb * sizeof(double);
}
static int precise_cap(const srhip_program* P, const View& v, int cap) {
  return (int)std::max<int64_t>(std::min<int64_t>(cap, (int64_t)(PRECISE_SLAB_MAX / precise_per_tree(P, v))), 4);
}
static int ensure_dev_precise(srhip_ctx* ctx, const srhip_program* P, const View& v, int* cap, ResultSet* rs) {
  int sa = 32;
  const size_t per_tree = precise_per_tree(P, v, &sa);
  *cap = precise_cap(P, v, *cap);
  HIP_TRY(ctx->slab_prec.ensure((size_t)*cap * per_tree));
  HIP_TRY(rs->h_pout.ensure(PREC_SUMS_OFF +
                            (size_t)DEV_PRECISE_MAX * sa * sizeof(double), hipHostMallocCoherent));
  return SRHIP_OK;
}
static int enqueue_dev_precise(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const View& v,
                               int32_t* ulist, int cap, int G, int* out_stride, ResultSet* rs) {
  const int dtype = P->dtype;
  const int stride = std::max(1, P->max_ops);
  const int Rp = pick_rows_per_lane(dtype, K_MAX, MODE_PRECISE, v.m);
  G = std::max(1, std::min(G, cap));
  LaunchPlan Lp = plan_launch(ctx, dtype, ds->nfeat, false, false, v.m, G, 64 * Rp);
  Lp.rb_rows = 64 * Rp;
  Lp.nrb = (int)((v.m + Lp.rb_rows - 1) / Lp.rb_rows);
  {
    int c = cap;
    const int rc = ensure_dev_precise(ctx, P, v, &c, rs);
    if (rc) return rc;
    if (c < cap) return fail(SRHIP_ERR_INVALID, "precise list of %d trees past its capacity %d", cap, c);
  }
  EvalArgs q{};
  q.code = P->code_dev;
  q.prog_off = P->off_dev;
  q.order = ulist + 1;
  q.X = v.X;
  q.ld = v.ld;
  q.nvalid = v.m;
  q.ntrees = cap;
  q.grid_interleave = 1;  // grid.y = G workgroups share the list's slots interleaved
  q.nfeat = (int32_t)ds->nfeat;
  q.rb_rows = Lp.rb_rows;
  q.nrb = Lp.nrb;
  q.trees_per_group = 1;
  q.slab_prec = ctx->slab_prec.p;
  q.prec_stride = stride;
  q.max_steps = P->max_len;
  q.dev_count = ulist;
  q.wg_waves = 1;
  q.prec_assign = 1;  // one-tile row blocks
  // at most PRECISE_GRID_X workgroups per group, each striding over the row blocks: the launch runs
  // whether or not the list holds a tree, and with an empty list its cost is the workgroups'
  // dispatch (10M rows: 19532 x G one-wave workgroups, 41 us)
  q.block_stride = 1;
  HIP_TRY(launch_eval(dtype, q, Rp, K_MAX, MODE_PRECISE, false, dim3(std::min(Lp.nrb, PRECISE_GRID_X), G), 16,
                      ctx->stream));
  int32_t* hl = (int32_t*)rs->h_pout.p;
  double* hs = (double*)((uint8_t*)rs->h_pout.p + PREC_SUMS_OFF);
  HIP_TRY(launch_precise_reduce((const double*)ctx->slab_prec.p, Lp.nrb, stride, ulist, cap, G, DEV_PRECISE_MAX, hl,
                                hs, ctx->stream));
  *out_stride = stride;
  return SRHIP_OK;
}

// An evaluation between its launches (eval_issue) and the reading of its records (eval_collect): what
// the second half needs of the first.  The launches of several jobs may be in flight on the context's
// stream at once (srhip_eval_loss_submit), each with its own result set.
struct EvalJob {
  ResultSet* rs = nullptr;
  bool launched = false, persistent = false, devp = false;
  int mode = 0, dtype = 0;
  int32_t nt = 0;
  int32_t expect_items = 0;  // persistent launches: the items its workgroups must report evaluated
  std::vector<int32_t> live;
  UndecidedList ul;
  DevBuf pred;  // MODE_PRED's device output (synchronous calls only)
  bool fused = false;  // single-block launch: the interpreter wrote the records (no reduction)
  float fbound = 0.0f;  // Float32: the features' max |x| (the +/- bound's F)
};
// the features' max |x| over a view's rows (+Inf if any entry is non-finite), rounded up to Float32:
// the F of the Float32 interpreter's +/- bound (EvalArgs::fbound)
static float feature_bound(const View& v, int64_t nfeat) {
  double F = 0.0;
  for (int64_t f = 0; v.stats && f < nfeat; ++f) {
    if (v.stats[f].nonfinite > 0 || !(v.stats[f].maxabs < INFINITY)) return INFINITY;
    F = std::max(F, v.stats[f].maxabs);
  }
  if (!v.stats && nfeat > 0) return INFINITY;
  const float r = (float)F;
  return (double)r >= F ? r : std::nextafter(r, INFINITY);
}

static int eval_issue(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode, const srhip_loss* loss,
                      const View& v, void* out_pred, double* sums, double* chk, DevPrecise* dp, ShardDev* sd,
                      EvalJob& J) {
  const int dtype = P->dtype;
  const int32_t nt = P->ntrees;
  ResultSet* const rs = J.rs;
  J.mode = mode;
  J.dtype = dtype;
  J.nt = nt;
  const int64_t nf = ds->nfeat;
  const bool weighted = ds->weighted && mode == MODE_LOSS;
  for (size_t i = 0; i < sums_len(nt, nf); ++i) sums[i] = 0.0;
  for (int32_t t = 0; t < nt; ++t) {
    chk[t] = 0.0;
    sums[2 * (size_t)t + 1] = weighted ? v.sum_w : (double)v.m;
  }
  for (int64_t f = 0; f < nf; ++f) {
    sums[2 * (size_t)nt + 2 * f] = v.stats[f].sum;
    sums[2 * (size_t)nt + 2 * f + 1] = (double)v.stats[f].nonfinite;
  }
  sums[2 * (size_t)nt + 2 * nf] = (double)v.m;
  std::vector<int32_t>& live = J.live;
  live.clear();
  live.reserve(nt);
  for (int32_t t = 0; t < nt; ++t)
    if (!(P->dec.size() == (size_t)nt ? P->dec[t].static_fail : P->info[t].static_fail)) live.push_back(t);
  if (live.empty()) return SRHIP_OK;
  const size_t es = dtype_size(dtype);
  // stack slots of the kernel variant; the wide operators live only in the K_MAX variant
  bool wide = false;
  for (int32_t u : P->unaops) wide |= u == SRHIP_OP_ASIN || u == SRHIP_OP_ACOS || u == SRHIP_OP_ATANH_CLIP;
  auto kvariant = [&](int32_t kmax) { return wide ? K_MAX : (kmax <= 2 ? 2 : (kmax <= 4 ? 4 : 8)); };
  // derived-column program when its staging fits LDS (the R = 16 variant runs 2 workgroups per CU,
  // so it may use 80 KB); otherwise the plain program
  const int nd = (int)P->dspec.size();
  bool use_d = false;
  int K = 0, R = 0;
  LaunchPlan L{};
  // LDS a workgroup may stage: the 16-wave variant runs one workgroup per CU (160 KB, less the
  // kernel's static arrays); 8-wave workgroups run two (derived-column programs) or more
  // (the device's LDS per workgroup, read once per context, less 8 KB for the kernel's static arrays)
  const size_t lds_dev = (size_t)ctx->lds_max;
  auto lds_budget = [lds_dev](int r, int k, bool derived) -> size_t {
    if (eval_waves(r, k) >= 16) return lds_dev - 8 * 1024;
    return std::min<size_t>(lds_dev / 2, derived ? 64 * 1024 - 512 : 64 * 1024 - 64);
  };
  // Persistent launch (the wide Float32 variant's loss launches): one workgroup per CU claims short
  // row blocks from a counter and interprets the WHOLE population over each -- the dataset is read
  // from HBM once, every derived column is computed once per row block for all trees, and the tail
  // is one short block instead of a wave of workgroups.  A probe launch first evaluates the leading
  // row blocks with many small tree groups, so trees that fail there (DynamicExpressions' early
  // return: did_succeed = false whatever the other rows hold) are skipped by every later block.
  // SRHIP_NO_PERSISTENT=1: the grid launch; SRHIP_PRB_ROWS: row-block rows (default 2048: C2, one
  // MI355X, same box: 1024 rows 1.31 ms, 2048 1.19, 4096 1.35, grid launch 1.33);
  // SRHIP_PROBE_BLOCKS: probe row blocks (default 4).
  // (read per launch: tests and the bench toggle them inside one process)
  const bool no_persistent = env_flag("SRHIP_NO_PERSISTENT");
  const int prb_env = env_int("SRHIP_PRB_ROWS", 0);
  const int probe_env = env_int("SRHIP_PROBE_BLOCKS", -1);
  bool persistent = false;
  int probe_blocks = 0;
  // Few trees over many rows (the search's coalesced launches: C3 carries ~2.4 trees per launch over
  // 10M rows): a workgroup of one wave per tree per loss chunk of rows, X read from global memory.
  // The staged launches give each tree one wave per CU -- a 2048-row block staged for 2 trees leaves
  // 14 of its 16 waves idle.  SRHIP_SMALL_POP: the largest population launched this way (0: never).
  const int small_max = env_int("SRHIP_SMALL_POP", 16);
  const bool small = (mode == MODE_LOSS || mode == MODE_PRED) && debug_stop() == 0 && (int)live.size() <= small_max &&
                     v.m >= (int64_t)64 * ROW_ALIGN;
  if (small) {
    K = kvariant(P->kmax);
    R = pick_rows_per_lane(dtype, K, mode, v.m);
    L.rb_rows = std::max(64 * R, loss_chunk(dtype));
    L.xlds = false;
    L.lds = 16;
    L.nrb = (int)((v.m + L.rb_rows - 1) / L.rb_rows);
    L.groups = 1;
    L.tpg = (int)live.size();
  }
  if (!small) {
    const int Kp = kvariant(P->kmax);
    persistent = !no_persistent && mode == MODE_LOSS && debug_stop() == 0 && dtype == SRHIP_F32 &&
                 pick_rows_per_lane(dtype, Kp, mode, v.m) == R_F32_WIDE && R_F32_WIDE != R_F32 &&
                 (nd == 0 || kvariant(P->dkmax) == Kp);
    if (persistent) {
      K = Kp;
      R = R_F32_WIDE;
      const int tile = 64 * R;
      int rb = prb_env >= tile && prb_env <= ROW_ALIGN && (prb_env & (prb_env - 1)) == 0 ? prb_env : 2048;
      rb = std::max(rb, std::max(tile, loss_chunk(dtype)));
      const size_t es = dtype_size(dtype);
      const int base_cols = P->maxfeat + 1 + (weighted ? 1 : 0);
      use_d = nd > 0 && (size_t)(base_cols + nd) * rb * es <= lds_budget(R, K, true);
      const int ncols = base_cols + (use_d ? nd : 0);
      if ((size_t)ncols * rb * es > lds_budget(R, K, false)) {
        persistent = false;  // the block does not fit LDS: grid launch over global reads
        use_d = false;
      } else {
        L.rb_rows = rb;
        L.xlds = true;
        L.lds = (size_t)ncols * rb * es + 16;
        L.nrb = (int)((v.m + rb - 1) / rb);
        L.groups = 1;
        L.tpg = (int)live.size();
        probe_blocks = probe_env >= 0 ? probe_env : 4;
        probe_blocks = L.nrb >= 16 * std::max(1, probe_blocks) ? probe_blocks : 0;
      }
    }
  }
  if (!small && !persistent && nd > 0 && mode != MODE_PRECISE) {
    K = kvariant(P->dkmax);
    R = pick_rows_per_lane(dtype, K, mode, v.m);
    L = plan_launch(ctx, dtype, P->maxfeat + nd, weighted, mode == MODE_LOSS, v.m, (int32_t)live.size(), 64 * R,
                    lds_budget(R, K, true), eval_waves(R, K));
    use_d = L.xlds;
    // ... and only when its columns do not shrink the row block: a wave's early exit of a failed tree
    // saves the rest of its row block, and shorter blocks lose more than the shared columns save
    // (C2, one MI355X, warm, separate processes: 10 columns at 2048-row blocks 1.29 ms vs the plain
    // program at 4096 rows 1.27 ms with 16-wave workgroups; 1.56 vs 1.41 ms at 1024 / 2048 rows with
    // 8-wave workgroups)
    const char* always = env_get("SRHIP_DERIVE_ALWAYS");  // (tests: the derived program whatever the blocks)
    if (use_d && !(always && *always && *always != '0')) {
      const int Kp = kvariant(P->kmax), Rp = pick_rows_per_lane(dtype, Kp, mode, v.m);
      const LaunchPlan Lp = plan_launch(ctx, dtype, P->maxfeat, weighted, mode == MODE_LOSS, v.m, (int32_t)live.size(),
                                        64 * Rp, lds_budget(Rp, Kp, false), eval_waves(Rp, Kp));
      if (Lp.xlds && Lp.rb_rows > L.rb_rows) use_d = false;
    }
  }
  if (!small && !persistent && !use_d) {
    K = kvariant(P->kmax);
    R = pick_rows_per_lane(dtype, K, mode, v.m);
    L = plan_launch(ctx, dtype, P->maxfeat, weighted, mode == MODE_LOSS, v.m, (int32_t)live.size(), 64 * R,
                    lds_budget(R, K, false), eval_waves(R, K));
  }
  const int nl = (int)live.size();
  const void* d_order;
  // persistent launches: one group, the order globally by descending cost (the probe's uniform
  // groups of one tree per wave are consecutive slots of it)
  const std::vector<int32_t> goff = persistent ? std::vector<int32_t>{0, nl} : shape_groups(L, nl, ctx->num_cu);
  {
    std::lock_guard<std::mutex> g(P->ord_mu);
    if (P->upload_pending || P->ord_key[0] != L.groups || P->ord_key[1] != L.tpg || P->ord_key[2] != (int)use_d ||
        P->ord_goff != goff) {
      std::vector<int32_t>& order = P->ord_host;  // lives in the program: the copy below is asynchronous
      order = make_order(*P, live, goff, use_d);
      order.insert(order.end(), goff.begin(), goff.end());  // the group offsets follow the order
      if (P->upload_pending) {  // deferred program upload: program and order in one copy
        const size_t base = P->blob_off[6], bytes = order.size() * sizeof(int32_t);
        P->blob.resize(base + bytes);
        memcpy(P->blob.data() + base, order.data(), bytes);
        HIP_TRY(P->d_prog.ensure(base + bytes));
        HIP_TRY(hipMemcpyAsync(P->d_prog.p, P->blob.data(), base + bytes, hipMemcpyHostToDevice, ctx->stream));
        set_prog_pointers(*P);
        P->upload_pending = false;
        P->ord_dev = (const uint8_t*)P->d_prog.p + base;
      } else {
        HIP_TRY(P->d_order.ensure(order.size() * sizeof(int32_t)));
        HIP_TRY(hipMemcpyAsync(P->d_order.p, order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                               ctx->stream));
        P->ord_dev = P->d_order.p;
      }
      P->ord_key[0] = L.groups;
      P->ord_key[1] = L.tpg;
      P->ord_key[2] = (int)use_d;
      P->ord_goff = goff;
    }
    d_order = P->ord_dev;
  }
  const int nch = (int)((v.m + loss_chunk(dtype) - 1) / loss_chunk(dtype));
  const int cpb = L.rb_rows / loss_chunk(dtype);  // loss chunks per row block (row blocks are whole chunks)
  HIP_TRY(ctx->slab_loss.ensure((size_t)nl * L.nrb * cpb * 8));
  HIP_TRY(ctx->slab_chk.ensure((size_t)nl * L.nrb * 8));
  // the reduction writes the per-tree results straight into coherent pinned host memory (no
  // device-to-host copies on the stream)
  HIP_TRY(rs->h_loss.ensure((size_t)nt * 8, hipHostMallocCoherent));
  HIP_TRY(rs->h_chk.ensure((size_t)nt * 8, hipHostMallocCoherent));
  HIP_TRY(rs->h_rows.ensure((size_t)(nt + 1) * 8, hipHostMallocCoherent));  // [nt]: persistent items evaluated
  EvalArgs a{};
  a.code = use_d ? P->dcode_dev : P->code_dev;
  a.prog_off = use_d ? P->doff_dev : P->off_dev;
  a.order = (const int32_t*)d_order;
  a.nd = use_d ? nd : 0;
  a.dspec = use_d ? P->dspec_dev : nullptr;
  a.dmask = use_d ? P->dmask_dev : nullptr;
  if (dtype == SRHIP_F32) {
    // (every Float32 program carries its trees' +/- bounds: the interpreter folds no +/-)
    if (!P->sbound_dev || P->sbound.size() != 4 * (size_t)P->ntrees)
      return fail(SRHIP_ERR_INVALID, "Float32 program without its +/- bounds");
    J.fbound = feature_bound(v, ds->nfeat);
  }
  a.X = v.X;
  a.y = v.y;
  a.w = weighted ? v.w : nullptr;
  a.slab_loss = ctx->slab_loss.p;
  a.slab_chk = ctx->slab_chk.p;
  a.ld = v.ld;
  a.nvalid = v.m;
  a.ntrees = nl;
  a.nfeat = P->maxfeat;  // staged feature columns
  a.rb_rows = L.rb_rows;
  a.nrb = L.nrb;
  a.nch = nch;
  a.cpb = cpb;
  a.trees_per_group = L.tpg;
  a.group_off = (const int32_t*)d_order + nl;
  a.loss_kind = loss ? loss->kind : 0;
  a.loss_p0 = loss ? loss->p0 : 0.0;
  a.weighted = weighted ? 1 : 0;
  a.has_y = mode == MODE_LOSS ? 1 : 0;
  a.max_steps = use_d ? P->dmax_len : P->max_len;
  a.debug_stop = debug_stop();
  if (small) a.wg_waves = (int)live.size();  // one wave per tree (at most the variant's waves)
  // one row block: the waves finish the per-tree reduction themselves (SRHIP_NO_FUSED_REDUCE=1: the
  // reduce kernel instead; read per launch)
  const char* nofuse = env_get("SRHIP_NO_FUSED_REDUCE");
  if (L.nrb == 1 && !sd && !(nofuse && *nofuse && *nofuse != '0')) {
    a.fused = 1;
    a.fused_loss = mode == MODE_LOSS ? rs->h_loss.p : nullptr;
    a.fused_chk = dtype == SRHIP_I32 ? nullptr : rs->h_chk.p;
    a.fused_rows = (int64_t*)rs->h_rows.p;
  } else {
    HIP_TRY(ctx->slab_rows.ensure((size_t)nl * L.nrb * sizeof(int32_t)));
    a.slab_rows = (int32_t*)ctx->slab_rows.p;
  }
  const bool devp = dp && !a.fused && dtype != SRHIP_I32 && !env_flag("SRHIP_NO_DEVICE_PRECISE");
  // the device list's capacity: DEV_PRECISE_MAX (SRHIP_PRECISE_LIST: smaller, read per call -- the
  // tests' way to the overflow path), less for very long row ranges (ensure_dev_precise)
  int ucap = std::max(1, std::min(DEV_PRECISE_MAX, env_int("SRHIP_PRECISE_LIST", DEV_PRECISE_MAX)));
  if (devp) {
    const int rc = ensure_dev_precise(ctx, P, v, &ucap, rs);
    if (rc) return rc;
  }
  a.early_exit = mode == MODE_LOSS && early_exit_on() ? 1 : 0;
  if (a.early_exit) {
    const int rc = next_fail_epoch(ctx, nl, &a.fail_flag, &a.epoch);
    if (rc) return rc;
  }
  if (trace_on()) {
    HIP_TRY(ctx->h_dbg.ensure(64 * sizeof(int32_t), hipHostMallocCoherent));
    memset(ctx->h_dbg.p, 0xff, 64 * sizeof(int32_t));
    a.dbg = (int32_t*)ctx->h_dbg.p;
  }
  DevBuf& pred = J.pred;
  if (mode == MODE_PRED) {
    HIP_TRY(pred.ensure((size_t)nt * v.m * es));
    a.out_pred = pred.p;
  }
  dim3 grid(L.nrb, (unsigned)goff.size() - 1);
  // a probe with tile claims zeroes the counter itself, so a launch still in flight (an earlier
  // submitted evaluation, not yet seen to drain) needs no fill in front of this one
  const bool probe_zeroes = probe_blocks > 0 && !env_flag("SRHIP_PROBE_TREE_CLAIMS");
  if (persistent && (!ctx->block_ctr.p || (ctx->block_ctr_dirty && !probe_zeroes))) {
    // zeroed once: every persistent launch that drains its claims leaves it at zero (its last claim
    // resets it); again after a launch that was never seen to complete (an error return between the
    // launch and its synchronisation, or a lost row block below)
    // [claim counter, items evaluated]
    HIP_TRY(ctx->block_ctr.ensure(2 * sizeof(int32_t)));
    HIP_TRY(hipMemsetAsync(ctx->block_ctr.p, 0, 2 * sizeof(int32_t), ctx->stream));
    ctx->block_ctr_dirty = false;
  }
  if (persistent) ctx->block_ctr_dirty = true;  // until the launch is seen to have drained
  if (sd) HIP_TRY(hipMemsetAsync(sd->d_loss, 0, sd->zero_bytes, ctx->stream));
  HIP_TRY(hipEventRecord(rs->ev0, ctx->stream));
  if (persistent) {
    if (probe_blocks > 0) {
      // leading row blocks, one tree per wave (uniform groups of consecutive slots), with the plain
      // program: a probe workgroup serves 16 trees, too few to pay for deriving columns (the values,
      // partials and slots are the same either way)
      // workgroup (b, g) of the probe takes slots g, g + G, g + 2G, ... (grid_interleave): each CU
      // gets one of the most expensive trees and cheap ones, not 16 of the most expensive (which
      // four waves per SIMD would share)
      EvalArgs q = a;
      q.group_off = nullptr;
      q.trees_per_group = eval_waves(R, K);
      q.grid_interleave = 1;
      // one (tree, tile) per claim: the costliest tree's two tiles run on two waves at once (the
      // probe's duration is that tree's); chk / rows of the probe blocks combine by atomics from 0
      // (the probe's workgroups zero their own combining entries and the persistent launch's block
      // counter: no memset launches on the stream)
      if (probe_zeroes) {
        q.tile_claims = 1;
        q.zero_ctr = (int32_t*)ctx->block_ctr.p;
      }
      q.code = P->code_dev;
      q.prog_off = P->off_dev;
      q.max_steps = P->max_len;
      q.nd = 0;
      q.dspec = nullptr;
      q.dmask = nullptr;
      const size_t qlds = (size_t)(P->maxfeat + 1 + (weighted ? 1 : 0)) * L.rb_rows * es + 16;
      const dim3 pgrid(probe_blocks, (unsigned)((nl + q.trees_per_group - 1) / q.trees_per_group));
      HIP_TRY(launch_eval(dtype, q, R, K, mode, true, pgrid, qlds, ctx->stream));
    }
    a.persistent = 1;
    a.block0 = probe_blocks;
    a.block_ctr = (int32_t*)ctx->block_ctr.p;
    // (diagnostic, tests only) a counter left non-zero when the main launch starts (after the probe,
    // which zeroes it): the launch skips that many row blocks, which the lost-block check after it must
    // report
    if (const int seed = env_int("SRHIP_DEBUG_BLOCK_CTR", 0)) {
      const int32_t h = (int32_t)seed;
      HIP_TRY(hipMemcpyAsync(ctx->block_ctr.p, &h, sizeof(h), hipMemcpyHostToDevice, ctx->stream));
      HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    const int nmain = L.nrb - probe_blocks;
    const int wgs = std::max(1, std::min(nmain, ctx->num_cu));
    // SRHIP_TAIL_SLICES = S > 1: the row blocks past the last whole round of workgroups are claimed
    // as S interleaved population slices each (C2's 485 blocks on 256 workgroups leave 229 for a
    // second round that idles 27 CUs for a block).  Default 1 (whole blocks): every slice restages
    // the block and re-derives its columns, and that costs more than the idle CUs (C2, same box:
    // S = 1 1.215 ms, 8 1.250, 16 1.278)
    const int slices_env = env_int("SRHIP_TAIL_SLICES", 1);
    const int slices = std::max(1, std::min(slices_env, 64));
    a.tail_slices = slices;
    a.tail_blocks = slices > 1 && nmain > wgs && nl >= 16 * slices ? nmain % wgs : 0;
    J.expect_items = nmain - a.tail_blocks + a.tail_blocks * slices;
    HIP_TRY(launch_eval(dtype, a, R, K, mode, true, dim3(wgs, 1), L.lds, ctx->stream));
  } else {
    HIP_TRY(launch_eval(dtype, a, R, K, mode, L.xlds, grid, L.lds, ctx->stream));
  }
  HIP_TRY(hipEventRecord(rs->ev1, ctx->stream));
  J.launched = true;
  J.persistent = persistent;
  J.devp = devp;
  if (trace_on()) {  // poll the kernel's progress words for up to 10 s, then abort loudly
    const volatile int32_t* d = (const volatile int32_t*)ctx->h_dbg.p;
    int32_t last[16];
    for (int i = 0; i < 16; ++i) last[i] = -2;
    for (int it = 0; it < 10000; ++it) {
      hipError_t q = hipStreamQuery(ctx->stream);
      bool changed = false;
      for (int i = 0; i < 16; ++i) changed |= d[i] != last[i];
      if (changed) {
        for (int i = 0; i < 16; ++i) last[i] = d[i];
        fprintf(stderr, "[srhip] kernel progress: stage=%d tree=%d waves=%d,%d,%d,%d,%d,%d,%d,%d\n", last[0], last[1],
                last[8], last[9], last[10], last[11], last[12], last[13], last[14], last[15]);
        fflush(stderr);
      }
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) HIP_TRY(q);
      usleep(1000);
      if (it == 9999) {
        fprintf(stderr, "[srhip] kernel did not finish in 10 s; aborting\n");
        fflush(stderr);
        abort();
      }
    }
  }
  UndecidedList& ul = J.ul;
  int ul_groups = 4;
  if (devp) {
    if (!ctx->d_ulist.p) {
      // [count, DEV_PRECISE_MAX trees, the precise reduction's finished-workgroup counter]
      HIP_TRY(ctx->d_ulist.ensure((2 + DEV_PRECISE_MAX) * sizeof(int32_t)));
      HIP_TRY(hipMemsetAsync(ctx->d_ulist.p, 0, ctx->d_ulist.bytes, ctx->stream));
    }
    ul.ulist = (int32_t*)ctx->d_ulist.p;
    // trees past the list's capacity are settled by the same pass over a host-written list (run_eval).
    // The precise launch's workgroups per row block: the program's last count plus two (4 at least)
    ul.umax = ucap;
    ul.rows = (double)v.m;
    ul_groups = std::min(ul.umax, std::max(4, P->und_hint + 2));
  }
  J.fused = a.fused != 0;
  if (dtype == SRHIP_F32) {  // the reduction raises each tree's statistic to its +/- bound
    ul.sbound = P->sbound_dev;
    ul.fbound = J.fbound;
  }
  if (!a.fused)
    HIP_TRY(launch_reduce(dtype, mode == MODE_LOSS ? ctx->slab_loss.p : nullptr, nch, cpb,
                          dtype == SRHIP_I32 ? nullptr : ctx->slab_chk.p, L.nrb, nl, (const int32_t*)d_order,
                          mode == MODE_LOSS ? (sd ? sd->d_loss : rs->h_loss.p) : nullptr,
                          dtype == SRHIP_I32 ? nullptr : (sd ? sd->d_chk : rs->h_chk.p), ctx->stream, a.slab_rows,
                          (int64_t*)rs->h_rows.p, ul, sd != nullptr,
                          persistent ? (int32_t*)ctx->block_ctr.p + 1 : nullptr,
                          persistent ? (int64_t*)rs->h_rows.p + nt : nullptr));
  if (devp) {
    int stride = 1;
    const int rc = enqueue_dev_precise(ctx, ds, P, v, ul.ulist, ul.umax, ul_groups, &stride, rs);
    if (rc) return rc;
    dp->used = true;
    dp->stride = stride;
  }
  if (mode == MODE_PRED)
    HIP_TRY(hipMemcpyAsync(out_pred, pred.p, (size_t)nt * v.m * es, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipEventRecord(rs->done, ctx->stream));
  return SRHIP_OK;
}

// The second half: the records of a job whose work has completed (the caller waited for its stream or
// its result set's completion event).
static int eval_collect(srhip_ctx* ctx, const srhip_program* P, const View& v, double* sums, double* chk,
                        DevPrecise* dp, ShardDev* sd, EvalJob& J) {
  ResultSet* const rs = J.rs;
  const int dtype = J.dtype, mode = J.mode;
  const int32_t nt = J.nt;
  const std::vector<int32_t>& live = J.live;
  const bool persistent = J.persistent, devp = J.devp;
  const UndecidedList& ul = J.ul;
  ctx->last_ev0 = rs->ev0;
  ctx->last_ev1 = rs->ev1;
  ctx->timed = true;
  if (devp) {
    const int32_t* hl = (const int32_t*)rs->h_pout.p;
    const double* hs = (const double*)((const uint8_t*)rs->h_pout.p + PREC_SUMS_OFF);
    dp->count = hl[0];
    P->und_hint = dp->count;
    const int nu = std::min(dp->count, ul.umax);
    dp->list.assign(hl + 1, hl + 1 + nu);
    dp->opsums.assign(hs, hs + (size_t)nu * dp->stride);
  }
  // the reduction's records, read from the device-written (coherent) host buffers in bulk copies:
  // line-sized reads, not one uncached access per tree
  static thread_local std::vector<uint64_t> r_loss, r_chk, r_rows;
  r_loss.resize(nt);
  r_chk.resize(nt);
  r_rows.resize(nt);
  if (mode == MODE_LOSS) memcpy(r_loss.data(), rs->h_loss.p, (size_t)nt * 8);
  if (dtype != SRHIP_I32) memcpy(r_chk.data(), rs->h_chk.p, (size_t)nt * (dtype == SRHIP_F32 ? 4 : 8));
  memcpy(r_rows.data(), rs->h_rows.p, (size_t)nt * 8);
  for (int32_t t : live) {
    if (sd) break;  // the shard's loss sums and statistics are in the exchange's device buffer
    if (mode == MODE_LOSS)
      sums[2 * (size_t)t] = dtype == SRHIP_I32 ? (double)((const long long*)r_loss.data())[t] : ((const double*)r_loss.data())[t];
    if (dtype == SRHIP_F32) {
      const float m = ((const float*)r_chk.data())[t];
      // a single-block launch's records come straight from the interpreter: its +/- bound applied here
      chk[t] = J.fused ? skip_bound_apply(m, P->sbound.data() + 4 * (size_t)t, J.fbound) : m;
    } else if (dtype == SRHIP_F64) {
      chk[t] = ((const double*)r_chk.data())[t];
    }
  }
  if (persistent) {
    // every row block was claimed exactly once: the workgroups' evaluated items add up to the launch's
    // item count (a counter left non-zero by a launch that never drained would make this one skip
    // blocks silently -- and leave the skipped blocks' stale partials in the slabs)
    const int64_t done = ((const int64_t*)rs->h_rows.p)[nt];
    if (done != J.expect_items)
      return fail(SRHIP_ERR_DEVICE, "persistent launch evaluated %lld of %d row-block items (row-block counter "
                  "not at zero); the counter is reset for the next launch", (long long)done, (int)J.expect_items);
    ctx->block_ctr_dirty = false;
  }
  // the launch's work, counted on the device (rows each tree was evaluated on)
  for (int i = 0; i < 4; ++i) ctx->work[i] = 0;
  const bool pdec = P->dec.size() == (size_t)nt;
  for (int32_t t : live) {
    const int64_t rows = ((const int64_t*)r_rows.data())[t];
    const int64_t nn = pdec ? P->dec[t].nnodes : P->info[t].nnodes, no = pdec ? P->dec[t].nops : P->info[t].nops;
    ctx->work[0] += rows * nn;
    ctx->work[1] += v.m * nn;
    ctx->work[2] += rows * no;
    ctx->work[3] += rows;
  }
  g_tail_done = std::chrono::steady_clock::now();
  return SRHIP_OK;
}

// Device stage, synchronous: the launches, the wait, the records (result set 0).
static int eval_partials(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode, const srhip_loss* loss,
                         const View& v, void* out_pred, double* sums, double* chk, DevPrecise* dp = nullptr,
                         ShardDev* sd = nullptr) {
  EvalJob J;
  J.rs = &ctx->rs[0];
  int rc = eval_issue(ctx, ds, P, mode, loss, v, out_pred, sums, chk, dp, sd, J);
  if (rc || !J.launched) return rc;
  rc = stream_wait(ctx);
  if (rc) return rc;
  return eval_collect(ctx, P, v, sums, chk, dp, sd, J);
}

// Precise stage: per-(tree, operator node) f64 sums over the view's rows for the selected trees;
// opsums[u * max(1, max_ops) + k].
static int eval_precise(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const View& v,
                        const int32_t* trees, int32_t nu, double* opsums, bool grad = false) {
  const int dtype = P->dtype;
  const int stride = std::max(1, grad ? P->gmax_ops : P->max_ops);
  for (size_t i = 0; i < (size_t)nu * stride; ++i) opsums[i] = 0.0;
  if (nu == 0 || dtype == SRHIP_I32) return SRHIP_OK;
  const int R = pick_rows_per_lane(dtype, K_MAX, MODE_PRECISE, v.m);
  LaunchPlan Lp = plan_launch(ctx, dtype, ds->nfeat, false, false, v.m, nu, 64 * R);
  Lp.groups = 1;
  Lp.tpg = nu;
  const size_t slab_bytes = (size_t)nu * stride * Lp.nrb * sizeof(double);
  HIP_TRY(ctx->slab_prec.ensure(slab_bytes));
  HIP_TRY(hipMemsetAsync(ctx->slab_prec.p, 0, slab_bytes, ctx->stream));
  // the list [count | trees | the reduction's finished-workgroup counter] in one copy from pinned
  // staging: the precise launch reads the trees, precise_reduce_kernel the count and the counter
  HIP_TRY(ctx->h_plist.ensure((size_t)(nu + 2) * sizeof(int32_t)));
  int32_t* hlist = (int32_t*)ctx->h_plist.p;
  hlist[0] = nu;
  memcpy(hlist + 1, trees, (size_t)nu * sizeof(int32_t));
  hlist[1 + nu] = 0;
  HIP_TRY(ctx->order_prec.ensure((size_t)(nu + 2) * sizeof(int32_t)));
  HIP_TRY(hipMemcpyAsync(ctx->order_prec.p, hlist, (size_t)(nu + 2) * sizeof(int32_t), hipMemcpyHostToDevice,
                         ctx->stream));
  EvalArgs a{};
  a.code = grad ? (const Ins*)P->d_gcode.p : P->code_dev;
  a.prog_off = grad ? (const int32_t*)P->d_goff.p : P->off_dev;
  a.order = (const int32_t*)ctx->order_prec.p + 1;
  a.X = v.X;
  a.ld = v.ld;
  a.nvalid = v.m;
  a.ntrees = nu;
  a.nfeat = (int32_t)ds->nfeat;
  a.rb_rows = Lp.rb_rows;
  a.nrb = Lp.nrb;
  a.trees_per_group = nu;
  a.slab_prec = ctx->slab_prec.p;
  a.prec_stride = stride;
  a.max_steps = grad ? P->gmax_len : P->max_len;
  HIP_TRY(launch_eval(dtype, a, R, K_MAX, MODE_PRECISE, false, dim3(Lp.nrb, 1), 16, ctx->stream));
  // per-(tree, operator) sums over the row blocks on the device (precise_reduce_kernel: compensated
  // double-double in a fixed order, as the device-listed pass), into coherent host memory -- round 6:
  // the whole slab copied back and summed on the host in long double cost ~0.3 ms per tree at 10M rows
  // (row-shard steps)
  const size_t off = ((size_t)(nu + 1) * sizeof(int32_t) + 15) & ~(size_t)15;
  HIP_TRY(ctx->h_prec.ensure(off + (size_t)nu * stride * sizeof(double), hipHostMallocCoherent));
  HIP_TRY(launch_precise_reduce((const double*)ctx->slab_prec.p, Lp.nrb, stride, (int32_t*)ctx->order_prec.p, nu, nu,
                                nu, (int32_t*)ctx->h_prec.p, (double*)((uint8_t*)ctx->h_prec.p + off), ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  memcpy(opsums, (const uint8_t*)ctx->h_prec.p + off, (size_t)nu * stride * sizeof(double));
  return SRHIP_OK;
}

int srhip::precise_decide(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const View& v,
                          const int32_t* trees, int32_t nu, bool grad, uint8_t* out_ok) {
  if (nu <= 0) return SRHIP_OK;
  const int stride = std::max(1, grad ? P->gmax_ops : P->max_ops);
  std::vector<double> opsums((size_t)nu * stride);
  const int rc = eval_precise(ctx, ds, P, v, trees, nu, opsums.data(), grad);
  if (rc) return rc;
  finalize_precise(*P, trees, nu, opsums.data(), out_ok, grad);
  return SRHIP_OK;
}

int srhip::gathered_weight_sum(srhip_ctx* ctx, const srhip_dataset* ds, int64_t nidx, View& v) {
  std::vector<unsigned char> wbuf((size_t)nidx * dtype_size(ds->dtype));
  HIP_TRY(hipMemcpy(wbuf.data(), ctx->vw.p, wbuf.size(), hipMemcpyDeviceToHost));
  double s = 0.0;
  for (int64_t i = 0; i < nidx; ++i)
    s += ds->dtype == SRHIP_F64 ? ((double*)wbuf.data())[i] : (double)((float*)wbuf.data())[i];
  v.sum_w = s;
  return SRHIP_OK;
}

// (diagnostic) SRHIP_HOST_TIMING=1: run_eval's host time before the wait (argument checks, view,
// schedule, launches), in the wait, and after it (decisions), averaged over every 50 calls on stderr
int srhip::stream_wait(srhip_ctx* ctx) {
  g_wait_begin = std::chrono::steady_clock::now();
  static const bool spin = env_flag("SRHIP_SYNC_SPIN");
  if (!spin || !ctx->ev_sync) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    g_wait_done = std::chrono::steady_clock::now();
    return SRHIP_OK;
  }
  HIP_TRY(hipEventRecord(ctx->ev_sync, ctx->stream));
  for (;;) {
    const hipError_t q = hipEventQuery(ctx->ev_sync);
    if (q == hipSuccess) {
      g_wait_done = std::chrono::steady_clock::now();
      return SRHIP_OK;
    }
    if (q != hipErrorNotReady) HIP_TRY(q);
    __builtin_ia32_pause();
  }
}

// Single-device evaluation: partials -> decision -> precise pass for undecided trees, as two halves --
// run_issue (arguments, view, launches) and run_complete (records, decisions, the precise passes the
// device did not settle, outputs) -- so that srhip_eval_loss_submit can return between them.
struct RunJob {
  EvalJob J;
  View v{};
  std::vector<double> sums, chk;
  DevPrecise dp;
  const srhip_dataset* ds = nullptr;
  const srhip_program* P = nullptr;
  int mode = 0;
  bool empty = false;  // no trees: nothing to decide
};
static int run_issue(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode, const srhip_loss* loss,
                     const int64_t* idx, int64_t nidx, void* out_pred, RunJob& R) {
  int rc = check_eval_args(ctx, ds, P, mode, loss);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  R.ds = ds;
  R.P = P;
  R.mode = mode;
  rc = make_view(ctx, ds, idx, nidx, mode == MODE_LOSS, R.v);
  if (rc) return rc;
  if (idx && ds->weighted && mode == MODE_LOSS) {
    rc = gathered_weight_sum(ctx, ds, nidx, R.v);
    if (rc) return rc;
  }
  const int32_t nt = P->ntrees;
  if (nt == 0) {
    R.empty = true;
    return SRHIP_OK;
  }
  R.sums.assign(sums_len(nt, ds->nfeat), 0.0);
  R.chk.assign(nt, 0.0);
  return eval_issue(ctx, ds, P, mode, loss, R.v, out_pred, R.sums.data(), R.chk.data(), &R.dp, nullptr, R.J);
}
static int run_complete(srhip_ctx* ctx, RunJob& R, double* out_loss, uint8_t* out_ok) {
  if (R.empty) return SRHIP_OK;
  const srhip_dataset* ds = R.ds;
  const srhip_program* P = R.P;
  const View& v = R.v;
  std::vector<double>& sums = R.sums;
  DevPrecise& dp = R.dp;
  int rc = SRHIP_OK;
  if (R.J.launched) {
    rc = eval_collect(ctx, P, v, sums.data(), R.chk.data(), &dp, nullptr, R.J);
    if (rc) return rc;
  }
  const int32_t nt = P->ntrees;
  std::vector<uint8_t> status(nt), ok(nt);
  std::vector<double> lossv(nt);
  finalize(*P, ds->nfeat, sums.data(), R.chk.data(), lossv.data(), ok.data(), status.data());
  std::vector<int32_t> unc;
  for (int32_t t = 0; t < nt; ++t)
    if (status[t] == 2) unc.push_back(t);
  if (dp.used && !unc.empty()) {
    // undecided trees the device's precise pass already covered (every undecided tree is listed by
    // the device: its test is the host's minus the host-only checks, so the list is a superset)
    std::vector<int32_t> rest;
    for (int32_t t : unc) {
      const auto it = std::find(dp.list.begin(), dp.list.end(), t);
      if (it == dp.list.end()) {
        rest.push_back(t);
        continue;
      }
      const size_t u = (size_t)(it - dp.list.begin());
      uint8_t uok = 0;
      finalize_precise(*P, &t, 1, dp.opsums.data() + u * dp.stride, &uok);
      ok[t] = uok;
      lossv[t] = uok ? sums[2 * (size_t)t] / sums[2 * (size_t)t + 1] : INFINITY;
    }
    unc.swap(rest);
  }
  // trees past the device list's capacity (a program's first evaluation lists at most 4): the same
  // device-listed pass over a host-written list, DEV_PRECISE_MAX trees at a time -- every undecided
  // tree of a device evaluation is then settled by one summation path (SRHIP_PRECISE_OVERFLOW_HOST=1:
  // the host-launched pass of eval_precise instead).  (A submitted evaluation reaches this after the
  // work queued behind it; its view is the whole dataset -- submits of row subsets complete at once --
  // and its results land in its own result set.)
  ResultSet* const rs = R.J.rs;
  if (dp.used && !unc.empty() && !env_flag("SRHIP_PRECISE_OVERFLOW_HOST")) {
    const size_t bcap = (size_t)precise_cap(P, v, DEV_PRECISE_MAX);
    for (size_t b = 0; b < unc.size(); b += bcap) {
      const int32_t n = (int32_t)std::min<size_t>(bcap, unc.size() - b);
      std::vector<int32_t> lst(1 + n);
      lst[0] = n;
      std::copy(unc.begin() + b, unc.begin() + b + n, lst.begin() + 1);
      HIP_TRY(hipMemcpyAsync(ctx->d_ulist.p, lst.data(), lst.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                             ctx->stream));
      int stride = 1;
      rc = enqueue_dev_precise(ctx, ds, P, v, (int32_t*)ctx->d_ulist.p, n, n, &stride, rs);
      if (rc) return rc;
      rc = stream_wait(ctx);
      if (rc) return rc;
      const int32_t* hl = (const int32_t*)rs->h_pout.p;
      const double* hs = (const double*)((const uint8_t*)rs->h_pout.p + PREC_SUMS_OFF);
      if (hl[0] != n) return fail(SRHIP_ERR_DEVICE, "precise pass listed %d of %d trees", (int)hl[0], (int)n);
      for (int32_t u = 0; u < n; ++u) {
        const int32_t t = hl[1 + u];
        uint8_t uok = 0;
        finalize_precise(*P, &t, 1, hs + (size_t)u * stride, &uok);
        ok[t] = uok;
        lossv[t] = uok ? sums[2 * (size_t)t] / sums[2 * (size_t)t + 1] : INFINITY;
      }
    }
    unc.clear();
  }
  if (!unc.empty()) {
    const int stride = std::max(1, P->max_ops);
    std::vector<double> opsums(unc.size() * stride);
    rc = eval_precise(ctx, ds, P, v, unc.data(), (int32_t)unc.size(), opsums.data());
    if (rc) return rc;
    std::vector<uint8_t> uok(unc.size());
    finalize_precise(*P, unc.data(), (int32_t)unc.size(), opsums.data(), uok.data());
    for (size_t u = 0; u < unc.size(); ++u) {
      const int32_t t = unc[u];
      ok[t] = uok[u];
      lossv[t] = uok[u] ? sums[2 * (size_t)t] / sums[2 * (size_t)t + 1] : INFINITY;
    }
  }
  for (int32_t t = 0; t < nt; ++t) {
    if (out_ok) out_ok[t] = ok[t];
    if (out_loss) out_loss[t] = lossv[t];
  }
  return SRHIP_OK;
}

int srhip::run_eval(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, int mode, const srhip_loss* loss,
                    const int64_t* idx, int64_t nidx, double* out_loss, void* out_pred, uint8_t* out_ok) {
  static const bool timing = env_flag("SRHIP_HOST_TIMING");
  const auto t_entry = std::chrono::steady_clock::now();
  struct Report {  // on every return path
    bool on;
    std::chrono::steady_clock::time_point t0;
    ~Report() {
      if (!on) return;
      static thread_local double acc[4];
      static thread_local int cnt;
      const auto t3 = std::chrono::steady_clock::now();
      acc[0] += std::chrono::duration<double>(g_wait_begin - t0).count();
      acc[1] += std::chrono::duration<double>(g_wait_done - g_wait_begin).count();
      acc[2] += std::chrono::duration<double>(g_tail_done - g_wait_done).count();
      acc[3] += std::chrono::duration<double>(t3 - g_tail_done).count();
      static const bool each = [] {  // SRHIP_HOST_TIMING=2: every call
        const char* e = getenv("SRHIP_HOST_TIMING");
        return e && atoi(e) >= 2;
      }();
      if (++cnt % (each ? 1 : 50) == 0) {
        fprintf(stderr, "[srhip host] run_eval: before wait %.1f us, wait %.1f us, records %.1f us, decisions %.1f us "
                "(mean of %d)\n", acc[0] / cnt * 1e6, acc[1] / cnt * 1e6, acc[2] / cnt * 1e6, acc[3] / cnt * 1e6, cnt);
        acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
        cnt = 0;
      }
    }
  } report{timing, t_entry};
  RunJob R;
  R.J.rs = &ctx->rs[0];
  int rc = run_issue(ctx, ds, P, mode, loss, idx, nidx, out_pred, R);
  if (rc) return rc;
  if (R.J.launched) {
    rc = stream_wait(ctx);
    if (rc) return rc;
  }
  return run_complete(ctx, R, out_loss, out_ok);
}

// Row-sharded evaluation (srhip_eval_loss_sharded): this shard's partials written by the reduction
// into the exchange's device buffer [loss | chk | aux], ONE all-reduce group of it in place (loss sums
// SUM, chk MAX for Float32 / SUM otherwise -- a non-finite statistic stored as +Inf -- and the aux
// entries SUM: the weight sum, the feature statistics, the row count), one copy to the host, and the
// decision every rank takes identically from the same reduced values; for undecided trees a precise pass
// over this shard with a SUM all-reduce of its per-operator sums.  The exchanges are the caller's
// (srhip_comm.cpp: RCCL on the device); nfeat is the dataset's feature count on every rank.
int srhip::run_eval_sharded(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const srhip_loss* loss,
                            const int64_t* idx, int64_t nidx, const ShardIO& io, double* out_loss, uint8_t* out_ok) {
  int rc = check_eval_args(ctx, ds, P, MODE_LOSS, loss);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  View v;
  rc = make_view(ctx, ds, idx, nidx, true, v);
  if (rc) return rc;
  if (idx && ds->weighted) {
    rc = gathered_weight_sum(ctx, ds, nidx, v);
    if (rc) return rc;
  }
  const int32_t nt = P->ntrees;
  if (nt == 0) return SRHIP_OK;
  const int64_t nf = ds->nfeat;
  const size_t ns = sums_len(nt, nf);
  ShardLayout SL;
  SL.dtype = P->dtype;
  SL.nt = (size_t)nt;
  SL.naux = 2 + 2 * (size_t)nf;  // [weight sum | feature stats (2F) | rows]
  void* dbuf = nullptr;
  rc = io.buffer(SL.bytes(), &dbuf);
  if (rc) return rc;
  ShardDev sd;
  sd.d_loss = dbuf;
  sd.d_chk = (uint8_t*)dbuf + SL.chk_off();
  sd.zero_bytes = SL.chk_off() + SL.nt * SL.chk_size();
  std::vector<double> sums(ns, 0.0), chk(nt, 0.0);
  rc = eval_partials(ctx, ds, P, MODE_LOSS, loss, v, nullptr, sums.data(), chk.data(), nullptr, &sd);
  if (rc) return rc;
  // the host-known entries (the same for every tree): weight sum, feature statistics, rows
  std::vector<double> aux(SL.naux);
  aux[0] = sums[1];
  for (size_t i = 0; i < 2 * (size_t)nf + 1; ++i) aux[1 + i] = sums[2 * (size_t)nt + i];
  const void* red = nullptr;
  rc = io.reduce(SL, aux.data(), &red);
  if (rc) return rc;
  const uint8_t* rb = (const uint8_t*)red;
  const double* raux = (const double*)(rb + SL.aux_off());
  for (int32_t t = 0; t < nt; ++t) {
    sums[2 * (size_t)t] = P->dtype == SRHIP_I32 ? (double)((const long long*)rb)[t] : ((const double*)rb)[t];
    sums[2 * (size_t)t + 1] = raux[0];
    if (P->dtype == SRHIP_F32) chk[t] = ((const float*)(rb + SL.chk_off()))[t];
    else if (P->dtype == SRHIP_F64) chk[t] = ((const double*)(rb + SL.chk_off()))[t];
  }
  for (size_t i = 0; i < 2 * (size_t)nf + 1; ++i) sums[2 * (size_t)nt + i] = raux[1 + i];
  // (this shard's persistent launch was checked to have evaluated every row block by eval_collect,
  // from its own item count -- not from the all-reduced statistic, which another shard's failures can
  // make non-finite: ADVICE r05)
  std::vector<uint8_t> status(nt), ok(nt);
  std::vector<double> lossv(nt);
  finalize(*P, nf, sums.data(), chk.data(), lossv.data(), ok.data(), status.data());
  std::vector<int32_t> unc;
  for (int32_t t = 0; t < nt; ++t)
    if (status[t] == 2) unc.push_back(t);
  // every rank took the same decision from the same reduced partials: the undecided set agrees, and so
  // does whether the second exchange happens.  (The single-device path lists undecided trees on the
  // device; here the list depends on the all-reduced statistic, which the host already holds.)
  if (!unc.empty()) {
    const int stride = std::max(1, P->max_ops);
    std::vector<double> opsums(unc.size() * stride);
    rc = eval_precise(ctx, ds, P, v, unc.data(), (int32_t)unc.size(), opsums.data());
    if (rc) return rc;
    rc = io.reduce_host(opsums.data(), opsums.size());
    if (rc) return rc;
    std::vector<uint8_t> uok(unc.size());
    finalize_precise(*P, unc.data(), (int32_t)unc.size(), opsums.data(), uok.data());
    for (size_t u = 0; u < unc.size(); ++u) {
      const int32_t t = unc[u];
      ok[t] = uok[u];
      lossv[t] = uok[u] ? sums[2 * (size_t)t] / sums[2 * (size_t)t + 1] : INFINITY;
    }
  }
  for (int32_t t = 0; t < nt; ++t) {
    if (out_ok) out_ok[t] = ok[t];
    if (out_loss) out_loss[t] = lossv[t];
  }
  return SRHIP_OK;
}

// The launch order a fresh Float32 program's first large evaluation will use (eval_partials'
// persistent plan: one group, the live trees by descending cost, derived columns when they fit), made
// at creation -- on the thread that compiles, which in a pipeline overlaps the previous population's
// evaluation -- and uploaded with the program in its one copy, instead of sorting and copying it (a
// pageable-source copy the runtime stages synchronously) in front of the first launch.  Assumes an
// unweighted dataset of >= WIDE_MIN_ROWS rows; any other launch re-plans as before (the key differs).
static void plan_persistent_order(const srhip_ctx* ctx, srhip_program& P) {
  if (!ctx || P.dtype != SRHIP_F32 || P.ntrees == 0) return;
  if (env_flag("SRHIP_NO_PERSISTENT") || env_flag("SRHIP_NO_PREPLAN")) return;
  bool wide = false;
  for (int32_t u : P.unaops) wide |= u == SRHIP_OP_ASIN || u == SRHIP_OP_ACOS || u == SRHIP_OP_ATANH_CLIP;
  auto kvariant = [&](int32_t kmax) { return wide ? K_MAX : (kmax <= 2 ? 2 : (kmax <= 4 ? 4 : 8)); };
  const int nd = (int)P.dspec.size();
  const int Kp = kvariant(P.kmax);
  if (pick_rows_per_lane(SRHIP_F32, Kp, MODE_LOSS, WIDE_MIN_ROWS) != R_F32_WIDE || R_F32_WIDE == R_F32) return;
  if (nd != 0 && kvariant(P.dkmax) != Kp) return;
  const int prb_env = env_int("SRHIP_PRB_ROWS", 0);
  const int tile = 64 * R_F32_WIDE;
  int rb = prb_env >= tile && prb_env <= ROW_ALIGN && (prb_env & (prb_env - 1)) == 0 ? prb_env : 2048;
  rb = std::max(rb, std::max(tile, loss_chunk(SRHIP_F32)));
  const size_t budget = (size_t)ctx->lds_max - 8 * 1024;  // the 16-wave variant: one workgroup per CU
  const int base_cols = P.maxfeat + 1;
  const bool use_d = nd > 0 && (size_t)(base_cols + nd) * rb * 4 <= budget;
  if ((size_t)(base_cols + (use_d ? nd : 0)) * rb * 4 > budget) return;
  std::vector<int32_t> live;
  live.reserve(P.ntrees);
  for (int32_t t = 0; t < P.ntrees; ++t)
    if (!P.info[t].static_fail) live.push_back(t);
  if (live.empty()) return;
  const int nl = (int)live.size();
  const std::vector<int32_t> goff{0, nl};
  std::lock_guard<std::mutex> g(P.ord_mu);
  P.ord_host = make_order(P, live, goff, use_d);
  P.ord_host.insert(P.ord_host.end(), goff.begin(), goff.end());
  P.ord_key[0] = 1;
  P.ord_key[1] = nl;
  P.ord_key[2] = (int)use_d;
  P.ord_goff = goff;
}

// ---- deferred program teardown (srhip_program_destroy) -------------------------------------------
namespace {
struct Reaper {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<srhip_program*> q;
  bool started = false;
};
Reaper& reaper() {
  static Reaper* R = new Reaper();  // never destroyed: the thread may outlive static destruction
  return *R;
}
}  // namespace

static void reaper_push(srhip_program* P) {
  Reaper& R = reaper();
  std::lock_guard<std::mutex> g(R.mu);
  R.q.push_back(P);
  if (!R.started) {
    R.started = true;
    std::thread([&R] {
      for (;;) {
        std::vector<srhip_program*> batch;
        {
          std::unique_lock<std::mutex> lk(R.mu);
          R.cv.wait(lk, [&R] { return !R.q.empty(); });
          batch.swap(R.q);
        }
        for (srhip_program* p : batch) {
          if (p->device >= 0) (void)hipSetDevice(p->device);
          delete p;
        }
      }
    }).detach();
  }
  R.cv.notify_one();
}

template <typename T>
static void pack_column(const void* src, int64_t f, int64_t n, int64_t sf, int64_t sr, int64_t ld, T* dst) {
  const T* s = (const T*)src;
  for (int64_t j = 0; j < n; ++j) dst[j] = s[f * sf + j * sr];
  for (int64_t j = n; j < ld; ++j) dst[j] = dst[n - 1];
}

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
extern "C" {

const char* srhip_last_error(void) { return srhip::last_error(); }
const char* srhip_version(void) { return "srhip 0.1.0 gfx950"; }

int srhip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int srhip_ctx_create(int device, srhip_ctx** out) {
  if (!out) return fail(SRHIP_ERR_INVALID, "null out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(SRHIP_ERR_DEVICE, "no HIP device available");
  if (device < 0 || device >= n) return fail(SRHIP_ERR_INVALID, "device %d out of range (%d devices)", device, n);
  std::unique_ptr<srhip_ctx> c(new srhip_ctx());
  c->device = device;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  c->num_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  int lds_max = 0;
  if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lds_max > 0)
    c->lds_max = lds_max;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(SRHIP_ERR_UNSUPPORTED, "device %d is %s; libsrhip is built for gfx950 only", device, prop.gcnArchName);
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming));
  for (ResultSet& r : c->rs) {
    HIP_TRY(hipEventCreate(&r.ev0));
    HIP_TRY(hipEventCreate(&r.ev1));
    HIP_TRY(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
  }
  HIP_TRY(hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking));
  *out = c.release();
  return SRHIP_OK;
}

void srhip_ctx_destroy(srhip_ctx* ctx) {
  if (!ctx) return;
  for (srhip_ctx* a : ctx->aux) srhip_ctx_destroy(a);
  ctx->aux.clear();
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->ev_sync) (void)hipEventDestroy(ctx->ev_sync);
  for (ResultSet& r : ctx->rs)
    for (hipEvent_t e : {r.ev0, r.ev1, r.done})
      if (e) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->up_stream) (void)hipStreamDestroy(ctx->up_stream);
  delete ctx;
  (void)hipGetLastError();
}

int srhip_ctx_synchronize(srhip_ctx* ctx) {
  if (!ctx) return fail(SRHIP_ERR_INVALID, "null ctx");
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return SRHIP_OK;
}

int srhip_dataset_create(srhip_ctx* ctx, int dtype, const void* X, int64_t nfeat, int64_t n, int64_t sf, int64_t sr,
                         const void* y, const void* w, srhip_dataset** out) {
  if (!ctx || !out) return fail(SRHIP_ERR_INVALID, "null argument");
  *out = nullptr;
  if (dtype != SRHIP_F32 && dtype != SRHIP_F64 && dtype != SRHIP_I32) return fail(SRHIP_ERR_UNSUPPORTED, "dtype %d", dtype);
  if (n <= 0) return fail(SRHIP_ERR_INVALID, "dataset needs n >= 1 rows");
  if (nfeat < 0 || nfeat > 65535) return fail(SRHIP_ERR_INVALID, "nfeatures %lld out of range", (long long)nfeat);
  if (nfeat > 0 && !X) return fail(SRHIP_ERR_INVALID, "null X");
  if (dtype == SRHIP_I32 && w) return fail(SRHIP_ERR_UNSUPPORTED, "weights on Int32 datasets");
  HIP_TRY(hipSetDevice(ctx->device));
  std::unique_ptr<srhip_dataset> d(new srhip_dataset());
  static std::atomic<uint64_t> g_ds_serial{0};
  d->serial = ++g_ds_serial;
  d->ctx = ctx;
  d->device = ctx->device;
  d->dtype = dtype;
  d->nfeat = nfeat;
  d->n = n;
  d->ld = (n + ROW_ALIGN - 1) / ROW_ALIGN * ROW_ALIGN;
  d->has_y = y != nullptr;
  d->weighted = w != nullptr;
  const size_t es = dtype_size(dtype);
  const size_t colb = (size_t)d->ld * es;
  HIP_TRY(d->X.ensure(std::max<size_t>(1, (size_t)nfeat) * colb));
  HostBuf stage;
  HIP_TRY(stage.ensure(colb));
  for (int64_t f = 0; f < nfeat; ++f) {
    if (dtype == SRHIP_F64) pack_column<uint64_t>(X, f, n, sf, sr, d->ld, (uint64_t*)stage.p);
    else pack_column<uint32_t>(X, f, n, sf, sr, d->ld, (uint32_t*)stage.p);  // bit copy
    HIP_TRY(hipMemcpy((char*)d->X.p + f * colb, stage.p, colb, hipMemcpyHostToDevice));
  }
  if (y) {
    HIP_TRY(d->y.ensure(colb));
    if (dtype == SRHIP_F64) pack_column<uint64_t>(y, 0, n, 0, 1, d->ld, (uint64_t*)stage.p);
    else pack_column<uint32_t>(y, 0, n, 0, 1, d->ld, (uint32_t*)stage.p);
    HIP_TRY(hipMemcpy(d->y.p, stage.p, colb, hipMemcpyHostToDevice));
  }
  if (w) {
    HIP_TRY(d->w.ensure(colb));
    double s = 0.0;
    if (dtype == SRHIP_F64) {
      double* st = (double*)stage.p;
      for (int64_t j = 0; j < d->ld; ++j) st[j] = j < n ? ((const double*)w)[j] : 0.0;
      for (int64_t j = 0; j < n; ++j) s += st[j];
    } else {
      float* st = (float*)stage.p;
      for (int64_t j = 0; j < d->ld; ++j) st[j] = j < n ? ((const float*)w)[j] : 0.0f;
      for (int64_t j = 0; j < n; ++j) s += st[j];
    }
    d->sum_w = s;
    HIP_TRY(hipMemcpy(d->w.p, stage.p, colb, hipMemcpyHostToDevice));
  }
  d->hstats.assign(std::max<int64_t>(1, nfeat), FeatStat{0.0, 0});
  if (dtype != SRHIP_I32 && nfeat > 0) {
    HIP_TRY(d->stats.ensure(feature_stats_scratch(nfeat) * sizeof(FeatStat)));
    HIP_TRY(launch_feature_stats(dtype, d->X.p, d->ld, n, (int)nfeat, (FeatStat*)d->stats.p, ctx->stream));
    HIP_TRY(hipMemcpyAsync(d->hstats.data(), d->stats.p, (size_t)nfeat * sizeof(FeatStat), hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  *out = d.release();
  return SRHIP_OK;
}

void srhip_dataset_destroy(srhip_dataset* ds) {
  if (!ds) return;
  (void)hipSetDevice(ds->device);
  delete ds;
  (void)hipGetLastError();  // no sticky error from the ignored calls above
}

int srhip_program_create(srhip_ctx* ctx, int dtype, const srhip_node* nodes, const int64_t* offsets, int32_t ntrees,
                         const srhip_operators* ops, srhip_program** out) {
  if (!out || !ops || (!offsets && ntrees > 0)) return fail(SRHIP_ERR_INVALID, "null argument");
  *out = nullptr;
  if (ntrees < 0) return fail(SRHIP_ERR_INVALID, "ntrees < 0");
  if (dtype != SRHIP_F32 && dtype != SRHIP_F64 && dtype != SRHIP_I32) return fail(SRHIP_ERR_UNSUPPORTED, "dtype %d", dtype);
  std::unique_ptr<srhip_program> P(new srhip_program());
  P->ctx = ctx;
  P->device = ctx ? ctx->device : -1;
  P->dtype = dtype;
  P->ntrees = ntrees;
  for (int i = 0; i < ops->nbin; ++i) {
    int sb, hb;
    if (!classify_binop(ops->binops[i], &sb, &hb)) return fail(SRHIP_ERR_UNSUPPORTED, "binary op code %d", ops->binops[i]);
    P->binops.push_back(ops->binops[i]);
  }
  for (int i = 0; i < ops->nuna; ++i) {
    if (classify_unop(ops->unaops[i]) < 0) return fail(SRHIP_ERR_UNSUPPORTED, "unary op code %d", ops->unaops[i]);
    P->unaops.push_back(ops->unaops[i]);
  }
  P->offsets.assign(offsets, offsets + ntrees + 1);
  if (ntrees > 0) {
    if (P->offsets[0] != 0) return fail(SRHIP_ERR_INVALID, "tree_offsets[0] must be 0");
    for (int32_t t = 0; t < ntrees; ++t)
      if (P->offsets[t + 1] <= P->offsets[t]) return fail(SRHIP_ERR_INVALID, "tree %d is empty", (int)t);
    P->nodes.assign(nodes, nodes + P->offsets[ntrees]);
  }
  int rc = compile_program(*P);
  if (rc) return rc;
  if (ctx) {  // ctx == NULL: host-only program (compile + did_succeed metadata, e.g. for finalize)
    plan_persistent_order(ctx, *P);
    rc = upload_program(*P, true, false, ctx->up_stream);
    if (rc) return rc;
  }
  *out = P.release();
  return SRHIP_OK;
}

void srhip_program_destroy(srhip_program* P) {
  if (!P) return;
  // a program's teardown is host work only (its device buffers go back to the allocation cache): a
  // background thread does it, so the caller -- e.g. a pipeline between two evaluations -- does not
  // wait for freeing a large population's per-tree metadata (~0.1 ms for 1024 trees)
  if (!env_flag("SRHIP_SYNC_DESTROY")) {
    reaper_push(P);
    return;
  }
  if (P->device >= 0) (void)hipSetDevice(P->device);
  delete P;
  (void)hipGetLastError();
}

int srhip_program_num_constants(const srhip_program* P, int32_t* out) {
  if (!P || !out) return fail(SRHIP_ERR_INVALID, "null argument");
  for (int32_t t = 0; t < P->ntrees; ++t) out[t] = P->info[t].nconst;
  return SRHIP_OK;
}

static void set_consts_rec(std::vector<srhip_node>& nodes, int64_t base, int64_t i, const double*& c) {
  srhip_node& n = nodes[base + i];
  if (n.degree == 0) {
    if (n.constant) n.val = *c++;
    return;
  }
  set_consts_rec(nodes, base, n.l, c);
  if (n.degree == 2) set_consts_rec(nodes, base, n.r, c);
}

static void get_consts_rec(const std::vector<srhip_node>& nodes, int64_t base, int64_t i, double*& c) {
  const srhip_node& n = nodes[base + i];
  if (n.degree == 0) {
    if (n.constant) *c++ = n.val;
    return;
  }
  get_consts_rec(nodes, base, n.l, c);
  if (n.degree == 2) get_consts_rec(nodes, base, n.r, c);
}

int srhip_program_get_constants(const srhip_program* P, double* consts) {
  if (!P || (!consts && P->ntrees > 0)) return fail(SRHIP_ERR_INVALID, "null argument");
  double* c = consts;
  for (int32_t t = 0; t < P->ntrees; ++t) get_consts_rec(P->nodes, P->offsets[t], 0, c);
  return SRHIP_OK;
}

int srhip_program_set_constants(srhip_program* P, const double* consts) {
  if (!P || (!consts && P->ntrees > 0)) return fail(SRHIP_ERR_INVALID, "null argument");
  const double* c = consts;
  for (int32_t t = 0; t < P->ntrees; ++t) set_consts_rec(P->nodes, P->offsets[t], 0, c);
  {
    // new constants can change which trees fail statically (non-finite leaves): the next evaluation
    // plans its launch order again
    std::lock_guard<std::mutex> g(P->ord_mu);
    P->ord_key[0] = P->ord_key[1] = P->ord_key[2] = -1;
    P->ord_goff.clear();
  }
  int rc = compile_program(*P);
  if (rc) return rc;
  return P->ctx ? upload_program(*P) : SRHIP_OK;
}

int srhip_eval_loss(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog, const srhip_loss* loss,
                    const int64_t* idx, int64_t nidx, double* out_loss, uint8_t* out_ok) {
  if (!out_loss || !out_ok) return fail(SRHIP_ERR_INVALID, "null output");
  return run_eval(ctx, ds, prog, MODE_LOSS, loss, idx, nidx, out_loss, nullptr, out_ok);
}

// srhip_eval_loss_submit / _wait: an evaluation whose launches return at once (queued on the context's
// stream behind whatever is in flight there) and whose records, decisions and outputs are taken at wait.
struct srhip_eval_ticket {
  srhip_ctx* ctx = nullptr;
  RunJob R;
  bool done = false;  // evaluated at submit (row subsets)
  std::vector<double> loss;
  std::vector<uint8_t> ok;
};

int srhip_eval_loss_submit(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog, const srhip_loss* loss,
                           const int64_t* idx, int64_t nidx, srhip_eval_ticket** out) {
  if (!out) return fail(SRHIP_ERR_INVALID, "null ticket output");
  *out = nullptr;
  if (!ctx || !prog) return fail(SRHIP_ERR_INVALID, "null argument");
  std::unique_ptr<srhip_eval_ticket> t(new srhip_eval_ticket());
  t->ctx = ctx;
  if (idx) {
    // a row subset's gather synchronises the stream and its buffers are the context's: evaluated here
    t->loss.resize(prog->ntrees);
    t->ok.resize(prog->ntrees);
    const int rc = run_eval(ctx, ds, prog, MODE_LOSS, loss, idx, nidx, t->loss.data(), nullptr, t->ok.data());
    if (rc) return rc;
    t->done = true;
    *out = t.release();
    return SRHIP_OK;
  }
  int k = -1;
  for (int i = 1; i < RESULT_SETS && k < 0; ++i)
    if (!ctx->rs[i].busy) k = i;
  if (k < 0) return fail(SRHIP_ERR_INVALID, "%d evaluations already in flight on this context", RESULT_SETS - 1);
  t->R.J.rs = &ctx->rs[k];
  const int rc = run_issue(ctx, ds, prog, MODE_LOSS, loss, nullptr, 0, nullptr, t->R);
  if (rc) {
    (void)hipStreamSynchronize(ctx->stream);  // launches may have been queued before the failure
    return rc;
  }
  ctx->rs[k].busy = true;
  *out = t.release();
  return SRHIP_OK;
}

int srhip_eval_loss_wait(srhip_eval_ticket* ticket, double* out_loss, uint8_t* out_ok) {
  if (!ticket) return fail(SRHIP_ERR_INVALID, "null ticket");
  std::unique_ptr<srhip_eval_ticket> t(ticket);
  if (t->done) {
    for (size_t i = 0; i < t->loss.size(); ++i) {
      if (out_loss) out_loss[i] = t->loss[i];
      if (out_ok) out_ok[i] = t->ok[i];
    }
    return SRHIP_OK;
  }
  srhip_ctx* ctx = t->ctx;
  ResultSet* rs = t->R.J.rs;
  struct Release {  // the result set is free again on every path
    ResultSet* r;
    ~Release() { r->busy = false; }
  } release{rs};
  HIP_TRY(hipSetDevice(ctx->device));
  if (t->R.J.launched) HIP_TRY(hipEventSynchronize(rs->done));
  return run_complete(ctx, t->R, out_loss, out_ok);
}

int srhip_eval_predict(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* prog, const int64_t* idx,
                       int64_t nidx, void* out_pred, uint8_t* out_ok) {
  if (!out_pred || !out_ok) return fail(SRHIP_ERR_INVALID, "null output");
  return run_eval(ctx, ds, prog, MODE_PRED, nullptr, idx, nidx, nullptr, out_pred, out_ok);
}

int srhip_eval_loss_batch(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_node* nodes, const int64_t* offsets,
                          int32_t ntrees, const srhip_operators* ops, const srhip_loss* loss, const int64_t* idx,
                          int64_t nidx, double* out_loss, uint8_t* out_ok) {
  if (!ds) return fail(SRHIP_ERR_INVALID, "null dataset");
  srhip_program* P = nullptr;
  int rc = srhip_program_create(ctx, ds->dtype, nodes, offsets, ntrees, ops, &P);
  if (rc) return rc;
  rc = srhip_eval_loss(ctx, ds, P, loss, idx, nidx, out_loss, out_ok);
  srhip_program_destroy(P);
  return rc;
}

int srhip_eval_loss_partials(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const srhip_loss* loss,
                             const int64_t* idx, int64_t nidx, double* sums, double* chk) {
  if (!sums || !chk) return fail(SRHIP_ERR_INVALID, "null output");
  int rc = check_eval_args(ctx, ds, P, MODE_LOSS, loss);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  View v;
  rc = make_view(ctx, ds, idx, nidx, true, v);
  if (rc) return rc;
  if (idx && ds->weighted) {
    rc = gathered_weight_sum(ctx, ds, nidx, v);
    if (rc) return rc;
  }
  return eval_partials(ctx, ds, P, MODE_LOSS, loss, v, nullptr, sums, chk);
}

int srhip_partials_finalize(const srhip_program* P, int64_t nfeatures, const double* sums, const double* chk,
                            double* out_loss, uint8_t* out_ok, uint8_t* out_status) {
  if (!P || !sums || (!chk && P->dtype != SRHIP_I32)) return fail(SRHIP_ERR_INVALID, "null argument");
  if (nfeatures < 0) return fail(SRHIP_ERR_INVALID, "nfeatures < 0");
  for (const TreeInfo& I : P->info)
    for (int f : I.feat_checks)
      if (f >= nfeatures) return fail(SRHIP_ERR_INVALID, "tree checks feature %d of %lld", f + 1, (long long)nfeatures);
  finalize(*P, nfeatures, sums, chk, out_loss, out_ok, out_status);
  return SRHIP_OK;
}

int srhip_eval_precise_partials(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_program* P, const int64_t* idx,
                                int64_t nidx, const int32_t* trees, int32_t ntrees_sel, double* opsums) {
  if (!opsums || (!trees && ntrees_sel > 0) || ntrees_sel < 0) return fail(SRHIP_ERR_INVALID, "null argument");
  int rc = check_eval_args(ctx, ds, P, MODE_PRED, nullptr);
  if (rc) return rc;
  for (int32_t u = 0; u < ntrees_sel; ++u)
    if (trees[u] < 0 || trees[u] >= P->ntrees) return fail(SRHIP_ERR_INVALID, "tree index %d out of range", trees[u]);
  HIP_TRY(hipSetDevice(ctx->device));
  View v;
  rc = make_view(ctx, ds, idx, nidx, false, v);
  if (rc) return rc;
  return eval_precise(ctx, ds, P, v, trees, ntrees_sel, opsums);
}

int srhip_precise_finalize(const srhip_program* P, const int32_t* trees, int32_t ntrees_sel, const double* opsums,
                           uint8_t* out_ok) {
  if (!P || !opsums || !out_ok || (!trees && ntrees_sel > 0)) return fail(SRHIP_ERR_INVALID, "null argument");
  for (int32_t u = 0; u < ntrees_sel; ++u)
    if (trees[u] < 0 || trees[u] >= P->ntrees) return fail(SRHIP_ERR_INVALID, "tree index %d out of range", trees[u]);
  finalize_precise(*P, trees, ntrees_sel, opsums, out_ok);
  return SRHIP_OK;
}

int srhip_chk_reduce_op(int dtype) { return dtype == SRHIP_F32 ? 0 : 1; }

int32_t srhip_program_max_ops(const srhip_program* P) { return P ? std::max(1, P->max_ops) : 0; }

double srhip_last_kernel_ms(const srhip_ctx* ctx) {
  if (!ctx || !ctx->timed || !ctx->last_ev0 || !ctx->last_ev1) return -1.0;
  float ms = -1.0f;
  if (hipEventElapsedTime(&ms, ctx->last_ev0, ctx->last_ev1) != hipSuccess) return -1.0;
  return (double)ms;
}

int srhip_code_cache_stats(int64_t* hits, int64_t* misses, int64_t* inserts) {
  if (hits) *hits = g_cache_hits.load();
  if (misses) *misses = g_cache_misses.load();
  if (inserts) *inserts = g_cache_inserts.load();
  return SRHIP_OK;
}

int srhip_last_work(const srhip_ctx* ctx, int64_t* out) {
  if (!ctx || !out) return fail(SRHIP_ERR_INVALID, "null argument");
  for (int i = 0; i < 4; ++i) out[i] = ctx->work[i];
  return SRHIP_OK;
}

int srhip_program_stats(const srhip_program* P, int64_t* total_nodes, int64_t* total_opnodes, int32_t* max_stack) {
  if (!P) return fail(SRHIP_ERR_INVALID, "null program");
  if (total_nodes) *total_nodes = P->total_nodes;
  if (total_opnodes) *total_opnodes = P->total_ops;
  if (max_stack) *max_stack = P->kmax;
  return SRHIP_OK;
}

int srhip_program_derived(const srhip_program* P, int32_t* count, uint32_t* spec, int32_t cap) {
  if (!P) return fail(SRHIP_ERR_INVALID, "null program");
  if (count) *count = (int32_t)P->dspec.size();
  for (int32_t d = 0; spec && d < cap && d < (int32_t)P->dspec.size(); ++d) spec[d] = P->dspec[d];
  return SRHIP_OK;
}

}  // extern "C"
