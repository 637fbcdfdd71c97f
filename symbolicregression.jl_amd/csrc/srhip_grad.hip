// srhip_grad.hip — batched forward-mode (dual-number) constant gradients for the constant optimizer.
//
// Replaces (reference): the objective of _optimize_constants (src/ConstantOptimization.jl:43-81),
// f(c) = eval_loss(tree(c), dataset, options; regularization=false), whose gradient Optim obtains
// by finite differences (no g! is passed, :50).  Here one launch returns, for every tree, the loss
// and its exact gradient with respect to the tree's constants (get_constants order,
// test/test_derivatives.jl:123-147), by carrying KT tangent components per value through the
// same bytecode interpreter as the evaluator (the "gradient program": constants not folded, each
// constant leaf tagged with its index).  A "chunk" is (tree, first constant c0): trees with more
// than KT constants take several chunks.  One lane owns one row (R = 1); values and tangents
// live in VGPRs.  Operator values are computed by the same functions as srhip_eval_impl.h, so the
// loss equals srhip_eval_loss's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "srhip_grad.h"
#include "srhip_isa.h"
#include "srhip_kernels.h"
#include "srhip_ops.h"

#define UNR _Pragma("unroll")
#ifndef GRAD_R
#define GRAD_R 1  // 2 measured slower on C4 (2.60 -> 2.80 ms: 155 VGPRs, 3 waves per SIMD)
#endif
#define DI __device__ __attribute__((always_inline)) inline

namespace srhip {

#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) Ins GIns;  // bytecode through the scalar cache
#else
typedef const Ins GIns;
#endif

template <typename T> struct V2 { typedef T type __attribute__((ext_vector_type(2))); };
template <typename T> struct V4 { typedef T type __attribute__((ext_vector_type(4))); };

// ---- operator values and partial derivatives ------------------------------------------------
template <int U> constexpr bool dun_inline() { return un_grad_inline(U); }

// f(x) and f'(x) for a heavy unary operator U; D = false: the value alone (value-only passes: the
// derivative of cos is a sin, of log a division -- out of line the compiler cannot drop them), the
// same f.  Out of line per (T, U, D) (dual_un_heavy), and for value-only passes once per R rows
// (dual_un_heavy_rows: one call per node and tile instead of R, the same body per row)
template <typename T, int U, bool D> DI typename V2<T>::type dual_un_body(T x) {
  using O = FOps<T>;
  T f = T(0), df = T(0);
  switch (U) {
    case UN_COS:
      if constexpr (D && sizeof(T) == 8) {  // one Float64 reduction for both (srm_sincos: the same bits)
        double sn, cs;
        srm_sincos(x, &sn, &cs);
        f = cs;
        df = -sn;
      } else {
        f = O::cos(x);
        if constexpr (D) df = -O::sin(x);
      }
      break;
    case UN_SIN:
      if constexpr (D && sizeof(T) == 8) {
        double sn, cs;
        srm_sincos(x, &sn, &cs);
        f = sn;
        df = cs;
      } else {
        f = O::sin(x);
        if constexpr (D) df = O::cos(x);
      }
      break;
    case UN_TAN: f = O::tan(x); if constexpr (D) df = T(1) + f * f; break;
    case UN_EXP: f = O::exp(x); if constexpr (D) df = f; break;
    case UN_LOG: f = O::log(x); if constexpr (D) df = T(1) / x; break;
    case UN_LOG2: f = O::log2(x); if constexpr (D) df = T(1) / (x * T(0.69314718055994530942)); break;
    case UN_LOG10: f = O::log10(x); if constexpr (D) df = T(1) / (x * T(2.30258509299404568402)); break;
    case UN_LOG1P: f = O::log1p(x); if constexpr (D) df = T(1) / (T(1) + x); break;
    case UN_SQRT: f = O::sqrt(x); if constexpr (D) df = T(0.5) / f; break;
    case UN_ACOSH: f = O::acosh(x); if constexpr (D) df = T(1) / m_sqrt(x * x - T(1)); break;
    case UN_ATANH_CLIP: {
      f = O::atanh_clip(x);
      if constexpr (D) {
        const T u = O::mod(x + T(1), T(2)) - T(1);
        df = T(1) / (T(1) - u * u);
      }
      break;
    }
    case UN_SINH: f = O::sinh(x); if constexpr (D) df = O::cosh(x); break;
    case UN_COSH: f = O::cosh(x); if constexpr (D) df = O::sinh(x); break;
    case UN_TANH: f = O::tanh(x); if constexpr (D) df = T(1) - f * f; break;
    case UN_ASIN: f = O::asin(x); if constexpr (D) df = T(1) / m_sqrt(T(1) - x * x); break;
    case UN_ACOS: f = O::acos(x); if constexpr (D) df = -T(1) / m_sqrt(T(1) - x * x); break;
    case UN_ATAN: f = O::atan(x); if constexpr (D) df = T(1) / (T(1) + x * x); break;
    case UN_ASINH: f = O::asinh(x); if constexpr (D) df = T(1) / m_sqrt(x * x + T(1)); break;
    case UN_ERF: f = O::erf(x); if constexpr (D) df = T(1.12837916709551257390) * O::exp(-x * x); break;
    case UN_ERFC: f = O::erfc(x); if constexpr (D) df = -T(1.12837916709551257390) * O::exp(-x * x); break;
    case UN_GAMMA: f = O::gamma(x); if constexpr (D) df = FP<T>::nan(); break;  // no digamma: no gradient (optimizer keeps c)
    case UN_EXP2: f = O::exp2(x); if constexpr (D) df = f * T(0.69314718055994530942); break;
    case UN_EXPM1: f = O::expm1(x); if constexpr (D) df = f + T(1); break;
    case UN_CBRT: f = O::cbrt(x); if constexpr (D) df = T(1) / (T(3) * f * f); break;
    default: f = FP<T>::nan(); df = FP<T>::nan(); break;
  }
  typename V2<T>::type r;
  r[0] = f;
  r[1] = df;
  return r;
}
template <typename T, int U, bool D> __device__ __attribute__((noinline)) typename V2<T>::type dual_un_heavy(T x) {
  return dual_un_body<T, U, D>(x);
}
template <typename T, int R> struct VR { typedef T type __attribute__((ext_vector_type(R))); };
template <typename T> struct VR<T, 1> { typedef T type; };
#ifndef GRAD_ROWS_FENCE
#define GRAD_ROWS_FENCE 1  // rows of dual_un_heavy_rows one after another (no interleaving)
#endif
template <typename T, int U, int R>
__device__ __attribute__((noinline)) typename VR<T, R>::type dual_un_heavy_rows(typename VR<T, R>::type x) {
  if constexpr (R == 1) {
    return dual_un_body<T, U, false>(x)[0];
  } else {
    UNR for (int r = 0; r < R; ++r) {
      x[r] = dual_un_body<T, U, false>(x[r])[0];
      if (GRAD_ROWS_FENCE) __builtin_amdgcn_sched_barrier(0);
    }
    return x;
  }
}

template <typename T, int U, bool D = true> DI void dual_un(T x, T& f, T& df) {
  using O = FOps<T>;
  if constexpr (dun_inline<U>()) {
    switch (U) {
      case UN_NEG: f = O::neg(x); df = T(-1); break;
      case UN_SQUARE: f = O::square(x); df = T(2) * x; break;
      case UN_CUBE: f = O::cube(x); df = T(3) * x * x; break;
      case UN_ABS: f = O::abs(x); df = x > T(0) ? T(1) : (x < T(0) ? T(-1) : T(0)); break;
      case UN_RELU: f = O::relu(x); df = x > T(0) ? T(1) : T(0); break;
      case UN_SIGN: f = O::sign(x); df = T(0); break;
      case UN_ROUND: f = O::round(x); df = T(0); break;
      case UN_FLOOR: f = O::floor(x); df = T(0); break;
      case UN_CEIL: f = O::ceil(x); df = T(0); break;
      default: break;
    }
  } else {
    const typename V2<T>::type r = dual_un_heavy<T, U, D>(x);
    f = r[0];
    df = r[1];
  }
}

// f(a, b), df/da, df/db for a specialised (cheap) binary operator SB
template <typename T, int SB> DI void dual_spec(T a, T b, T& f, T& fa, T& fb) {
  using O = FOps<T>;
  switch (SB) {
    case SB_ADD: f = O::add(a, b); fa = T(1); fb = T(1); break;
    case SB_SUB: f = O::sub(a, b); fa = T(1); fb = T(-1); break;
    case SB_MUL: f = O::mul(a, b); fa = b; fb = a; break;
    case SB_DIV: { f = O::div(a, b); const T ib = T(1) / b; fa = ib; fb = -f * ib; break; }
    case SB_GREATER: f = O::greater(a, b); fa = T(0); fb = T(0); break;
    case SB_COND: f = O::cond(a, b); fa = T(0); fb = a > T(0) ? T(1) : T(0); break;
    case SB_LOGICAL_OR: f = O::logical_or(a, b); fa = T(0); fb = T(0); break;
    case SB_LOGICAL_AND: f = O::logical_and(a, b); fa = T(0); fb = T(0); break;
    case SB_MAX: f = O::max(a, b); fa = a > b ? T(1) : T(0); fb = a > b ? T(0) : T(1); break;
    case SB_MIN: f = O::min(a, b); fa = a < b ? T(1) : T(0); fb = a < b ? T(0) : T(1); break;
    default: f = FP<T>::nan(); fa = f; fb = f; break;
  }
}

// heavy binary (pow, mod, atan2): out of line; returns (f, df/da, df/db, -)
template <typename T, int HB, bool D> __device__ __attribute__((noinline)) typename V4<T>::type dual_heavy(T a, T b) {
  using O = FOps<T>;
  T f, fa = T(0), fb = T(0);
  switch (HB) {
    case HB_POW:
      f = O::pow(a, b);
      if constexpr (D) {
        fa = b * O::pow(a, b - T(1));
        fb = a > T(0) ? f * m_log(a) : T(0);
      }
      break;
    case HB_MOD: f = O::mod(a, b); if constexpr (D) { fa = T(1); fb = -m_floor(a / b); } break;
    case HB_ATAN2: {
      f = O::atan2(a, b);
      if constexpr (D) { const T r = T(1) / (a * a + b * b); fa = b * r; fb = -a * r; }
      break;
    }
    default: f = FP<T>::nan(); fa = f; fb = f; break;
  }
  typename V4<T>::type r;
  r[0] = f;
  r[1] = fa;
  r[2] = fb;
  r[3] = T(0);
  return r;
}

// d loss / d prediction for the distance losses of srhip_ops.h loss_elem (diff = pred - y)
template <typename T> DI T dloss_elem(int kind, T d, T p0) {
  const T sg = d > T(0) ? T(1) : (d < T(0) ? T(-1) : T(0));
  switch (kind) {
    case SRHIP_LOSS_L2: return T(2) * d;
    case SRHIP_LOSS_L1: return sg;
    case SRHIP_LOSS_LP: return p0 * m_pow(m_abs(d), p0 - T(1)) * sg;
    case SRHIP_LOSS_HUBER: return m_abs(d) <= p0 ? d : p0 * sg;
    case SRHIP_LOSS_L1_EPS_INS: return m_abs(d) > p0 ? sg : T(0);
    case SRHIP_LOSS_L2_EPS_INS: return T(2) * m_max(T(0), m_abs(d) - p0) * sg;
    case SRHIP_LOSS_LOGIT_DIST: { const T e = m_exp(d); return (e - T(1)) / (e + T(1)); }
    case SRHIP_LOSS_PERIODIC: {
      const T k = T(2) * T(3.14159265358979323846) / p0;
      return k * m_sin(d * k);
    }
    case SRHIP_LOSS_QUANTILE: return p0 - (d < T(0) ? T(1) : T(0));
    default: return FP<T>::nan();
  }
}

// (loss, d loss / d output) of the other distance losses, out of line: inline, their math bodies
// raised the kernel's register count for every loss kind
// d loss / d agreement of the margin losses of srhip_ops.h margin_loss (a = target * output)
template <typename T> DI T dmargin(int kind, T a, T p0) {
  switch (kind) {
    case SRHIP_LOSS_ZERO_ONE: return T(0);
    case SRHIP_LOSS_PERCEPTRON: return a >= T(0) ? T(0) : T(-1);
    case SRHIP_LOSS_LOGIT_MARGIN: return T(-1) / (T(1) + m_exp(a));
    case SRHIP_LOSS_L1_HINGE: return a >= T(1) ? T(0) : T(-1);
    case SRHIP_LOSS_L2_HINGE: return a >= T(1) ? T(0) : T(2) * (a - T(1));
    case SRHIP_LOSS_SMOOTHED_L1_HINGE: return a >= T(1) - p0 ? (a >= T(1) ? T(0) : (a - T(1)) / p0) : T(-1);
    case SRHIP_LOSS_MODIFIED_HUBER: return a >= T(-1) ? (a > T(1) ? T(0) : T(2) * a - T(2)) : T(-4);
    case SRHIP_LOSS_L2_MARGIN: return T(2) * (a - T(1));
    case SRHIP_LOSS_EXP: return -m_exp(-a);
    case SRHIP_LOSS_SIGMOID: { const T t = m_tanh(a); return -(T(1) - t * t); }
    case SRHIP_LOSS_DWD_MARGIN:
      return a <= p0 / (p0 + T(1)) ? T(-1) : -m_pow(p0 / (p0 + T(1)), p0 + T(1)) / m_pow(a, p0 + T(1));
    default: return FP<T>::nan();
  }
}
// (loss, d loss / d output) of one row for the kinds other than L2: distance losses of
// output - target, margin losses of target * output (chain rule: target * dL/da)
template <typename T>
__device__ __attribute__((noinline)) typename V2<T>::type loss_dloss_generic(int kind, T out, T y, T p0) {
  if (loss_is_margin(kind)) {
    const T a = y * out;
    return typename V2<T>::type{margin_loss<T>(kind, a, p0), y * dmargin<T>(kind, a, p0)};
  }
  const T d = out - y;
  return typename V2<T>::type{loss_elem<T>(kind, d, p0), dloss_elem<T>(kind, d, p0)};
}

// ---- the dual-number interpreter ----------------------------------------------------------------
template <typename T> DI T imm_bits(uint64_t b) {
  if constexpr (sizeof(T) == 8) return __builtin_bit_cast(T, b);
  else return __builtin_bit_cast(T, (uint32_t)b);
}

// KT = 0: values only (the line search's trial points): the primal code and its row-sum order are
// the same as with tangents, so a value-only loss is bit-identical to the loss of a gradient launch
template <typename T, int KT> struct Dual {
  T v;
  T d[KT > 0 ? KT : 1];
};

// leaves: tangents are seeded on the constants (GMODE_LOSS / GMODE_ROWC: rel = constant index - c0)
// or on the features (GMODE_ROWF: rel = feature index - c0)
template <int GM, typename T, int KT> DI void set_const(Dual<T, KT>& a, T c, int rel) {
  a.v = c;
  UNR for (int j = 0; j < KT; ++j) a.d[j] = (GM != GMODE_ROWF && rel == j) ? T(1) : T(0);
}
template <int GM, typename T, int KT> DI void set_feat(Dual<T, KT>& a, T x, int rel) {
  a.v = x;
  UNR for (int j = 0; j < KT; ++j) a.d[j] = (GM == GMODE_ROWF && rel == j) ? T(1) : T(0);
}
// out = f(l, r) with partials: out.d = fl * l.d + fr * r.d (out may alias l or r)
template <typename T, int KT>
DI void combine(Dual<T, KT>& out, const Dual<T, KT>& l, const Dual<T, KT>& r, T f, T fl, T fr) {
  T d[KT > 0 ? KT : 1];
  UNR for (int j = 0; j < KT; ++j) d[j] = fl * l.d[j] + fr * r.d[j];
  out.v = f;
  UNR for (int j = 0; j < KT; ++j) out.d[j] = d[j];
}

// check statistic, as in the evaluator: max |v| (Float32, NaN-propagating) / sum |v| 2^-512 (Float64)
DI void chk_fold(float& M, float v) { M = __builtin_elementwise_maximum(M, __builtin_fabsf(v)); }
DI void chk_fold(double& M, double v) { M = __builtin_fma(__builtin_fabs(v), 0x1p-512, M); }

// XLDS: the workgroup stages its row block of X (and y) into LDS once -- feature leaves then read
// LDS instead of issuing a dependent global load per leaf per tile (grad_lds_bytes: [nfeat + 1][rb_rows])
// R rows per lane: a tile is 64 R rows (row tile_base + 64 r + lane), one bytecode dispatch per tile.
// Every lane still folds its rows in ascending row order (tile-major, r inner), so losses and
// gradients are bit-identical for any R.
// The value of lane (lane ^ O) for the xor butterflies of the per-(chunk, row block) sums: DPP for
// O <= 8 (quad permutes; half-row / row mirrors composed with them), ds_swizzle for 16, ds_bpermute
// for 32 -- the partner's exact bits, so every sum is the one __shfl_xor gave, with four of the six
// levels off the LDS crossbar's latency.
template <int O> DI uint32_t xor_lane_u32(uint32_t v, int lane) {
  if constexpr (O == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad [1,0,3,2]
  else if constexpr (O == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad [2,3,0,1]
  else if constexpr (O == 4)  // half-row mirror (i ^ 7), then quad mirror (^ 3)
    return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF, false);
  else if constexpr (O == 8)  // row mirror (i ^ 15), then half-row mirror (^ 7)
    return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false), 0x141, 0xF, 0xF, false);
  else if constexpr (O == 16)  // bitmask swizzle within 32 lanes: and 0x1f, or 0, xor 0x10
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
  else
    return (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ O) << 2, (int)v);
}
template <int O> DI double xor_lane(double x, int lane) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint64_t r = (uint64_t)xor_lane_u32<O>((uint32_t)b, lane) | ((uint64_t)xor_lane_u32<O>((uint32_t)(b >> 32), lane) << 32);
  return __builtin_bit_cast(double, r);
}
template <int O> DI float xor_lane(float x, int lane) {
  return __builtin_bit_cast(float, xor_lane_u32<O>(__builtin_bit_cast(uint32_t, x), lane));
}

// SRHIP_GRAD_WPE = W > 0 (build level, A/B): the tangent-carrying variants (KT >= 4) are compiled for at
// least W waves per SIMD (the register allocator's target; 0 leaves it free)
#ifndef SRHIP_GRAD_WPE
#define SRHIP_GRAD_WPE 0
#endif
template <typename T, int KT, int K, int GM, bool XLDS, int R>
__global__ __launch_bounds__(64 * GRAD_WAVES)
#if SRHIP_GRAD_WPE > 0
__attribute__((amdgpu_waves_per_eu(KT >= 4 ? SRHIP_GRAD_WPE : 1)))
#endif
void grad_kernel(GradArgs p) {
  constexpr int CW = GM == GMODE_LOSS ? 2 : 4;  // ints per chunk record
  const int lane = threadIdx.x & 63;
  const int rb = blockIdx.x + p.block0;
  const int64_t row_base = (int64_t)rb * p.rb_rows;
  const int ntiles = p.rb_rows / (64 * R);
  // valid rows of this block, block-relative: the row tests below are 32-bit (scalar for the tile test)
  const int nrel = __builtin_amdgcn_readfirstlane((int)min<int64_t>(max<int64_t>(p.nvalid - row_base, 0), (int64_t)p.rb_rows));
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int group_base = blockIdx.y * p.chunks_per_group;
  const int group_n = min(p.chunks_per_group, p.nchunks - group_base);
  const T* Xg = reinterpret_cast<const T*>(p.X);
  const T* Yg = reinterpret_cast<const T*>(p.y);
  const T* W = reinterpret_cast<const T*>(p.w);
  extern __shared__ __attribute__((aligned(16))) unsigned char grad_lds[];
  T* xs = reinterpret_cast<T*>(grad_lds);
  const int rbr = p.rb_rows;
  // chunks are claimed dynamically from an LDS counter (wave w starts with chunk w): the host orders
  // each group's chunks by descending cost, so the waves of a workgroup finish within about one cheap
  // chunk of each other (a static round-robin left the cost spread idle at every workgroup's end);
  // every (chunk, row block) record is computed by one wave as before, so the bits do not change
  __shared__ int next_chunk;
  if (threadIdx.x == 0) next_chunk = GRAD_WAVES;
  if constexpr (XLDS) {
    const int nf = p.nfeat;
    const bool has_y = GM == GMODE_LOSS && Yg != nullptr;
    for (int i = threadIdx.x; i < (nf + 1) * rbr; i += 64 * GRAD_WAVES) {
      const int f = i / rbr, r = i - f * rbr;
      const int64_t row = row_base + r;
      T v = T(0);
      if (row < p.ld) v = f < nf ? Xg[(int64_t)f * p.ld + row] : (has_y ? Yg[row] : T(0));
      xs[i] = v;
    }
  }
  __syncthreads();
  // feature f / target at block-relative row rr of this row block
  // (a derived view's derived columns, f >= nfeat, are read from global memory)
  auto xat = [&](int f, int rr) -> T {
    if constexpr (XLDS) {
      if (f < p.nfeat) return xs[f * rbr + rr];
    }
    return Xg[(int64_t)f * p.ld + row_base + rr];
  };
  auto yat = [&](int rr) -> T {
    if constexpr (XLDS) return xs[p.nfeat * rbr + rr];
    else return Yg[row_base + rr];
  };
  GIns* code = (GIns*)(uintptr_t)p.code;
  const T p0 = (T)p.loss_p0;
  const int max_steps = __builtin_amdgcn_readfirstlane(p.max_steps);
  auto claim = [&]() {
    int c = 0;
    if (lane == 0) c = atomicAdd(&next_chunk, 1);
    return __builtin_amdgcn_readfirstlane(c);
  };
  for (int ci = wave; ci < group_n; ci = claim()) {
    const int chunk = group_base + ci;
    int tree, c0;
    if (GM == GMODE_LOSS && !p.chunks) {  // the list in the kernel arguments
      tree = __builtin_amdgcn_readfirstlane(p.inl[2 * chunk]);
      c0 = __builtin_amdgcn_readfirstlane(p.inl[2 * chunk + 1]);
    } else {
      tree = __builtin_amdgcn_readfirstlane(p.chunks[CW * chunk]);
      c0 = __builtin_amdgcn_readfirstlane(p.chunks[CW * chunk + 1]);
    }
    if constexpr (GM == GMODE_LOSS && KT == 0) {
      if (p.screened) {
        // the screen launch's record of row block 0 for this chunk: a non-finite check statistic (a
        // NaN / Inf operator output in its rows) fails the tree; the blocks left unwritten here only
        // ever reach the reduction's check statistic, which block 0 already makes non-finite
        const double m0 = p.slab[(int64_t)chunk * p.nrb * 2 + 1];  // [chunk][block 0][loss, chk]
        if (__builtin_amdgcn_readfirstlane((int)!__builtin_isfinite(m0))) continue;
      }
    }
    const int pc0 = __builtin_amdgcn_readfirstlane(p.prog_off[tree]);
    double lacc = 0.0;
    double gacc[KT > 0 ? KT : 1];
    UNR for (int j = 0; j < KT; ++j) gacc[j] = 0.0;
    T M = T(0);
    for (int tile = 0; tile < ntiles; ++tile) {
      const int tb = tile * 64 * R;  // block-relative first row of the tile
      if (tb >= nrel) break;
      // rows up to ld are finite replicas; masked at the loss
      Dual<T, KT> A[R], S[K][R];
      UNR for (int r = 0; r < R; ++r) set_feat<GMODE_LOSS>(A[r], T(0), -1);
      GIns* prog = code + pc0;
      Ins nxt = prog[0];
      for (int step = 0; step < max_steps; ++step) {
        const Ins ins = nxt;
        nxt = prog[step + 1];
        if (ins.h == H_END) break;
        const int opnd = (int)(ins.a & 0xffff);
        const T imm = imm_bits<T>(ins.imm);
#define RR(...) UNR for (int r = 0; r < R; ++r) { const int rr = tb + 64 * r + lane; (void)rr; __VA_ARGS__ }
        switch (ins.h) {
          case H_LOADF:
            RR(set_feat<GM>(A[r], xat(opnd, rr), opnd - c0);)
            if (opnd >= p.nfeat) {
              // a derived column: the operator's output (its check fold), and its tangents f'(x) * 0
              // (+-0, or NaN where f' is not finite) from the tangent-zero column
              RR(chk_fold(M, A[r].v);)
              if constexpr (KT > 0) {
                RR(const T z = Xg[(int64_t)(opnd + p.gd_nd) * p.ld + row_base + rr];
                   UNR for (int j = 0; j < KT; ++j) A[r].d[j] = z;)
              }
            }
            break;
          case H_LOADC: RR(set_const<GM>(A[r], imm, opnd - c0);) break;
#define GK_CASES(BASE, ...)                                                                        \
  case BASE + 0: if constexpr (0 < K) { constexpr int k = 0; __VA_ARGS__ } break;                \
  case BASE + 1: if constexpr (1 < K) { constexpr int k = 1; __VA_ARGS__ } break;                \
  case BASE + 2: if constexpr (2 < K) { constexpr int k = 2; __VA_ARGS__ } break;                \
  case BASE + 3: if constexpr (3 < K) { constexpr int k = 3; __VA_ARGS__ } break;                \
  case BASE + 4: if constexpr (4 < K) { constexpr int k = 4; __VA_ARGS__ } break;                \
  case BASE + 5: if constexpr (5 < K) { constexpr int k = 5; __VA_ARGS__ } break;                \
  case BASE + 6: if constexpr (6 < K) { constexpr int k = 6; __VA_ARGS__ } break;                \
  case BASE + 7: if constexpr (7 < K) { constexpr int k = 7; __VA_ARGS__ } break;
          GK_CASES(H_PUSH0, { RR(S[k][r] = A[r];) })
#if SRHIP_GRAD_SUPER_LEVEL >= 1
          // superinstructions (round 6): a push fused with the plain feature / constant load after it
          GK_CASES(H_PUSHLF0, { RR(S[k][r] = A[r]; set_feat<GM>(A[r], xat(opnd, rr), opnd - c0);) })
          GK_CASES(H_PUSHLC0, { RR(S[k][r] = A[r]; set_const<GM>(A[r], imm, opnd - c0);) })
#endif
          GK_CASES(H_SLOADF0, { RR(set_feat<GM>(S[k][r], xat(opnd, rr), opnd - c0);) })
          GK_CASES(H_SLOADC0, { RR(set_const<GM>(S[k][r], imm, opnd - c0);) })
// (AC / CA / SA / AS forms with UN_UNIFORM_FLAG in the operand field: two constant subtrees, one
// value per lane -- row 0 evaluated, copied to the others with their check folds)
#define GK_UNI_ROWS()                                                                              \
  UNR for (int r = 1; r < R; ++r) A[r] = A[0];                                                     \
  UNR for (int r = 0; r < R; ++r) chk_fold(M, A[r].v);
#if SRHIP_GRAD_SUPER_LEVEL >= 2
#define GK_LEAFLEAF(NAME)                                                                          \
  /* leaf-leaf forms (round 6): X[a] op X[imm], X[a] op c, c op X[a] -- c's index in the upper half */ \
  case h_spec(SB_##NAME, SPEC_FF): {                                                               \
    const int f2 = (int)(ins.imm & 0xffff);                                                        \
    RR(Dual<T, KT> o; set_feat<GM>(A[r], xat(opnd, rr), opnd - c0); set_feat<GM>(o, xat(f2, rr), f2 - c0); \
       T f, fl, fr; dual_spec<T, SB_##NAME>(A[r].v, o.v, f, fl, fr); combine(A[r], A[r], o, f, fl, fr); \
       chk_fold(M, A[r].v);) break; }                                                              \
  case h_spec(SB_##NAME, SPEC_FC): {                                                               \
    const int ci = (int)(ins.a >> 16) - c0;                                                        \
    RR(Dual<T, KT> o; set_feat<GM>(A[r], xat(opnd, rr), opnd - c0); set_const<GM>(o, imm, ci);     \
       T f, fl, fr; dual_spec<T, SB_##NAME>(A[r].v, o.v, f, fl, fr); combine(A[r], A[r], o, f, fl, fr); \
       chk_fold(M, A[r].v);) break; }                                                              \
  case h_spec(SB_##NAME, SPEC_CF): {                                                               \
    const int ci = (int)(ins.a >> 16) - c0;                                                        \
    RR(Dual<T, KT> o; set_feat<GM>(A[r], xat(opnd, rr), opnd - c0); set_const<GM>(o, imm, ci);     \
       T f, fl, fr; dual_spec<T, SB_##NAME>(o.v, A[r].v, f, fl, fr); combine(A[r], o, A[r], f, fl, fr); \
       chk_fold(M, A[r].v);) break; }
#else
#define GK_LEAFLEAF(NAME)
#endif
#define GK_SPEC(NAME, FN)                                                                          \
  GK_LEAFLEAF(NAME)                                                                                \
  case h_spec(SB_##NAME, SPEC_AF): {                                                               \
    RR(Dual<T, KT> o; set_feat<GM>(o, xat(opnd, rr), opnd - c0);                                   \
       T f, fl, fr; dual_spec<T, SB_##NAME>(A[r].v, o.v, f, fl, fr); combine(A[r], A[r], o, f, fl, fr); \
       chk_fold(M, A[r].v);) break; }                                                              \
  case h_spec(SB_##NAME, SPEC_FA): {                                                               \
    RR(Dual<T, KT> o; set_feat<GM>(o, xat(opnd, rr), opnd - c0);                                   \
       T f, fl, fr; dual_spec<T, SB_##NAME>(o.v, A[r].v, f, fl, fr); combine(A[r], o, A[r], f, fl, fr); \
       chk_fold(M, A[r].v);) break; }                                                              \
  case h_spec(SB_##NAME, SPEC_AC): {                                                               \
    const int ci = (opnd & ~(int)UN_UNIFORM_FLAG) - c0;                                            \
    if (R > 1 && (ins.a & UN_UNIFORM_FLAG)) {                                                      \
      Dual<T, KT> o; set_const<GM>(o, imm, ci);                                                    \
      T f, fl, fr; dual_spec<T, SB_##NAME>(A[0].v, o.v, f, fl, fr); combine(A[0], A[0], o, f, fl, fr); \
      GK_UNI_ROWS() break;                                                                         \
    }                                                                                              \
    RR(Dual<T, KT> o; set_const<GM>(o, imm, ci);                                                   \
       T f, fl, fr; dual_spec<T, SB_##NAME>(A[r].v, o.v, f, fl, fr); combine(A[r], A[r], o, f, fl, fr); \
       chk_fold(M, A[r].v);) break; }                                                              \
  case h_spec(SB_##NAME, SPEC_CA): {                                                               \
    const int ci = (opnd & ~(int)UN_UNIFORM_FLAG) - c0;                                            \
    if (R > 1 && (ins.a & UN_UNIFORM_FLAG)) {                                                      \
      Dual<T, KT> o; set_const<GM>(o, imm, ci);                                                    \
      T f, fl, fr; dual_spec<T, SB_##NAME>(o.v, A[0].v, f, fl, fr); combine(A[0], o, A[0], f, fl, fr); \
      GK_UNI_ROWS() break;                                                                         \
    }                                                                                              \
    RR(Dual<T, KT> o; set_const<GM>(o, imm, ci);                                                   \
       T f, fl, fr; dual_spec<T, SB_##NAME>(o.v, A[r].v, f, fl, fr); combine(A[r], o, A[r], f, fl, fr); \
       chk_fold(M, A[r].v);) break; }                                                              \
  GK_CASES(h_spec(SB_##NAME, SPEC_SA0), {                                                          \
    if (R > 1 && (ins.a & UN_UNIFORM_FLAG)) {                                                      \
      T f, fl, fr; dual_spec<T, SB_##NAME>(S[k][0].v, A[0].v, f, fl, fr);                          \
      combine(A[0], S[k][0], A[0], f, fl, fr); GK_UNI_ROWS() break;                                \
    }                                                                                              \
    RR(T f, fl, fr; dual_spec<T, SB_##NAME>(S[k][r].v, A[r].v, f, fl, fr);                         \
       combine(A[r], S[k][r], A[r], f, fl, fr); chk_fold(M, A[r].v);) })                           \
  GK_CASES(h_spec(SB_##NAME, SPEC_AS0), {                                                          \
    if (R > 1 && (ins.a & UN_UNIFORM_FLAG)) {                                                      \
      T f, fl, fr; dual_spec<T, SB_##NAME>(A[0].v, S[k][0].v, f, fl, fr);                          \
      combine(A[0], A[0], S[k][0], f, fl, fr); GK_UNI_ROWS() break;                                \
    }                                                                                              \
    RR(T f, fl, fr; dual_spec<T, SB_##NAME>(A[r].v, S[k][r].v, f, fl, fr);                         \
       combine(A[r], A[r], S[k][r], f, fl, fr); chk_fold(M, A[r].v);) })
          SRHIP_SPEC_BINOPS(GK_SPEC)
#undef GK_SPEC
#undef GK_LEAFLEAF
#define GK_HEAVY(NAME, FN)                                                                         \
  GK_CASES(h_heavy(HB_##NAME, HEAVY_SA0), {                                                        \
    RR(const typename V4<T>::type q = dual_heavy<T, HB_##NAME, (KT > 0)>(S[k][r].v, A[r].v);                 \
       combine(A[r], S[k][r], A[r], q[0], q[1], q[2]); chk_fold(M, A[r].v);) })                    \
  GK_CASES(h_heavy(HB_##NAME, HEAVY_AS0), {                                                        \
    RR(const typename V4<T>::type q = dual_heavy<T, HB_##NAME, (KT > 0)>(A[r].v, S[k][r].v);                 \
       combine(A[r], A[r], S[k][r], q[0], q[1], q[2]); chk_fold(M, A[r].v);) })
          SRHIP_HEAVY_BINOPS(GK_HEAVY)
#undef GK_HEAVY
#define GK_UN(NAME, FN)                                                                            \
  case h_un(UN_##NAME): {                                                                          \
    if (R > 1 && (ins.a & UN_UNIFORM_FLAG)) {  /* a constant subtree's rows: one evaluation */     \
      T f, df;                                                                                     \
      dual_un<T, UN_##NAME, (KT > 0)>(A[0].v, f, df);                                              \
      A[0].v = f;                                                                                  \
      UNR for (int j = 0; j < KT; ++j) A[0].d[j] = df * A[0].d[j];                                 \
      UNR for (int r = 0; r < R; ++r) { A[r] = A[0]; chk_fold(M, A[r].v); }                        \
      break;                                                                                       \
    }                                                                                              \
    if constexpr (KT == 0 && !dun_inline<UN_##NAME>()) {                                           \
      typename VR<T, R>::type xv;                                                                  \
      if constexpr (R == 1) xv = A[0].v;                                                           \
      else { UNR for (int r = 0; r < R; ++r) xv[r] = A[r].v; }                                     \
      xv = dual_un_heavy_rows<T, UN_##NAME, R>(xv);                                                \
      if constexpr (R == 1) { A[0].v = xv; chk_fold(M, A[0].v); }                                  \
      else { UNR for (int r = 0; r < R; ++r) { A[r].v = xv[r]; chk_fold(M, A[r].v); } }            \
      break;                                                                                       \
    }                                                                                              \
    RR(T f, df; dual_un<T, UN_##NAME, (KT > 0)>(A[r].v, f, df);                                              \
       A[r].v = f;                                                                                 \
       UNR for (int j = 0; j < KT; ++j) A[r].d[j] = df * A[r].d[j];                                \
       chk_fold(M, A[r].v);) break; }
          SRHIP_UNOPS(GK_UN)
#undef GK_UN
#undef GK_CASES
          default: break;
        }
#undef RR
      }
      if constexpr (GM != GMODE_LOSS) {
        // record: (tree, c0, end component, output row of component c0)
        const int cend = __builtin_amdgcn_readfirstlane(p.chunks[CW * chunk + 2]);
        const int orow = __builtin_amdgcn_readfirstlane(p.chunks[CW * chunk + 3]);
        UNR for (int r = 0; r < R; ++r) {
          const int64_t row = row_base + tb + 64 * r + lane;
          if (row < p.nvalid) {
            T* der = reinterpret_cast<T*>(p.out_der) + (int64_t)orow * p.nvalid + row;
            UNR for (int j = 0; j < KT; ++j)
              if (c0 + j < cend) der[(int64_t)j * p.nvalid] = A[r].d[j];
          }
        }
        continue;
      }
      UNR for (int r = 0; r < R; ++r) {
        const int rr = tb + 64 * r + lane;
        if (rr < nrel) {
          const T d = A[r].v - yat(rr);
          T l, dl;
          if (p.loss_kind == SRHIP_LOSS_L2) {
            l = d * d;
            dl = T(2) * d;
          } else {
            const typename V2<T>::type q = loss_dloss_generic<T>(p.loss_kind, A[r].v, yat(rr), p0);
            l = q[0];
            dl = q[1];
          }
          if (p.weighted) {
            const T w = W[row_base + rr];
            l = w * l;
            dl = w * dl;
          }
          lacc += (double)l;
          UNR for (int j = 0; j < KT; ++j) gacc[j] += (double)(dl * A[r].d[j]);
        }
      }
    }
    if constexpr (GM != GMODE_LOSS) continue;
    // wave reductions, one slab entry per (chunk, row block)
    auto level = [&](auto oc) {
      constexpr int O = decltype(oc)::value;
      lacc += xor_lane<O>(lacc, lane);
      UNR for (int j = 0; j < KT; ++j) gacc[j] += xor_lane<O>(gacc[j], lane);
      if constexpr (sizeof(T) == 4) M = __builtin_elementwise_maximum(M, xor_lane<O>(M, lane));
      else M += xor_lane<O>(M, lane);
    };
    level(std::integral_constant<int, 32>());
    level(std::integral_constant<int, 16>());
    level(std::integral_constant<int, 8>());
    level(std::integral_constant<int, 4>());
    level(std::integral_constant<int, 2>());
    level(std::integral_constant<int, 1>());
    if (lane == 0) {
      double* out = p.slab + ((int64_t)chunk * p.nrb + rb) * (KT + 2);
      out[0] = lacc;
      UNR for (int j = 0; j < KT; ++j) out[1 + j] = gacc[j];
      out[KT + 1] = (double)M;
    }
  }
}

// per-chunk fixed-order reduction over row blocks: one wave per chunk
template <int KT, bool CHK_MAX>
__global__ __launch_bounds__(256) void grad_reduce_kernel(const double* __restrict__ slab, int nrb, int nchunks,
                                                          double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (chunk >= nchunks) return;
  // (each lane folds its row blocks b = lane, lane + 64, ... in order -- the loads of a batch issued
  // before its adds: a strided loop waited out one memory latency per block and element)
  constexpr int BB = 8;
  for (int e = 0; e < KT + 2; ++e) {
    const bool is_max = CHK_MAX && e == KT + 1;
    double s = 0.0;
    for (int b0 = lane; b0 < nrb; b0 += 64 * BB) {
      double v[BB];
      UNR for (int j = 0; j < BB; ++j) {
        const int b = b0 + 64 * j;
        v[j] = b < nrb ? slab[((int64_t)chunk * nrb + b) * (KT + 2) + e] : 0.0;
      }
      UNR for (int j = 0; j < BB; ++j) {
        if (b0 + 64 * j >= nrb) break;
        s = is_max ? __builtin_elementwise_maximum(s, v[j]) : s + v[j];
      }
    }
    UNR for (int o = 32; o > 0; o >>= 1) {
      const double t = __shfl_xor(s, o);
      s = is_max ? __builtin_elementwise_maximum(s, t) : s + t;
    }
    if (lane == 0) out[(int64_t)chunk * (KT + 2) + e] = s;
  }
}

// LDS staging of the row block when it fits (few features): [nfeat + 1][rb_rows] elements
constexpr size_t GRAD_LDS_MAX = 48 * 1024;
template <typename T> static size_t grad_lds_bytes(const GradArgs& a) {
  return (size_t)(a.nfeat + 1) * (size_t)a.rb_rows * sizeof(T);
}

// rows per lane: value-only passes (no tangents) carry 4 rows per lane (one dispatch per 256-row
// block); with tangents the register budget decides (GRAD_R)
// (K = 2, the common shallow-stack population -- C4's size-20 trees all fit it -- leaves room for two
// rows per lane with 4 tangents: half the dispatches per row at the same waves per SIMD)
template <int KT, int K> constexpr int grad_rows() {
  return KT == 0 ? 4 : (KT <= 4 && K <= 2 ? 2 : (KT <= 4 && K <= 4 ? GRAD_R : 1));
}

template <typename T, int KT, int K, int GM = GMODE_LOSS>
static hipError_t launch_grad_t(const GradArgs& a, dim3 grid, hipStream_t s) {
  constexpr int R = grad_rows<KT, K>();
  if (a.rb_rows % (64 * R)) return hipErrorInvalidValue;
  const size_t lds = grad_lds_bytes<T>(a);
  if (lds <= GRAD_LDS_MAX)
    hipLaunchKernelGGL((grad_kernel<T, KT, K, GM, true, R>), grid, dim3(64 * GRAD_WAVES), lds, s, a);
  else
    hipLaunchKernelGGL((grad_kernel<T, KT, K, GM, false, R>), grid, dim3(64 * GRAD_WAVES), 0, s, a);
  return hipGetLastError();
}

template <typename T, int GM>
static hipError_t launch_grad_rows_t(int K, const GradArgs& a, dim3 grid, hipStream_t s) {
  return K <= 4 ? launch_grad_t<T, GRAD_ROW_KT, 4, GM>(a, grid, s) : launch_grad_t<T, GRAD_ROW_KT, 8, GM>(a, grid, s);
}

hipError_t launch_grad_rows(int dtype, int K, int gmode, const GradArgs& a, dim3 grid, hipStream_t s) {
  if (gmode != GMODE_ROWC && gmode != GMODE_ROWF) return hipErrorInvalidValue;
  switch (dtype) {
    case SRHIP_F32:
      return gmode == GMODE_ROWC ? launch_grad_rows_t<float, GMODE_ROWC>(K, a, grid, s)
                                 : launch_grad_rows_t<float, GMODE_ROWF>(K, a, grid, s);
    case SRHIP_F64:
      return gmode == GMODE_ROWC ? launch_grad_rows_t<double, GMODE_ROWC>(K, a, grid, s)
                                 : launch_grad_rows_t<double, GMODE_ROWF>(K, a, grid, s);
    default: return hipErrorInvalidValue;
  }
}


// A derived view's derived columns (srhip_optim.cpp derived_view): Xd[j][row] = U_j(X[f_j][row]) over
// the view's ld rows, with the gradient kernel's own value function (the bits the kernel computes in
// place), and after the nd of them the tangent-zero columns Xd[nd + j][row] = U_j'(x) * 0 -- what the
// kernel's tangents of U_j(feature) are (a feature's tangent is +0): +-0, or NaN where U_j' is not finite.
struct DeriveSpec {
  uint32_t key[32];  // u << 16 | feature column
};
template <typename T>
__global__ __launch_bounds__(256) void grad_derive_kernel(const T* __restrict__ X, T* __restrict__ Xd, int64_t ld,
                                                          DeriveSpec spec) {
  const int j = blockIdx.y;
  const int u = (int)(spec.key[j] >> 16), f = (int)(spec.key[j] & 0xffff);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ld; i += (int64_t)gridDim.x * blockDim.x) {
    const T x = X[(int64_t)f * ld + i];
    T v = x, dv = T(0), v1, dv1;
    switch (u) {
#define X_(NAME, FN) \
  case UN_##NAME: dual_un<T, UN_##NAME, false>(x, v, dv1); dual_un<T, UN_##NAME, true>(x, v1, dv); break;
      SRHIP_UNOPS(X_)
#undef X_
      default: break;
    }
    Xd[(int64_t)j * ld + i] = v;
    Xd[(int64_t)(gridDim.y + j) * ld + i] = dv * T(0);
  }
}
hipError_t launch_grad_derive(int dtype, const void* X, void* Xd, int64_t ld, const uint32_t* keys, int nd,
                              hipStream_t s) {
  if (nd <= 0) return hipSuccess;
  if (nd > 32) return hipErrorInvalidValue;
  DeriveSpec spec{};
  for (int j = 0; j < nd; ++j) spec.key[j] = keys[j];
  const dim3 grid((unsigned)std::min<int64_t>((ld + 255) / 256, 1024), (unsigned)nd);
  if (dtype == SRHIP_F64)
    hipLaunchKernelGGL(grad_derive_kernel<double>, grid, dim3(256), 0, s, (const double*)X, (double*)Xd, ld, spec);
  else
    hipLaunchKernelGGL(grad_derive_kernel<float>, grid, dim3(256), 0, s, (const float*)X, (float*)Xd, ld, spec);
  return hipGetLastError();
}
hipError_t launch_grad(int dtype, int K, int kt, const GradArgs& a, dim3 grid, hipStream_t s) {
  if (kt != 0 && kt != 4 && kt != GRAD_KT) return hipErrorInvalidValue;
  switch (dtype) {
    case SRHIP_F32:
      if (kt == 0) return K <= 4 ? launch_grad_t<float, 0, 4>(a, grid, s) : launch_grad_t<float, 0, 8>(a, grid, s);
      if (kt == 4) return K <= 4 ? launch_grad_t<float, 4, 4>(a, grid, s) : launch_grad_t<float, 4, 8>(a, grid, s);
      return K <= 4 ? launch_grad_t<float, GRAD_KT, 4>(a, grid, s) : launch_grad_t<float, GRAD_KT, 8>(a, grid, s);
    case SRHIP_F64:  // K = 2 variants for shallow-stack populations (fewer VGPRs: two rows per lane)
      if (kt == 0)
        return K <= 2 ? launch_grad_t<double, 0, 2>(a, grid, s)
             : K <= 4 ? launch_grad_t<double, 0, 4>(a, grid, s) : launch_grad_t<double, 0, 8>(a, grid, s);
      if (kt == 4)
        return K <= 2 ? launch_grad_t<double, 4, 2>(a, grid, s)
             : K <= 4 ? launch_grad_t<double, 4, 4>(a, grid, s) : launch_grad_t<double, 4, 8>(a, grid, s);
      return K <= 2 ? launch_grad_t<double, GRAD_KT, 2>(a, grid, s)
           : K <= 4 ? launch_grad_t<double, GRAD_KT, 4>(a, grid, s) : launch_grad_t<double, GRAD_KT, 8>(a, grid, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_grad_reduce(int dtype, int kt, const double* slab, int nrb, int nchunks, double* out, hipStream_t s) {
  if (kt != 0 && kt != 4 && kt != GRAD_KT) return hipErrorInvalidValue;
  dim3 grid((nchunks + 3) / 4), block(256);
  if (kt == 0) {
    if (dtype == SRHIP_F32) hipLaunchKernelGGL((grad_reduce_kernel<0, true>), grid, block, 0, s, slab, nrb, nchunks, out);
    else hipLaunchKernelGGL((grad_reduce_kernel<0, false>), grid, block, 0, s, slab, nrb, nchunks, out);
    return hipGetLastError();
  }
  if (dtype == SRHIP_F32) {
    if (kt == 4) hipLaunchKernelGGL((grad_reduce_kernel<4, true>), grid, block, 0, s, slab, nrb, nchunks, out);
    else hipLaunchKernelGGL((grad_reduce_kernel<GRAD_KT, true>), grid, block, 0, s, slab, nrb, nchunks, out);
  } else {
    if (kt == 4) hipLaunchKernelGGL((grad_reduce_kernel<4, false>), grid, block, 0, s, slab, nrb, nchunks, out);
    else hipLaunchKernelGGL((grad_reduce_kernel<GRAD_KT, false>), grid, block, 0, s, slab, nrb, nchunks, out);
  }
  return hipGetLastError();
}

}  // namespace srhip
