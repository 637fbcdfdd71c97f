// srhip_eval_impl.h — the interpreter kernel eval_kernel<T, R, K, MODE, XLDS> and its device helpers,
// included by the per-variant translation units srhip_eval_<dtype>_<mode>.hip (each instantiates one
// slice of the variant space, so the slices compile in parallel) and by srhip_eval.hip (reduction,
// gather, feature statistics and the launch dispatch).
//
// One workgroup owns a block of RB dataset rows
// (staged once into LDS: X[f][RB], y, w) and its waves interpret many trees over those rows.
// A wave holds R rows per lane (64*R rows = one tile) in VGPRs; the bytecode is wave-uniform
// and read with scalar loads, so the interpreter's dispatch runs on the SALU/branch unit while
// the VALU does the arithmetic.  MUST be compiled with
//     -mllvm -structurizecfg-skip-uniform-regions=true
// so the uniform opcode switch lowers to a scalar branch tree with in-place VGPR updates
// (without it, the CFG structurizer inserts R phi copies per case per dispatch).
//
// Replaces (reference): DynamicExpressions.eval_tree_array's array-at-a-time recursion (one
// Vector{T}(n) per node + an isfinite(sum) pass per child array) and LossFunctions' mean/sum
// (src/LossFunctions.jl:13-33, 45-75).  See DESIGN.md for the did_succeed mapping.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "srhip_isa.h"
#include "srhip_kernels.h"
#include "srhip_ops.h"

#define UNR _Pragma("unroll")
// SRHIP_KDEBUG builds (diagnostic only): lane 0 of wave 0 of block (0,0) printfs its progress.
#ifdef SRHIP_KDEBUG
#define KDBG(...) do { if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) printf(__VA_ARGS__); } while (0)
#else
#define KDBG(...) do { } while (0)
#endif
// Progress words for SRHIP_TRACE runs of SRHIP_KTRACE builds (make EXTRA=-DSRHIP_KTRACE, diagnostic
// only): lane 0 of wave 0 of block (0,0) stores (slot, value) to host-coherent memory with system
// scope, so the host can read them while the kernel runs.  Compiled out otherwise: the stores'
// operands pinned v0-v1 and moved the accumulator off v0-v15 after every tile.
#ifdef SRHIP_KTRACE
#define KMARK(slot, val)                                                                       \
  do {                                                                                         \
    if (p.dbg && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                      \
      __hip_atomic_store(p.dbg + (slot), (int32_t)(val), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
  } while (0)
#else
#define KMARK(slot, val) do { } while (0)
#endif
#ifndef SRHIP_HEAVY_ILP
#define SRHIP_HEAVY_ILP 1  // rows a heavy operator body may interleave
#endif
#ifndef SRHIP_TRIG_ILP
#ifndef SRHIP_JTRIG_FAST
#define SRHIP_JTRIG_FAST 1  // Julia's Float32 trig kernels in Horner form, tie rows re-evaluated (round 6)
#endif
#define SRHIP_TRIG_ILP SRHIP_HEAVY_ILP  // rows Julia's Float32 trig bodies interleave (jtrigf_*); 1/2/4 measured alike (C2 1.278-1.289 ms)
#endif
#ifndef SRHIP_TRIG_ROWS
#define SRHIP_TRIG_ROWS 1  // Float32 cos/sin/tan batched over the rows (trigf_rows)
#endif
// Hot handlers (SRHIP_HOT_CASES): the switch's binary search is built weighted by case likelihood,
// so the commonest handlers -- loads, pushes, + - * / in every operand form, the common unary
// operators -- sit near the root of the compare-and-branch tree
#ifndef SRHIP_HOT_CASES
#define SRHIP_HOT_CASES 0
#endif
#if SRHIP_HOT_CASES
#define SRHIP_LK [[likely]]
#else
#define SRHIP_LK
#endif
#define SRHIP_HOTB_ADD SRHIP_LK
#define SRHIP_HOTB_SUB SRHIP_LK
#define SRHIP_HOTB_MUL SRHIP_LK
#define SRHIP_HOTB_DIV SRHIP_LK
#define SRHIP_HOTB_GREATER
#define SRHIP_HOTB_COND
#define SRHIP_HOTB_LOGICAL_OR
#define SRHIP_HOTB_LOGICAL_AND
#define SRHIP_HOTB_MAX
#define SRHIP_HOTB_MIN
#define SRHIP_HOTU_NEG SRHIP_LK
#define SRHIP_HOTU_SQUARE SRHIP_LK
#define SRHIP_HOTU_CUBE SRHIP_LK
#define SRHIP_HOTU_ABS SRHIP_LK
#define SRHIP_HOTU_RELU
#define SRHIP_HOTU_COS SRHIP_LK
#define SRHIP_HOTU_SIN SRHIP_LK
#define SRHIP_HOTU_TAN
#define SRHIP_HOTU_EXP SRHIP_LK
#define SRHIP_HOTU_LOG SRHIP_LK
#define SRHIP_HOTU_LOG2
#define SRHIP_HOTU_LOG10
#define SRHIP_HOTU_LOG1P
#define SRHIP_HOTU_SQRT
#define SRHIP_HOTU_ACOSH
#define SRHIP_HOTU_ATANH_CLIP
#define SRHIP_HOTU_SINH
#define SRHIP_HOTU_COSH
#define SRHIP_HOTU_TANH
#define SRHIP_HOTU_ASIN
#define SRHIP_HOTU_ACOS
#define SRHIP_HOTU_ATAN
#define SRHIP_HOTU_ASINH
#define SRHIP_HOTU_ERF
#define SRHIP_HOTU_ERFC
#define SRHIP_HOTU_GAMMA
#define SRHIP_HOTU_ROUND
#define SRHIP_HOTU_FLOOR
#define SRHIP_HOTU_CEIL
#define SRHIP_HOTU_SIGN
#define SRHIP_HOTU_EXP2
#define SRHIP_HOTU_EXPM1
#define SRHIP_HOTU_CBRT
// SRHIP_ASM_DEF=1 (default): the tile's accumulator and stack registers are defined by empty asm
// statements instead of 16 x (K + 1) clears per (tree, tile) (C2, one MI355X: 1.12-1.15 ->
// 1.085-1.095 ms; -DSRHIP_ASM_DEF=0 restores the clears)
#ifndef SRHIP_ASM_DEF
#define SRHIP_ASM_DEF 1
#endif
#ifndef SRHIP_ROW_FENCE
#define SRHIP_ROW_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

namespace srhip {

template <typename T> constexpr bool kIsInt = std::is_same<T, int32_t>::value;

// threadIdx.x for the once-per-row-block setup code (staging, mark snapshot, derived columns): an
// opaque copy at the use site, so the LDS addresses derived from it are computed there instead of
// hoisted to the kernel's entry -- hoisted, they stayed live across the interpreter loop and the
// register allocator spilled seven of them to scratch in every wave's preamble (28 bytes per lane,
// ~7 MB of scratch writes per launch of 4096 waves)
__device__ __attribute__((always_inline)) inline int tid_x() {
  int t = (int)__builtin_amdgcn_workitem_id_x();
  asm volatile("" : "+v"(t));
  return t;
}

template <typename T>
using OpsT = typename std::conditional<kIsInt<T>, IOps, FOps<typename std::conditional<kIsInt<T>, float, T>::type>>::type;

// Which handlers exist for T (Int32 trees: ring ops and comparisons only).
template <typename T> __device__ constexpr bool sb_ok(int sb) {
  return !kIsInt<T> || sb != SB_DIV;
}
template <typename T> __device__ constexpr bool hb_ok(int) { return !kIsInt<T>; }
template <typename T> __device__ constexpr bool un_ok(int u) {
  return !kIsInt<T> || u == UN_NEG || u == UN_SQUARE || u == UN_CUBE || u == UN_ABS ||
         u == UN_RELU || u == UN_SIGN;
}

// 16-byte vector of T
template <typename T> struct Vec16;
template <> struct Vec16<float> { typedef float __attribute__((ext_vector_type(4))) type; };
template <> struct Vec16<int32_t> { typedef int32_t __attribute__((ext_vector_type(4))) type; };
template <> struct Vec16<double> { typedef double __attribute__((ext_vector_type(2))) type; };

// A lane's R rows of one tile, as one vector value (a VGPR tuple): packed row-pair operations
// (v_pk_*) read and write aligned sub-pairs of it in place.
template <typename T, int R> struct RowVec { typedef T type __attribute__((ext_vector_type(R))); };
template <typename T, int R> using RV = typename RowVec<T, R>::type;

// Rows of one tile owned by a lane: register r holds tile row
//   (r / VEC) * 64 * VEC + lane * VEC + (r % VEC)        (VEC = 16 / sizeof(T))
// so every access to a column is one 16-byte load per lane, contiguous across the wave.
template <typename T, int R>
__device__ __attribute__((always_inline)) inline void load_rows(const T* base, int lane, RV<T, R>& v) {
  constexpr int VEC = 16 / sizeof(T);
  using V = typename Vec16<T>::type;
  UNR for (int j = 0; j < R / VEC; ++j) {
    const V q = reinterpret_cast<const V*>(base)[j * 64 + lane];
    UNR for (int e = 0; e < VEC; ++e) v[j * VEC + e] = q[e];
  }
}

#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) Ins CIns;  // constant address space: scalar loads
#else
typedef const Ins CIns;
#endif

template <typename T> __device__ __attribute__((always_inline)) inline T imm_as(uint64_t bits) {
  if constexpr (sizeof(T) == 8) {
    return __builtin_bit_cast(T, bits);
  } else {
    return __builtin_bit_cast(T, (uint32_t)bits);
  }
}

// ---- heavy operators: one out-of-line body per (T, R, op), called by every kernel variant ----
// Transcendentals are 20-60 VALU instructions per row; inlining them R times into every handler of
// every kernel variant made a ~700k-instruction kernel whose hot loop thrashed the instruction
// cache (SQ_IFETCH ~ 0.4 x SQ_INSTS).  Out of line, the dispatch loop and the cheap handlers stay
// compact and each heavy body exists once; the R rows travel in VGPRs (vector argument/return).

// v_cvt_i32_f64 as an opaque instruction: saturating for out-of-range input and 0 for NaN (the C++
// conversion of such values is undefined, and the compiler may exploit that).
__device__ __attribute__((always_inline)) inline int cvt_i32_sat(double k) {
  int m;
  asm("v_cvt_i32_f64 %0, %1" : "=v"(m) : "v"(k));
  return m;
}

// srm_sincosf_fast (include/srhip_math.h) for the device rows, bit-identical for every finite x:
// the sign (-1)^(m+1) of cos is a free negation modifier on the product plus the bit of m, and
// Inf / NaN need no select: they reach here unreduced and come out of the reduction as NaN.
template <int KIND>
__device__ __attribute__((always_inline)) inline float sincosf_dev(double x) {
  const double invpi = 0.3183098861837907, pi_hi = 3.141592653589793, pi_lo = 1.2246467991473532e-16;
  double k = __builtin_rint(__builtin_fma(x, invpi, KIND == 0 ? -0.5 : 0.0));
  const int m = cvt_i32_sat(k);
  if (KIND == 0) k += 0.5;
  const double y = __builtin_fma(-k, pi_lo, __builtin_fma(-k, pi_hi, x));
  const double p = srm_psin(y * y);
  const float r = KIND == 0 ? (float)(-y * p) : (float)(y * p);
  // sign flip by m's low bit: adding m << 31 is the xor on the sign bit (the carry leaves the word),
  // one v_lshl_add_u32 instead of a shift and an xor
  uint32_t o;
  asm("v_lshl_add_u32 %0, %1, 31, %2" : "=v"(o) : "v"(m), "v"(__builtin_bit_cast(uint32_t, r)));
  return __builtin_bit_cast(float, o);
}

// Julia's Float32 exp (include/srhip_math.h srm_expf) on two rows per instruction: the clamp to
// [-104, 89] (NaN-propagating minimum / maximum) replaces srm_expf's Inf / 0 branches and every other
// step is the same Float32 operation, packed (v_pk_mul_f32, v_pk_fma_f32); v_cvt_i32_f32 saturates and
// maps NaN to 0, v_ldexp_f32 rounds once.  tools/check_expf.c proves this formulation bit-identical
// to srm_expf on all 2^32 inputs (NaN in, NaN out).
typedef float F2 __attribute__((ext_vector_type(2)));
__device__ __attribute__((always_inline)) inline int cvt_i32_f32(float x) {
  int m;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(m) : "v"(x));
  return m;
}
__device__ __attribute__((always_inline)) inline F2 expf2_dev(F2 x) {
  x = __builtin_elementwise_minimum(__builtin_elementwise_maximum(x, (F2)(-104.0f)), (F2)(89.0f));
  F2 n = x * (F2)(SRM_EXPF_LOG2E);
  n.x = __builtin_rintf(n.x);
  n.y = __builtin_rintf(n.y);
  F2 r = __builtin_elementwise_fma(n, (F2)(SRM_EXPF_NLN2_HI), x);
  r = __builtin_elementwise_fma(n, (F2)(SRM_EXPF_NLN2_LO), r);
  F2 p = __builtin_elementwise_fma(r, (F2)(SRM_EXPF_C6), (F2)(SRM_EXPF_C5));
  p = __builtin_elementwise_fma(r, p, (F2)(SRM_EXPF_C4));
  p = __builtin_elementwise_fma(r, p, (F2)(SRM_EXPF_C3));
  p = __builtin_elementwise_fma(r, p, (F2)(0.5f));
  p = __builtin_elementwise_fma(r, p, (F2)(1.0f));
  p = __builtin_elementwise_fma(r, p, (F2)(1.0f));
  F2 out;
  out.x = __builtin_ldexpf(p.x, cvt_i32_f32(n.x));
  out.y = __builtin_ldexpf(p.y, cvt_i32_f32(n.y));
  return out;
}

// The same exp for waves whose inputs all satisfy |x| <= 87 (EXPF_FAST_MAX): no clamp; n = rint(x log2 e)
// by adding and removing 1.5 * 2^23 (the same ties-to-even rounding of the same Float32 product), and
// 2^n (a normal float for |n| <= 126) built in the exponent field from the low bits of that sum, one
// multiply instead of v_cvt_i32 + v_ldexp (both round the exact p 2^n once).  tools/check_expf.c
// proves it bit-identical to srm_expf on every float in range.
constexpr float EXPF_FAST_MAX = 87.0f;
__device__ __attribute__((always_inline)) inline F2 expf2_fast(F2 x) {
  const F2 t = x * (F2)(SRM_EXPF_LOG2E) + (F2)(12582912.0f);
  const F2 n = t - (F2)(12582912.0f);
  F2 r = __builtin_elementwise_fma(n, (F2)(SRM_EXPF_NLN2_HI), x);
  r = __builtin_elementwise_fma(n, (F2)(SRM_EXPF_NLN2_LO), r);
  F2 p = __builtin_elementwise_fma(r, (F2)(SRM_EXPF_C6), (F2)(SRM_EXPF_C5));
  p = __builtin_elementwise_fma(r, p, (F2)(SRM_EXPF_C4));
  p = __builtin_elementwise_fma(r, p, (F2)(SRM_EXPF_C3));
  p = __builtin_elementwise_fma(r, p, (F2)(0.5f));
  p = __builtin_elementwise_fma(r, p, (F2)(1.0f));
  p = __builtin_elementwise_fma(r, p, (F2)(1.0f));
  // (opaque per row: left to itself the compiler built one scale and broadcast it to both rows)
  float s0, s1;
  asm("v_lshl_add_u32 %0, %1, 23, 1.0" : "=v"(s0) : "v"(t.x));
  asm("v_lshl_add_u32 %0, %1, 23, 1.0" : "=v"(s1) : "v"(t.y));
  return p * (F2){s0, s1};
}

// Float32 cos/sin/tan over a lane's R rows.  Every row takes the fast path; rows outside it are
// redone by the scalar srm_trigf out of line, once per call and only if some row needs it.  The
// same pieces as the scalar srm_trigf (include/srhip_math.h), so the values are bit-identical.
// (A call inside the batched body would pin its live rows to callee-saved, high-numbered VGPRs.)
// cos / sin: no per-row range test or select.  Large, Inf and NaN rows reduce to garbage; one
// NaN-propagating max |x| over the lane's rows (v_maximum3_f32, half an instruction per row) tells
// whether any row needs the scalar path, which redoes exactly the rows with !(|x| < 2^28 pi/2) from
// the inputs (Inf / NaN -> NaN as srm_trigf).  Measured against a per-row v_cmp + v_cndmask that
// marks the rows by keeping x (one instruction fewer per row, as the inputs need not stay live):
// the select form was 1-2 % slower on C2 (scripts/ab.sh, round 2).  tan (KIND 2): Inf / NaN handled
// inline, finite large rows redone the same way.
// Smallest float above SRM_PIO2F_BIG (not itself a float): for every float a,
// (double)|a| < SRM_PIO2F_BIG  <=>  |a| < SRM_PIO2F_BIG_F.
#define SRM_PIO2F_BIG_F 421657440.0f
template <int R>
__device__ __attribute__((noinline)) RV<float, R> trigf_fix_tan(RV<float, R> v, RV<float, R> res) {
  UNR for (int r = 0; r < R; ++r) {
    const float x = v[r];
    if (x - x == 0.0f && srm_pio2f_is_big((double)x)) res[r] = srm_trigf(2, x);
  }
  return res;
}
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> trigf_fix(RV<float, R> v, RV<float, R> res) {
  UNR for (int r = 0; r < R; ++r) {
    const float x = v[r];
    if (!(__builtin_fabsf(x) < SRM_PIO2F_BIG_F)) res[r] = srm_trigf(KIND, x);  // Inf / NaN: x - x
  }
  return res;
}
// Float32 cos / sin of a lane's R rows as two leaf bodies: the handler tests the wave's rows first
// (one NaN-propagating max |x| per row pair, a ballot) and calls trigf_fast -- every row in the
// fast range, computed in place, no call inside, so no return-address save and no copy of the
// inputs -- or, if any row of the wave is outside it (|x| >= 2^28 pi/2, Inf, NaN), trigf_slow,
// which takes the scalar srm_trigf path for those rows.  The same values as trigf_rows.
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> trigf_fast(RV<float, R> v) {
  UNR for (int r = 0; r < R; ++r) {
    v[r] = sincosf_dev<KIND>((double)v[r]);
    if ((r + 1) % SRHIP_HEAVY_ILP == 0) SRHIP_ROW_FENCE();
  }
  return v;
}
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> trigf_slow(RV<float, R> v) {
  UNR for (int r = 0; r < R; ++r) {
    const float x = v[r];
    v[r] = __builtin_fabsf(x) < SRM_PIO2F_BIG_F ? sincosf_dev<KIND>((double)x) : srm_trigf(KIND, x);
  }
  return v;
}
// NaN-propagating max (min) |v| over a lane's rows folded into m: one v_maximum3_f32 (v_minimum3_f32)
// per row pair, the whole chain in ONE asm statement -- the hazard recognizer cannot see into an asm
// statement and padded every dependent pair of single-instruction statements with an s_nop (one per
// two rows of every check fold; the chain itself has no hazard)
#define SRHIP_M3(OP, a, b) OP " %0, %0, |%" #a "|, |%" #b "|\n\t"
template <int R, bool MAX>
__device__ __attribute__((always_inline)) inline float abs_fold(float m, const RV<float, R>& v) {
#define SRHIP_OPC (MAX ? "v_maximum3_f32" : "v_minimum3_f32")
  if constexpr (R == 16) {
    if constexpr (MAX)
      asm(SRHIP_M3("v_maximum3_f32", 1, 2) SRHIP_M3("v_maximum3_f32", 3, 4) SRHIP_M3("v_maximum3_f32", 5, 6)
          SRHIP_M3("v_maximum3_f32", 7, 8) SRHIP_M3("v_maximum3_f32", 9, 10) SRHIP_M3("v_maximum3_f32", 11, 12)
          SRHIP_M3("v_maximum3_f32", 13, 14) SRHIP_M3("v_maximum3_f32", 15, 16)
          : "+v"(m) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
            "v"(v[8]), "v"(v[9]), "v"(v[10]), "v"(v[11]), "v"(v[12]), "v"(v[13]), "v"(v[14]), "v"(v[15]));
    else
      asm(SRHIP_M3("v_minimum3_f32", 1, 2) SRHIP_M3("v_minimum3_f32", 3, 4) SRHIP_M3("v_minimum3_f32", 5, 6)
          SRHIP_M3("v_minimum3_f32", 7, 8) SRHIP_M3("v_minimum3_f32", 9, 10) SRHIP_M3("v_minimum3_f32", 11, 12)
          SRHIP_M3("v_minimum3_f32", 13, 14) SRHIP_M3("v_minimum3_f32", 15, 16)
          : "+v"(m) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
            "v"(v[8]), "v"(v[9]), "v"(v[10]), "v"(v[11]), "v"(v[12]), "v"(v[13]), "v"(v[14]), "v"(v[15]));
  } else if constexpr (R == 32) {
    RV<float, 16> lo, hi;
    UNR for (int r = 0; r < 16; ++r) { lo[r] = v[r]; hi[r] = v[16 + r]; }
    m = abs_fold<16, MAX>(m, lo);
    m = abs_fold<16, MAX>(m, hi);
  } else if constexpr (R == 8) {
    if constexpr (MAX)
      asm(SRHIP_M3("v_maximum3_f32", 1, 2) SRHIP_M3("v_maximum3_f32", 3, 4) SRHIP_M3("v_maximum3_f32", 5, 6)
          SRHIP_M3("v_maximum3_f32", 7, 8)
          : "+v"(m) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
    else
      asm(SRHIP_M3("v_minimum3_f32", 1, 2) SRHIP_M3("v_minimum3_f32", 3, 4) SRHIP_M3("v_minimum3_f32", 5, 6)
          SRHIP_M3("v_minimum3_f32", 7, 8)
          : "+v"(m) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
  } else {
    static_assert(R % 2 == 0, "row pairs");
    UNR for (int r = 0; r < R; r += 2) {
      if constexpr (MAX) asm("v_maximum3_f32 %0, %1, |%2|, |%3|" : "=v"(m) : "v"(m), "v"(v[r]), "v"(v[r + 1]));
      else asm("v_minimum3_f32 %0, %1, |%2|, |%3|" : "=v"(m) : "v"(m), "v"(v[r]), "v"(v[r + 1]));
    }
  }
#undef SRHIP_OPC
  return m;
}

template <int R> __device__ __attribute__((always_inline)) inline bool trigf_rows_fast(const RV<float, R>& A) {
  const float mx = abs_fold<R, true>(0.0f, A);
  return __builtin_amdgcn_ballot_w64(!(mx < SRM_PIO2F_BIG_F)) == 0;  // false for NaN
}

// ---- Julia's own Float32 cos / sin (the default: SRHIP_JULIA_TRIG, include/srhip_math.h) -----------
// Julia evaluates sin(x::Float32) / cos(x::Float32) by quadrant with two different Float64 kernels
// (FreeBSD __kernel_sindf / __kernel_cosdf) after its rem_pio2_kernel, whose reduction itself changes
// with |x|.  Per row that is a case analysis a SIMD lane would pay in full, so the handler classifies
// the WAVE by its largest |x| (one NaN-propagating max per row pair and up to three ballots) and runs
// one of four branch-free leaf bodies, each proven equal to srm_jtrigf on every float it may see
// (tools/check_trigf.c, all 2^32 inputs):
//   A  every |x| < Float32(pi)/4: no reduction, ONE kernel (sin: the sign of x copied onto it);
//   B  every |x| <= pi*9/4: fn = rint(xd 2/pi), y = xd - fn (pi/2) (Julia's +-k pi/2 cases, one
//      rounding), both kernels, the quadrant picks one and its sign;
//   C  every |x| < 2^28 pi/2: per row Julia's choice between that y and its Cody-Waite reduction (cos:
//      Cody-Waite for every row -- on every float it returns what the +-k pi/2 cases return; sin
//      differs at x = +-3.0061);
//   slow  any larger / Inf / NaN row: C for the rest, the scalar srm_jtrigf (Payne-Hanek) for those.
// C2's cos-of-operator tiles fall 11 % / 47 % / 36 % / 6 % into A / B / C / slow
// (scripts/trig_arg_tiers.py).
template <int KIND>
__device__ __attribute__((always_inline)) inline float jtrigf_q_dev(double fn, double y) {
  const int n = cvt_i32_sat(fn);
  const float fs = (float)srm_jsin_kernel(y), fc = (float)srm_jcos_kernel(y);
  const float r = ((n & 1) ^ KIND) ? fs : fc;
  // the sign: bit 1 of n + 1 - KIND (cos: quadrants 1, 2; sin: 2, 3), added into bit 31 (the xor)
  uint32_t o;
  asm("v_lshl_add_u32 %0, %1, 31, %2" : "=v"(o) : "v"((n + 1 - KIND) >> 1), "v"(__builtin_bit_cast(uint32_t, r)));
  return __builtin_bit_cast(float, o);
}
template <int R, int KIND>
__device__ __attribute__((always_inline)) inline RV<float, R> jtrigf_a_exact(RV<float, R> v) {
  UNR for (int r = 0; r < R; ++r) {
    const float x = v[r];
    if constexpr (KIND == 0) {
      v[r] = (float)srm_jcos_kernel((double)x);
    } else {
      v[r] = __builtin_copysignf((float)srm_jsin_kernel((double)x), x);
    }
    if ((r + 1) % SRHIP_TRIG_ILP == 0) SRHIP_ROW_FENCE();
  }
  return v;
}
template <int KIND, bool CW>
__device__ __attribute__((always_inline)) inline double jtrigf_red(float x, double& fn) {
  const double xd = (double)x;
  fn = srm_jfn(xd);
  double y;
  if constexpr (CW && KIND == 0) {
    // cos: the Cody-Waite reduction gives Julia's result on every float, the +-k pi/2 cases included
    // (tools/check_trigf.c), so a tier-C wave needs no per-row choice
    y = srm_jred_cw(xd, fn);
  } else {
    y = srm_jred_near(xd, fn);
    if constexpr (CW) y = __builtin_fabsf(x) <= SRM_J9PIO4F ? y : srm_jred_cw(xd, fn);
  }
  return y;
}
template <int KIND, bool CW>
__device__ __attribute__((always_inline)) inline float jtrigf_row(float x) {
  double fn;
  const double y = jtrigf_red<KIND, CW>(x, fn);
  const float r = jtrigf_q_dev<KIND>(fn, y);
  return (KIND == 1 && x == 0.0f) ? x : r;  // sin(-0) = -0 (the reduction gives +0)
}
template <int R, int KIND, bool CW>
__device__ __attribute__((always_inline)) inline RV<float, R> jtrigf_bc_exact(RV<float, R> v) {
  UNR for (int r = 0; r < R; ++r) {
    v[r] = jtrigf_row<KIND, CW>(v[r]);
    if ((r + 1) % SRHIP_TRIG_ILP == 0) SRHIP_ROW_FENCE();
  }
  return v;
}
#if SRHIP_JTRIG_FAST
// Round 6: the kernels in Horner form with fmas (srm_jsin_fma / srm_jcos_fma, include/srhip_math.h),
// Julia's reduction unchanged.  A row whose fast Float64 value lies within SRM_JTIE_K ulps of a Float32
// rounding midpoint is flagged (srm_jtie: 3 VALU) and, when any lane of the wave flags it (a uniform
// branch, ~1e-7 of the inputs: tools/check_trigf.c counts 48-182 of ~2^31 floats per tier and kind),
// re-evaluated by Julia's own kernels from the same reduced argument; check_trigf proves every
// unflagged row equal to srm_jtrigf.  Tier B per row: 35 -> 27 VALU; tier A cos 13 -> 10.
// (Both polynomials pass through an empty asm so that the quadrant select stays a v_cndmask: as a
// C select of two expressions the compiler branched on it, executing both under exec masks.)
// v_fma_f64 with the addend in an SGPR pair (one scalar operand: the constant-bus limit): as a C fma the
// compiler chose v_fmac_f64 and copied every constant addend into VGPRs, two v_mov per fma
__device__ __attribute__((always_inline)) inline double fma_vvs(double a, double b, double c) {
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
}
// Horner forms of srm_jsin_fma / srm_jcos_fma (the same operations, so the same bits), the leading
// coefficients S4 / C3 held in VGPRs by the caller (once per body)
__device__ __attribute__((always_inline)) inline double jsin_fma_dev(double y, double z, double s4v) {
  const double p = fma_vvs(z, fma_vvs(z, fma_vvs(z, s4v, SRM_JS3), SRM_JS2), SRM_JS1);
  return __builtin_fma(z * y, p, y);
}
__device__ __attribute__((always_inline)) inline double jcos_fma_dev(double z, double c3v) {
  return __builtin_fma(z, fma_vvs(z, fma_vvs(z, fma_vvs(z, c3v, SRM_JC2), SRM_JC1), SRM_JC0), 1.0);
}
__device__ __attribute__((always_inline)) inline void jtrig_coef_vgprs(double& s4v, double& c3v) {
  s4v = SRM_JS4;
  c3v = SRM_JC3;
  asm volatile("" : "+v"(s4v), "+v"(c3v));
}
// (a & m) | (b & ~m) per 32-bit half: a where m = -1, b where m = 0
// srm_jtie on the device: the shift-add with its constant in an SGPR (the compiler moved the literal into
// a VGPR per row: a VOP3 instruction takes no literal here)
__device__ __attribute__((always_inline)) inline bool jtie_dev(double v) {
  uint32_t w;
  asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(w) : "v"((uint32_t)__builtin_bit_cast(uint64_t, v)),
      "s"(0x80000000u + 8u * SRM_JTIE_K));
  return w <= 16u * SRM_JTIE_K;
}
// (gfx950's v_bitop3_b32 with the select's truth table 0xE4 = m ? a : b per bit, through the builtin: as
// plain C the compiler split it into four operations, as inline asm it added s_nops around it)
__device__ __attribute__((always_inline)) inline double bfi_f64(int m, double a, double b) {
  const uint64_t ab = __builtin_bit_cast(uint64_t, a), bb = __builtin_bit_cast(uint64_t, b);
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)ab, (uint32_t)bb, (uint32_t)m, 0xE4);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(ab >> 32), (uint32_t)(bb >> 32), (uint32_t)m, 0xE4);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int KIND>
__device__ __attribute__((always_inline)) inline float jtrigf_a_row_fast(float x, double s4v, double c3v) {
  const double xd = (double)x, z = xd * xd;
  double p = KIND == 0 ? jcos_fma_dev(z, c3v) : jsin_fma_dev(xd, z, s4v);
  if (__builtin_amdgcn_ballot_w64(jtie_dev(p)) != 0) [[unlikely]]
    p = KIND == 0 ? srm_jcos_kernel(xd) : srm_jsin_kernel(xd);
  return KIND == 0 ? (float)p : __builtin_copysignf((float)p, x);
}
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> jtrigf_a(RV<float, R> v) {
  double s4v, c3v;
  jtrig_coef_vgprs(s4v, c3v);
  UNR for (int r = 0; r < R; ++r) {
    v[r] = jtrigf_a_row_fast<KIND>(v[r], s4v, c3v);
    if ((r + 1) % SRHIP_TRIG_ILP == 0) SRHIP_ROW_FENCE();
  }
  return v;
}
template <int KIND, bool CW>
__device__ __attribute__((always_inline)) inline float jtrigf_row_fast(float x, double s4v, double c3v) {
  double fn;
  const double y = jtrigf_red<KIND, CW>(x, fn);
  // n1 = n + 1 - KIND: its bit 0 selects the cos kernel (cos: n even; sin: n odd), its bit 1 is the sign
  // (cos: quadrants 1, 2; sin: 2, 3)
  const int n1 = cvt_i32_sat(fn) + 1 - KIND;
  const double z = y * y;
  const double ps = jsin_fma_dev(y, z, s4v), pc = jcos_fma_dev(z, c3v);
  const int msk = __builtin_amdgcn_sbfe(n1, 0, 1);  // -1 where the cos kernel applies: a bit select, no compare
  double p = bfi_f64(msk, pc, ps);
  if (__builtin_amdgcn_ballot_w64(jtie_dev(p)) != 0) [[unlikely]]
    p = bfi_f64(msk, srm_jcos_kernel(y), srm_jsin_kernel(y));
  // the sign added into bit 31 (the xor)
  uint32_t o;
  asm("v_lshl_add_u32 %0, %1, 31, %2" : "=v"(o) : "v"(n1 >> 1), "v"(__builtin_bit_cast(uint32_t, (float)p)));
  const float r = __builtin_bit_cast(float, o);
  return (KIND == 1 && x == 0.0f) ? x : r;  // sin(-0) = -0 (the reduction gives +0)
}
template <int R, int KIND, bool CW>
__device__ __attribute__((noinline)) RV<float, R> jtrigf_bc(RV<float, R> v) {
  double s4v, c3v;
  jtrig_coef_vgprs(s4v, c3v);
  UNR for (int r = 0; r < R; ++r) {
    v[r] = jtrigf_row_fast<KIND, CW>(v[r], s4v, c3v);
    if ((r + 1) % SRHIP_TRIG_ILP == 0) SRHIP_ROW_FENCE();
  }
  return v;
}
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> jtrigf_slow(RV<float, R> v) {
  double s4v, c3v;
  jtrig_coef_vgprs(s4v, c3v);
  UNR for (int r = 0; r < R; ++r) {
    const float x = v[r];
    v[r] = __builtin_fabsf(x) < SRM_PIO2F_BIG_F ? jtrigf_row_fast<KIND, true>(x, s4v, c3v) : srm_jtrigf(KIND, x);
  }
  return v;
}
#else
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> jtrigf_a(RV<float, R> v) {
  return jtrigf_a_exact<R, KIND>(v);
}
template <int R, int KIND, bool CW>
__device__ __attribute__((noinline)) RV<float, R> jtrigf_bc(RV<float, R> v) {
  return jtrigf_bc_exact<R, KIND, CW>(v);
}
template <int R, int KIND>
__device__ __attribute__((noinline)) RV<float, R> jtrigf_slow(RV<float, R> v) {
  UNR for (int r = 0; r < R; ++r) {
    const float x = v[r];
    v[r] = __builtin_fabsf(x) < SRM_PIO2F_BIG_F ? jtrigf_row<KIND, true>(x) : srm_jtrigf(KIND, x);
  }
  return v;
}
#endif
template <int R, int KIND>
__device__ __attribute__((always_inline)) inline RV<float, R> jtrigf_rows(const RV<float, R>& A) {
  RV<float, R> v;
  UNR for (int r = 0; r < R; ++r) v[r] = A[r];
  const float mx = abs_fold<R, true>(0.0f, A);  // NaN-propagating: a NaN row fails every test below
  if (__builtin_amdgcn_ballot_w64(!(mx < SRM_JPIO4F)) == 0) return jtrigf_a<R, KIND>(v);
  if (__builtin_amdgcn_ballot_w64(!(mx <= SRM_J9PIO4F)) == 0) return jtrigf_bc<R, KIND, false>(v);
  if (__builtin_amdgcn_ballot_w64(!(mx < SRM_PIO2F_BIG_F)) == 0) return jtrigf_bc<R, KIND, true>(v);
  return jtrigf_slow<R, KIND>(v);
}

template <int R, int KIND>
__device__ __attribute__((always_inline)) inline RV<float, R> trigf_rows(RV<float, R> v) {
  RV<float, R> res;
  if constexpr (KIND == 2) {
    bool big = false;
    UNR for (int r = 0; r < R; ++r) {
      const float x = v[r];
      const bool fin = __builtin_isfinite(x);
      const double xd = (double)x;
      const bool b = srm_pio2f_is_big(xd);  // also true for Inf / NaN
      big |= b && fin;
      double y;
      const int n = srm_rem_pio2f_fast(b ? 0.0 : xd, &y);
      const float f = srm_trigf_finish(KIND, n, y);
      res[r] = fin ? f : x - x;
      if ((r + 1) % SRHIP_HEAVY_ILP == 0) SRHIP_ROW_FENCE();
    }
    if (big) res = trigf_fix_tan<R>(v, res);
  } else if constexpr (SRHIP_JULIA_TRIG) {
    res = jtrigf_rows<R, KIND>(v);
  } else {
    static_assert(R % 2 == 0, "row pairs");
    const float mx = abs_fold<R, true>(0.0f, v);
    UNR for (int r = 0; r < R; ++r) {
      res[r] = sincosf_dev<KIND>((double)v[r]);
      if ((r + 1) % SRHIP_HEAVY_ILP == 0) SRHIP_ROW_FENCE();
    }
    if (!(mx < SRM_PIO2F_BIG_F)) res = trigf_fix<R, KIND>(v, res);
  }
  return res;
}

template <typename T, int R, int U>
__device__ __attribute__((noinline)) RV<T, R> heavy_un(RV<T, R> v) {
  using O = OpsT<T>;
  if constexpr (SRHIP_TRIG_ROWS && std::is_same<T, float>::value && (U == UN_COS || U == UN_SIN || U == UN_TAN))
    return trigf_rows<R, U == UN_COS ? 0 : (U == UN_SIN ? 1 : 2)>(v);
  if constexpr (std::is_same<T, float>::value && U == UN_EXP && R % 2 == 0) {
    // one NaN-propagating max |x| per row pair decides for the whole wave (false for NaN)
    const float mx = abs_fold<R, true>(0.0f, v);
    if (__builtin_amdgcn_ballot_w64(!(mx <= EXPF_FAST_MAX)) == 0) {
      UNR for (int r = 0; r < R; r += 2) {
        const F2 e = expf2_fast((F2){v[r], v[r + 1]});
        v[r] = e.x;
        v[r + 1] = e.y;
      }
    } else {
      UNR for (int r = 0; r < R; r += 2) {
        const F2 e = expf2_dev((F2){v[r], v[r + 1]});
        v[r] = e.x;
        v[r + 1] = e.y;
      }
    }
    return v;
  }
  UNR for (int r = 0; r < R; ++r) {
    T x = v[r];
    switch (U) {
#define X_(NAME, FN) case UN_##NAME: if constexpr (un_ok<T>(UN_##NAME)) x = O::FN(x); break;
      SRHIP_UNOPS(X_)
#undef X_
      default: break;
    }
    v[r] = x;
    if ((r + 1) % SRHIP_HEAVY_ILP == 0) SRHIP_ROW_FENCE();  // rows in groups: bounds the callee's registers
  }
  return v;
}
// heavy binary: a op b per row
template <typename T, int R, int HB>
__device__ __attribute__((noinline)) RV<T, R> heavy_bin(RV<T, R> a, RV<T, R> b) {
  using O = OpsT<T>;
  UNR for (int r = 0; r < R; ++r) {
    T x = a[r];
    switch (HB) {
#define X_(NAME, FN) case HB_##NAME: if constexpr (hb_ok<T>(HB_##NAME)) x = O::FN(a[r], b[r]); break;
      SRHIP_HEAVY_BINOPS(X_)
#undef X_
      default: break;
    }
    a[r] = x;
    if ((r + 1) % SRHIP_HEAVY_ILP == 0) SRHIP_ROW_FENCE();
  }
  return a;
}
// "Wide" unary operators: OCML bodies with ~70-100 live VGPRs.  A kernel's register budget is the
// max over every callee it can reach, so only the K = K_MAX variant carries them; with them the
// common variants would drop from 5 to 4 waves per SIMD.  Programs whose operator table has one
// of them launch K_MAX (the host's variant choice).
constexpr bool un_wide(int u) { return un_wide_op(u); }

// unary operators cheap enough to inline into the handler (a few VALU instructions per row)
template <int U> constexpr bool un_inline() { return un_cheap(U); }
template <typename T, int R, int U>
__device__ __attribute__((always_inline)) inline void apply_un(RV<T, R>& A) {
  if constexpr (SRHIP_TRIG_ROWS && std::is_same<T, float>::value && (U == UN_COS || U == UN_SIN) && R % 2 == 0) {
    constexpr int KIND = U == UN_COS ? 0 : 1;
    RV<T, R> v;
    if constexpr (SRHIP_JULIA_TRIG) {
      v = jtrigf_rows<R, KIND>(A);
    } else {
      UNR for (int r = 0; r < R; ++r) v[r] = A[r];
      v = trigf_rows_fast<R>(A) ? trigf_fast<R, KIND>(v) : trigf_slow<R, KIND>(v);
    }
    UNR for (int r = 0; r < R; ++r) A[r] = v[r];
  } else if constexpr (un_inline<U>()) {
    using O = OpsT<T>;
    UNR for (int r = 0; r < R; ++r) {
      switch (U) {
#define X_(NAME, FN) case UN_##NAME: if constexpr (un_ok<T>(UN_##NAME)) A[r] = O::FN(A[r]); break;
        SRHIP_UNOPS(X_)
#undef X_
        default: break;
      }
    }
  } else {
    RV<T, R> v;
    UNR for (int r = 0; r < R; ++r) v[r] = A[r];
    v = heavy_un<T, R, U>(v);
    UNR for (int r = 0; r < R; ++r) A[r] = v[r];
  }
}
template <typename T, int R, int HB>
__device__ __attribute__((always_inline)) inline void apply_heavy(RV<T, R>& A, const RV<T, R>& X, const RV<T, R>& Y) {
  RV<T, R> a, b;
  UNR for (int r = 0; r < R; ++r) { a[r] = X[r]; b[r] = Y[r]; }
  a = heavy_bin<T, R, HB>(a, b);
  UNR for (int r = 0; r < R; ++r) A[r] = a[r];
}

// Check accumulator: max |v| over every operator output (NaN-propagating, v_maximum3_f32) for
// Float32; sum of |v| * 2^-512 for Float64 (Inf/NaN propagate, cannot overflow otherwise).
template <typename T> struct Chk {
  using type = T;
};
// Float32: one v_maximum3_f32 per two rows, chained through M (the compiler's reassociation into
// a pairwise tree costs R/2 + 2 instructions instead of R/2).
template <int R> __device__ __attribute__((always_inline)) inline void chk_update(float& M, const RV<float, R>& A) {
  M = abs_fold<R, true>(M, A);
}
template <int R> __device__ __attribute__((always_inline)) inline void chk_update(double& M, const RV<double, R>& A) {
  UNR for (int r = 0; r < R; ++r) M = __builtin_fma(__builtin_fabs(A[r]), 0x1p-512, M);
}
template <int R> __device__ __attribute__((always_inline)) inline void chk_update(int32_t&, const RV<int32_t, R>&) {}

// IEEE Float32 division of two rows: the compiler's own a / b expansion (v_div_scale of the
// denominator and of the numerator, v_rcp, Newton refinement, v_div_fmas with the numerator's scale
// flag, v_div_fixup for the special cases), with its five fma / mul steps on packed row pairs
// (v_pk_fma_f32, v_pk_mul_f32 round each lane exactly as the scalar instructions): the same bits as
// n / d, 8 instead of 11 VALU instructions per row.
__device__ __attribute__((always_inline)) inline F2 div2_dev(F2 n, F2 d) {
  bool unused0, unused1, f0, f1;
  const F2 ds = {__builtin_amdgcn_div_scalef(n.x, d.x, false, &unused0),
                 __builtin_amdgcn_div_scalef(n.y, d.y, false, &unused1)};
  F2 r = {__builtin_amdgcn_rcpf(ds.x), __builtin_amdgcn_rcpf(ds.y)};
  const F2 e = __builtin_elementwise_fma(-ds, r, (F2)(1.0f));
  r = __builtin_elementwise_fma(e, r, r);
  const F2 ns = {__builtin_amdgcn_div_scalef(n.x, d.x, true, &f0), __builtin_amdgcn_div_scalef(n.y, d.y, true, &f1)};
  F2 q = ns * r;
  const F2 e2 = __builtin_elementwise_fma(-ds, q, ns);
  q = __builtin_elementwise_fma(e2, r, q);
  const F2 e3 = __builtin_elementwise_fma(-ds, q, ns);
  F2 out;
  out.x = __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(e3.x, r.x, q.x, f0), d.x, n.x);
  out.y = __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(e3.y, r.y, q.y, f1), d.y, n.y);
  return out;
}

// The same division without its range machinery, for operands with |n|, |d| in [2^-40, 2^40]:
// there v_div_scale returns its operand unchanged with no scale flag (exponent difference < 96, no
// denormal divisor, reciprocal or quotient, numerator exponent > 23), so v_div_fmas is a plain fma,
// and v_div_fixup passes a finite normal quotient through -- the identical operation sequence on the
// same values, 4 instead of 8 VALU instructions per row.
__device__ __attribute__((always_inline)) inline F2 div2_inrange(F2 n, F2 d) {
  F2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const F2 e = __builtin_elementwise_fma(-d, r, (F2)(1.0f));
  r = __builtin_elementwise_fma(e, r, r);
  F2 q = n * r;
  const F2 e2 = __builtin_elementwise_fma(-d, q, n);
  q = __builtin_elementwise_fma(e2, r, q);
  const F2 e3 = __builtin_elementwise_fma(-d, q, n);
  return __builtin_elementwise_fma(e3, r, q);
}
constexpr float DIV_FAST_LO = 0x1p-40f, DIV_FAST_HI = 0x1p40f;

// A = A / B (SWAP: B / A) over a lane's rows: the whole wave takes div2_inrange when every operand
// of every lane is in its range (one NaN-propagating v_maximum3 and v_minimum3 of |a|, |b| per row,
// a ballot), else the full div2_dev.  C2's population: ~5 % of (division node, tile) pairs fall back.
// M (CHK): the check statistic is folded on the full path only -- an in-range quotient is finite
// with |q| <= 2^80, so its column sum cannot overflow (rows < 2^46) and the host decision (which
// bounds every folded output's sum by max|v| x rows) is unchanged.
// CONSTB: B is one wave-uniform constant, so only A's rows need the range test.
template <int R, bool SWAP, bool CHK, bool CONSTB = false>
__device__ __attribute__((always_inline)) inline void div_rows(RV<float, R>& A, const RV<float, R>& B, float& M) {
  float mx = 0.0f, mn = __builtin_inff();
  if constexpr (CONSTB) {
    mx = abs_fold<R, true>(mx, A);
    mn = abs_fold<R, false>(mn, A);
    const float c = __builtin_fabsf(B[0]);
    mx = __builtin_elementwise_maximum(mx, c);
    mn = __builtin_elementwise_minimum(mn, c);
  } else {
    mx = abs_fold<R, true>(abs_fold<R, true>(mx, A), B);
    mn = abs_fold<R, false>(abs_fold<R, false>(mn, A), B);
  }
  const bool fast = mx <= DIV_FAST_HI && mn >= DIV_FAST_LO;  // false for NaN
  if (__builtin_amdgcn_ballot_w64(!fast) == 0) {
    UNR for (int r = 0; r < R; r += 2) {
      const F2 a = {A[r], A[r + 1]}, b = {B[r], B[r + 1]};
      const F2 c = SWAP ? div2_inrange(b, a) : div2_inrange(a, b);
      A[r] = c.x;
      A[r + 1] = c.y;
    }
  } else {
    UNR for (int r = 0; r < R; r += 2) {
      const F2 a = {A[r], A[r + 1]}, b = {B[r], B[r + 1]};
      const F2 c = SWAP ? div2_dev(b, a) : div2_dev(a, b);
      A[r] = c.x;
      A[r + 1] = c.y;
    }
    if constexpr (CHK) chk_update<R>(M, A);
  }
}

// Specialised binary operator over a lane's rows: A = A op B (SWAP: A = B op A).  Float32 + - * /
// run on packed row pairs (v_pk_add_f32 / v_pk_mul_f32, div_rows: each lane rounded exactly as
// the scalar instruction would); the rest row by row.
typedef F2 PkF32;
// a - b on a row pair as v_pk_add_f32 with the second operand negated (the same IEEE result,
// signed zeros included); the compiler otherwise splits a <2 x float> subtraction into two v_sub_f32
__device__ __attribute__((always_inline)) inline F2 pk_sub(F2 a, F2 b) {
  F2 c;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(c) : "v"(a), "v"(b));
  return c;
}
#ifndef SRHIP_PK_BINOPS
#define SRHIP_PK_BINOPS 1
#endif
template <typename T, int SB> __device__ __attribute__((always_inline)) inline T sb_apply(T a, T b) {
  using O = OpsT<T>;
  switch (SB) {
#define X_(NAME, FN) case SB_##NAME: if constexpr (sb_ok<T>(SB_##NAME)) return O::FN(a, b); break;
    SRHIP_SPEC_BINOPS(X_)
#undef X_
    default: break;
  }
  return a;
}
template <typename T, int R, int SB, bool SWAP>
__device__ __attribute__((always_inline)) inline void bin_rows(RV<T, R>& A, const RV<T, R>& B) {
  if constexpr (std::is_same<T, float>::value && R % 2 == 0 && SB == SB_DIV) {
    float unused = 0.0f;
    div_rows<R, SWAP, false>(A, B, unused);
  } else if constexpr (SRHIP_PK_BINOPS && std::is_same<T, float>::value && R % 2 == 0 &&
                       (SB == SB_ADD || SB == SB_SUB || SB == SB_MUL)) {
    UNR for (int r = 0; r < R; r += 2) {
      const PkF32 a = {A[r], A[r + 1]}, b = {B[r], B[r + 1]};
      PkF32 c;
      if constexpr (SB == SB_ADD) c = SWAP ? b + a : a + b;
      else if constexpr (SB == SB_SUB) c = SWAP ? pk_sub(b, a) : pk_sub(a, b);
      else c = SWAP ? b * a : a * b;
      A[r] = c.x;
      A[r + 1] = c.y;
    }
  } else {
    UNR for (int r = 0; r < R; ++r) A[r] = SWAP ? sb_apply<T, SB>(B[r], A[r]) : sb_apply<T, SB>(A[r], B[r]);
  }
}
template <typename T, int R, int SB, bool SWAP>
__device__ __attribute__((always_inline)) inline void bin_rows_c(RV<T, R>& A, T c) {
  RV<T, R> B;
  UNR for (int r = 0; r < R; ++r) B[r] = c;
  bin_rows<T, R, SB, SWAP>(A, B);
}
// the interpreter's operator forms: the operation and the check fold of its output
template <typename T, int R, int SB, bool SWAP, bool CONSTB = false>
__device__ __attribute__((always_inline)) inline void bin_rows_chk(RV<T, R>& A, const RV<T, R>& B, typename Chk<T>::type& M) {
  if constexpr (std::is_same<T, float>::value && R % 2 == 0 && SB == SB_DIV) {
    div_rows<R, SWAP, true, CONSTB>(A, B, M);
  } else {
    bin_rows<T, R, SB, SWAP>(A, B);
    // Float32 + and -, and * by a constant, fold nothing (round 6): the reduction raises each tree's
    // statistic to the tree's bound on their outputs instead (UndecidedList::sbound, skip_bound_apply)
    if constexpr (!(std::is_same<T, float>::value && (SB == SB_ADD || SB == SB_SUB || (SB == SB_MUL && CONSTB))))
      chk_update<R>(M, A);
  }
}
template <typename T, int R, int SB, bool SWAP>
__device__ __attribute__((always_inline)) inline void bin_rows_c_chk(RV<T, R>& A, T c, typename Chk<T>::type& M) {
  RV<T, R> B;
  UNR for (int r = 0; r < R; ++r) B[r] = c;
  bin_rows_chk<T, R, SB, SWAP, true>(A, B, M);
}

template <typename T> using LAccT = typename std::conditional<kIsInt<T>, long long, double>::type;


// Wave reductions on DPP lane moves (no LDS round trip per step): quad butterflies, half-row and
// row mirrors, then row_bcast15 / row_bcast31 fold the four rows into lane WAVE_LAST.  Only that
// lane's result is meaningful; the order is fixed, so results are deterministic.
constexpr int WAVE_LAST = 63;
// (v_mov_b32_dpp with an undefined old value: lanes of rows outside ROWS keep whatever the
// destination held, which only feeds lanes whose results are never read -- lane WAVE_LAST's chain
// reads row 3's own lanes, lane 47 before the bcast15 step and lane 31 after it; a zero old value
// cost a v_mov per 32-bit half per step)
template <int CTRL, int ROWS = 0xf>
__device__ __attribute__((always_inline)) inline uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf, typename U>
__device__ __attribute__((always_inline)) inline U dpp(U v) {
  if constexpr (sizeof(U) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = (uint64_t)dpp32<CTRL, ROWS>((uint32_t)b) | ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(b >> 32)) << 32);
    return __builtin_bit_cast(U, r);
  } else {
    return __builtin_bit_cast(U, dpp32<CTRL, ROWS>(__builtin_bit_cast(uint32_t, v)));
  }
}
template <typename U, typename F>
__device__ __attribute__((always_inline)) inline U wave_fold(U v, F op) {
  v = op(v, dpp<0xB1>(v));       // quad_perm [1,0,3,2]
  v = op(v, dpp<0x4E>(v));       // quad_perm [2,3,0,1]
  v = op(v, dpp<0x141>(v));      // row_half_mirror
  v = op(v, dpp<0x140>(v));      // row_mirror: every lane of a row holds the row's fold
  v = op(v, dpp<0x142, 0xa>(v)); // row_bcast15 -> rows 1, 3
  v = op(v, dpp<0x143, 0xc>(v)); // row_bcast31 -> rows 2, 3: lane 63 holds the wave's fold
  return v;
}
__device__ __attribute__((always_inline)) inline double wave_sum(double v) {
  return wave_fold(v, [](double a, double b) { return a + b; });
}
__device__ __attribute__((always_inline)) inline double wave_sum_d(double v) { return wave_sum(v); }
__device__ __attribute__((always_inline)) inline long long wave_sum(long long v) {
  return wave_fold(v, [](long long a, long long b) { return a + b; });
}
__device__ __attribute__((always_inline)) inline float wave_chk(float v) {
  return wave_fold(v, [](float a, float b) { return __builtin_elementwise_maximum(a, b); });
}
__device__ __attribute__((always_inline)) inline double wave_chk(double v) { return wave_sum(v); }
__device__ __attribute__((always_inline)) inline int32_t wave_chk(int32_t v) { return v; }

// MODE_PRECISE: exact per-(tree, operator node, row block) sums, used only for the rare trees
// whose fast max|v| bound cannot decide DynamicExpressions' isfinite(sum(array)) checks.
// One wave owns a (tree, row block), so plain read-modify-write of its slab entry is race-free.
template <typename T, int R>
// ord: the operator's ordinal (1-based) in the tree's program, counted by the interpreter in execution
// order -- the order the host numbered them (push_op), so a gradient program's leaf-constant
// superinstructions can carry their constant's index in the instruction's upper half instead
__device__ __attribute__((always_inline)) inline void precise_hook(const EvalArgs& p, uint32_t ord, const RV<T, R>& A,
                                                                   int slot, int rb, int lane, int64_t row0) {
  if constexpr (!kIsInt<T>) {
    const uint32_t opidx = ord;
    if (opidx == 0) return;
    constexpr int VEC = 16 / sizeof(T);
    double s = 0.0;
    UNR for (int r = 0; r < R; ++r) {
      const int64_t row = row0 + (r / VEC) * 64 * VEC + lane * VEC + (r % VEC);
      const double v = sizeof(T) == 8 ? (double)A[r] * 0x1p-64 : (double)A[r];
      s += row < p.nvalid ? v : 0.0;
    }
    s = wave_sum_d(s);
    if (lane == WAVE_LAST) {
      // the launch's order slot (a listed tree's index in the device list), not its index inside the
      // workgroup's group: a device-listed launch runs one tree per group
      double* e = reinterpret_cast<double*>(p.slab_prec) + ((int64_t)slot * p.prec_stride + (opidx - 1)) * p.nrb + rb;
      if (p.prec_assign) *e = s;  // the block's only tile: no read-modify-write round trip per operator
      else *e += s;
    }
  }
}

// The other distance losses, out of line: their bodies call math routines, and inline they made
// the allocator move the accumulator off the registers the operator bodies use for it.
template <typename T, int R>
__device__ __attribute__((noinline)) RV<T, R> loss_rows_generic(RV<T, R> a, RV<T, R> y, int kind, T p0) {
  UNR for (int r = 0; r < R; ++r) a[r] = loss_row<T>(kind, a[r], y[r], p0);
  return a;
}

// Per-tile loss epilogue for a given loss kind (KIND < 0: runtime kind).
template <typename T, int R>
__device__ __attribute__((always_inline)) inline void loss_tile(const EvalArgs& p, RV<T, R>& A, const T* ybase,
                                                                const T* wbase, int lane, int64_t row0, bool full,
                                                                LAccT<T>* lacc) {
  // lacc[CPT]: this lane's sum per loss chunk of the tile (a tile longer than a chunk, R = 32, covers
  // two: register r of a lane belongs to chunk r / (R / CPT))
  constexpr int CHK = sizeof(T) == 8 ? LOSS_CHUNK_8B : LOSS_CHUNK_4B;
  constexpr int CPT = 64 * R > CHK ? 64 * R / CHK : 1, RPC = R / CPT;
  // full: every row of the tile is valid (wave-uniform)
  RV<T, R> yv;
  load_rows<T, R>(ybase, lane, yv);
  constexpr int VEC = 16 / sizeof(T);
  if constexpr (kIsInt<T>) {
    UNR for (int r = 0; r < R; ++r) {
      int32_t l = loss_elem_int(p.loss_kind, IOps::sub(A[r], yv[r]));
      long long c = (long long)l;
      if (!full) {
        const int64_t row = row0 + (r / VEC) * 64 * VEC + lane * VEC + (r % VEC);
        c = row < p.nvalid ? c : 0;
      }
      lacc[r / RPC] += c;
    }
  } else {
    RV<T, R> wv;
    if (p.weighted) load_rows<T, R>(wbase, lane, wv);
    const T p0 = (T)p.loss_p0;
    // (A is dead after the epilogue -- the next tile clears it -- so the residual overwrites it in place)
    RV<T, R>& lv = A;
    if (p.loss_kind == SRHIP_LOSS_L2) {
      bin_rows<T, R, SB_SUB, false>(lv, yv);
      RV<T, R> dv;
      UNR for (int r = 0; r < R; ++r) dv[r] = lv[r];
      bin_rows<T, R, SB_MUL, false>(lv, dv);
    } else if (p.loss_kind == SRHIP_LOSS_L1) {
      UNR for (int r = 0; r < R; ++r) lv[r] = m_abs(A[r] - yv[r]);
    } else {
      lv = loss_rows_generic<T, R>(A, yv, p.loss_kind, p0);  // (A first: it stays in v0-v15)
    }
    if (p.weighted) {
      // padded rows carry w = 0 and a replicated (finite when ok) prediction
      UNR for (int r = 0; r < R; ++r) lacc[r / RPC] += (double)(wv[r] * lv[r]);
    } else {
      if (!full) {
        UNR for (int r = 0; r < R; ++r) {
          const int64_t row = row0 + (r / VEC) * 64 * VEC + lane * VEC + (r % VEC);
          lv[r] = row < p.nvalid ? lv[r] : T(0);
        }
      }
      if constexpr (sizeof(T) == 4 && R % 4 == 0 && VEC == 4) {
        // Float32: a lane's 4 consecutive rows (one 16-byte group: the same rows in every launch
        // geometry) summed in Float32, (l0 + l2) + (l1 + l3) -- one packed add of the two register
        // pairs, one add -- then widened once: relative error <= 2^-23 for the non-negative
        // distance losses, against the 1e-6 parity bar; one bit pattern per tree and dataset
        UNR for (int r = 0; r < R; r += 4) {
          const F2 a = {lv[r], lv[r + 1]}, b = {lv[r + 2], lv[r + 3]};
          const F2 q = a + b;
          lacc[r / RPC] += (double)(q.x + q.y);
        }
      } else {
        UNR for (int r = 0; r < R; ++r) lacc[r / RPC] += (double)lv[r];
      }
    }
  }
}

template <typename T, int R>
__device__ __attribute__((always_inline)) inline void store_pred(const EvalArgs& p, const RV<T, R>& A, int tree, int lane,
                                                                 int64_t row0) {
  constexpr int VEC = 16 / sizeof(T);
  using V = typename Vec16<T>::type;
  T* out = reinterpret_cast<T*>(p.out_pred) + (int64_t)tree * p.nvalid;
  UNR for (int j = 0; j < R / VEC; ++j) {
    const int64_t row = row0 + j * 64 * VEC + lane * VEC;
    if (row + VEC <= p.nvalid && ((p.nvalid % VEC) == 0)) {
      V q;
      UNR for (int e = 0; e < VEC; ++e) q[e] = A[j * VEC + e];
      *reinterpret_cast<V*>(out + row) = q;
    } else {
      UNR for (int e = 0; e < VEC; ++e)
        if (row + e < p.nvalid) out[row + e] = A[j * VEC + e];
    }
  }
}

// Derived columns (srhip_isa.h): U(X[f]) for this workgroup's rows, computed once into LDS column
// nfeat + d by the same out-of-line operator bodies the interpreter calls (rows are independent
// and -ffp-contract=off, so the values are bit-identical to evaluating U inside a tree).  The
// column's check statistic over the block's rows (max |v| for Float32, sum |v| 2^-512 for
// Float64) lands in dchk[d]; a tree that reads the column folds it into its own statistic, exactly
// as its U instruction would have.
template <typename T, int R>
__device__ __attribute__((noinline)) RV<T, R> derive_un(int u, RV<T, R> v) {
  switch (u) {
#define X_(NAME, FN)                                                                     \
  case UN_##NAME:                                                                        \
    if constexpr (un_ok<T>(UN_##NAME) && un_derivable(UN_##NAME)) return heavy_un<T, R, UN_##NAME>(v); \
    break;
    SRHIP_UNOPS(X_)
#undef X_
    default: break;
  }
  return v;
}

// A thread takes one 16-byte vector (DV rows) of a column per call; each wave folds its column
// statistic with DPP and parks it in LDS, and one barrier after all columns lets the first nd
// threads fold the wave partials in wave order (fixed: deterministic).  (DV = 2 for Float32 kept all
// 512 threads busy but cost more VALU in call overhead; the kernel is VALU-issue bound.)
template <typename T>
__device__ __attribute__((always_inline)) inline void derive_columns(const EvalArgs& p, T* lx, int rbb,
                                                                     typename Chk<T>::type* dchk) {
  using CT = typename Chk<T>::type;
  constexpr int DV = 16 / sizeof(T);
  __shared__ CT part[EVAL_WAVES_MAX][DERIVE_MAX];
  const int tid = tid_x();
  const int lane = tid & 63, wave = tid >> 6;
  for (int d = 0; d < p.nd; ++d) {
    const uint32_t spec = __builtin_amdgcn_readfirstlane(p.dspec[d]);
    const int u = (int)(spec >> 16), f = (int)(spec & 0xffff);
    const T* src = lx + (int64_t)f * rbb;
    T* dst = lx + (int64_t)(p.nfeat + d) * rbb;
    CT m = 0;
    for (int c = tid; c < rbb / DV; c += blockDim.x) {
      RV<T, DV> v = reinterpret_cast<const RV<T, DV>*>(src)[c];
      v = derive_un<T, DV>(u, v);
      reinterpret_cast<RV<T, DV>*>(dst)[c] = v;
      UNR for (int e = 0; e < DV; ++e) {
        if constexpr (sizeof(T) == 4) m = __builtin_elementwise_maximum(m, __builtin_fabsf(v[e]));
        else m = __builtin_fma(__builtin_fabs(v[e]), 0x1p-512, m);
      }
    }
    m = wave_chk(m);
    if (lane == WAVE_LAST) part[wave][d] = m;
  }
  __syncthreads();
  const int tf = tid_x();
  if (tf < p.nd) {
    const int d = tf;
    CT t = part[0][d];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      if constexpr (sizeof(T) == 4) t = __builtin_elementwise_maximum(t, part[w][d]);
      else t += part[w][d];
    }
    dchk[d] = t;
  }
  __syncthreads();
}

// Derived columns for one row block, a wave per (column, tile): the wave runs the interpreter's own
// R-row operator body over one tile of the source feature (the same call the U instruction makes,
// so the values are the same bits), stores it into the column and parks the tile's check statistic
// in LDS; after one barrier the first nd threads fold each column's tiles in tile order.
template <typename T, int R>
__device__ __attribute__((always_inline)) inline void derive_columns_tiles(const EvalArgs& p, T* lx, int rbb,
                                                                           typename Chk<T>::type* dchk) {
  using CT = typename Chk<T>::type;
  constexpr int TILE = 64 * R, VEC = 16 / sizeof(T);
  constexpr int MAX_TILES = ROW_ALIGN / TILE > 0 ? ROW_ALIGN / TILE : 1;
  __shared__ CT part[DERIVE_MAX][MAX_TILES];
  const int tid = tid_x();
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), nwaves = blockDim.x >> 6;
  const int ntiles = rbb / TILE;
  for (int item = wave; item < p.nd * ntiles; item += nwaves) {
    const int d = item / ntiles, j = item - d * ntiles;
    const uint32_t spec = __builtin_amdgcn_readfirstlane(p.dspec[d]);
    const int u = (int)(spec >> 16), f = (int)(spec & 0xffff);
    RV<T, R> v;
    load_rows<T, R>(lx + (int64_t)f * rbb + (int64_t)j * TILE, lane, v);
    RV<T, R> rv;
    UNR for (int r = 0; r < R; ++r) rv[r] = v[r];
    rv = derive_un<T, R>(u, rv);
    CT m = 0;
    using V = typename Vec16<T>::type;
    T* dst = lx + (int64_t)(p.nfeat + d) * rbb + (int64_t)j * TILE;
    UNR for (int q = 0; q < R / VEC; ++q) {
      V o;
      UNR for (int e = 0; e < VEC; ++e) {
        o[e] = rv[q * VEC + e];
        if constexpr (sizeof(T) == 4) m = __builtin_elementwise_maximum(m, __builtin_fabsf(o[e]));
        else m = __builtin_fma(__builtin_fabs(o[e]), 0x1p-512, m);
      }
      reinterpret_cast<V*>(dst)[q * 64 + lane] = o;
    }
    m = wave_chk(m);
    if (lane == WAVE_LAST) part[d][j] = m;
  }
  __syncthreads();
  const int tf = tid_x();
  if (tf < p.nd) {
    const int d = tf;
    CT t = part[d][0];
    for (int j = 1; j < ntiles; ++j) {
      if constexpr (sizeof(T) == 4) t = __builtin_elementwise_maximum(t, part[d][j]);
      else t += part[d][j];
    }
    dchk[d] = t;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// The interpreter kernel.
//   grid.x = row blocks (RB rows each), grid.y = tree groups; block = WAVES wavefronts.
//   MODE_LOSS: fused loss partial + check partial per (tree, row block) -> slabs
//   MODE_PRED: prediction rows -> out_pred[tree][row], check partial -> slab
// ------------------------------------------------------------------------------------------------
// One (row block, tree group) of the launch: stage the block, derive its columns, interpret the
// group's trees over it.  rb = row block, gy = tree group (grid.y; 0 in persistent launches, whose
// one group is the whole population).  gstride > 1 (a persistent launch's tail items): the group is
// the order slots gslice, gslice + gstride, ... -- an interleaved 1/gstride of the population, so
// the slices of a block cost about the same.
template <typename T, int R, int K, int MODE, bool XLDS>
__device__ __attribute__((always_inline)) inline void eval_block(const EvalArgs& p, unsigned char* smem, const int rb,
                                                                 const int gy, const int gslice = 0,
                                                                 const int gstride = 1) {
  constexpr int WAVES = eval_waves(R, K);
  using O = OpsT<T>;
  using CT = typename Chk<T>::type;
  constexpr int TILE = 64 * R;
  const int lane = tid_x() & 63;  // (opaque: rematerialised instead of spilled across the block loop)
  const int64_t row_base = (int64_t)rb * p.rb_rows;
  const int ntiles = p.rb_rows / TILE;
  // valid rows of this block, block-relative (<= rb_rows): the tile loop's uniform row tests are
  // 32-bit scalar compares (a 64-bit ordering compare has no scalar form and made them VALU
  // compares, i.e. a divergent loop)
  const int nrel = __builtin_amdgcn_readfirstlane((int)min<int64_t>(max<int64_t>(p.nvalid - row_base, 0), (int64_t)p.rb_rows));

  // ---- stage this block's rows of X (and y, w) into LDS ----
  const T* xsrc;
  const T* ysrc;
  const T* wsrc;
  int64_t xstride;
  if constexpr (XLDS) {
    T* lx = reinterpret_cast<T*>(smem);
    const int rbb = p.rb_rows;
    const int ncols = p.nfeat + (p.has_y ? 1 : 0) + (p.weighted ? 1 : 0);
    using V = typename Vec16<T>::type;
    constexpr int VEC = 16 / sizeof(T);
    const int vec_per_col = rbb / VEC;
    const T* gX = reinterpret_cast<const T*>(p.X);
    const T* gy = reinterpret_cast<const T*>(p.y);
    const T* gw = reinterpret_cast<const T*>(p.w);
    for (int i = tid_x(); i < ncols * vec_per_col; i += blockDim.x) {
      const int c = i / vec_per_col;
      const int v = i - c * vec_per_col;
      const T* src = c < p.nfeat ? gX + (int64_t)c * p.ld : (c == p.nfeat ? gy : gw);
      const int lc = c < p.nfeat ? c : c + p.nd;  // LDS column: derived columns follow the features
      reinterpret_cast<V*>(lx + (int64_t)lc * rbb)[v] = reinterpret_cast<const V*>(src + row_base)[v];
    }
    xsrc = lx;
    ysrc = lx + (int64_t)(p.nfeat + p.nd) * rbb;
    wsrc = lx + (int64_t)(p.nfeat + p.nd + 1) * rbb;
    xstride = rbb;
  } else {
    xsrc = reinterpret_cast<const T*>(p.X) + row_base;
    ysrc = reinterpret_cast<const T*>(p.y) + row_base;
    wsrc = reinterpret_cast<const T*>(p.w) + row_base;
    xstride = p.ld;
  }
  KDBG("[k] staged, ntiles=%d rb_rows=%d nvalid=%ld max_steps=%d\n", ntiles, p.rb_rows, (long)p.nvalid, p.max_steps);
  __shared__ int next_tree;  // the group's next unclaimed tree (waves claim trees dynamically)
  if (threadIdx.x == 0) next_tree = blockDim.x >> 6;  // the waves present (a launch may run fewer than WAVES)
  // failed-tree marks of the group's first FLAG_SNAP trees as this workgroup starts (one coherent
  // load per thread, in parallel, instead of a memory round trip per wave and tree): workgroups that
  // start after another row block saw a tree fail skip it.  A stale snapshot only skips less.
  constexpr int FLAG_SNAP = 2048;
  constexpr bool SNAP = MODE == MODE_LOSS && !kIsInt<T>;
  __shared__ uint8_t failed_snap[SNAP ? FLAG_SNAP : 1];
  const int gb0 = p.group_off ? p.group_off[gy] : gy * p.trees_per_group;
  const int snap_base = gb0 + gslice;
  const int snap_n = gstride > 1 ? (p.ntrees - gslice + gstride - 1) / gstride
                                 : (p.group_off ? p.group_off[gy + 1] - gb0 : min(p.trees_per_group, p.ntrees - gb0));
  if constexpr (SNAP) {
    if (p.early_exit)
      for (int i = tid_x(); i < min(snap_n, FLAG_SNAP); i += blockDim.x)
        failed_snap[i] = __hip_atomic_load(p.fail_flag + snap_base + i * gstride, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) == p.epoch;
  }
  __syncthreads();
  constexpr bool DERIVED = XLDS && !kIsInt<T> && MODE != MODE_PRECISE;
  __shared__ CT dchk[DERIVED ? DERIVE_MAX : 1];
  if constexpr (DERIVED) {
    if (p.nd > 0) {
      if (p.persistent) derive_columns_tiles<T, R>(p, reinterpret_cast<T*>(smem), p.rb_rows, dchk);
      else derive_columns<T>(p, reinterpret_cast<T*>(smem), p.rb_rows, dchk);
    }
  }
  KMARK(0, 2);
  if (p.debug_stop == 2) return;  // (diagnostic runs are never persistent)

  // tree group of this workgroup: uniform, or the host's tail-shaped sizes (group_off)
  const int group_base = __builtin_amdgcn_readfirstlane(snap_base);
  int group_n = __builtin_amdgcn_readfirstlane(snap_n);
  if constexpr (MODE == MODE_PRECISE) {
    // device-listed trees: this group's slots (group_base, + gstride, ...) that the list filled
    if (p.dev_count) {
      const int cnt = __builtin_amdgcn_readfirstlane(*p.dev_count);
      group_n = max(0, min(group_n, (cnt - group_base + gstride - 1) / gstride));
    }
  }

  // the group's trees are in descending estimated cost (host make_order): wave w starts with tree w,
  // then each wave claims the next unclaimed tree from an LDS counter as it finishes one — longest
  // first, so the waves of a workgroup end within about one cheap tree of each other (a static
  // round-robin left up to the cost spread idle at every workgroup's end).  The counter only grows:
  // every wave leaves the loop once it passes group_n.
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const CIns* code = (const CIns*)(uintptr_t)p.code;
  KMARK(8 + wave, 10);
  // tile claims (the probe launch, R = 16: one tile = one loss chunk): a wave claims one (tree, tile)
  // at a time, so the two tiles of a row block's costliest tree run on two waves at once; the check
  // statistic and the row count then combine by atomics (max of non-negative float bits; NaN bits
  // order above every finite and infinite value), each loss chunk is still written by one wave
  const bool tile_claims = p.tile_claims != 0 && TILE == (sizeof(T) == 8 ? LOSS_CHUNK_8B : LOSS_CHUNK_4B);
  const int nclaims = tile_claims ? group_n * ntiles : group_n;
  for (int cl = wave; cl < nclaims;) {
    const int ti = tile_claims ? cl / ntiles : cl;
    const int tile0 = tile_claims ? cl - ti * ntiles : 0, tile_end = tile_claims ? tile0 + 1 : ntiles;
    KMARK(8 + wave, 11);
    const int slot = group_base + ti * gstride;  // order slot (uniform)
    const int tree = __builtin_amdgcn_readfirstlane(p.order[slot]);
    const int pc0 = __builtin_amdgcn_readfirstlane(p.prog_off[tree]);
    const int max_steps = __builtin_amdgcn_readfirstlane(p.max_steps);
    KDBG("[k] ti=%d tree=%d pc0=%d group_n=%d\n", ti, tree, pc0, group_n);
    KMARK(0, 3);
    KMARK(1, tree);
    if (p.debug_stop == 3) break;  // (diagnostic) skip the trees; a continue would not claim the next one

    if constexpr (MODE == MODE_PRECISE) {
      // device-listed trees: this wave owns the (tree, row block) entries, zeroed before accumulating
      if (p.dev_count && lane == WAVE_LAST)
        for (int k = 0; k < p.prec_stride; ++k)
          reinterpret_cast<double*>(p.slab_prec)[((int64_t)slot * p.prec_stride + k) * p.nrb + rb] = 0.0;
    }
    // loss chunks per tile (CPT > 1: R = 32 tiles span two chunks) / tiles per loss chunk
    constexpr int CHS = sizeof(T) == 8 ? LOSS_CHUNK_8B : LOSS_CHUNK_4B;
    constexpr int CPT = TILE > CHS ? TILE / CHS : 1, TPC = TILE > CHS ? 1 : CHS / TILE;
    static_assert(TILE > CHS ? TILE % CHS == 0 : CHS % TILE == 0, "tiles and loss chunks nest");
    LAccT<T> lacc[CPT];
    UNR for (int c = 0; c < CPT; ++c) lacc[c] = 0;
    CT M = 0;
    // another row block already saw this tree fail in this launch: nothing here can change its
    // result (did_succeed = false, loss L(Inf)); NaN partials and check statistic stand in
    bool failed = false;
    if constexpr (SNAP) {
      if (p.early_exit && ti < FLAG_SNAP) failed = __builtin_amdgcn_readfirstlane(failed_snap[ti]) != 0;
    }
    if constexpr (DERIVED) {
      if (p.nd > 0) {  // check statistics of the derived columns this tree reads
        uint64_t msk = p.dmask[tree];
        msk = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(msk >> 32)) << 32) |
              (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)msk);
        while (msk) {
          const int d = __builtin_ctzll(msk);
          msk &= msk - 1;
          if constexpr (sizeof(T) == 4) M = __builtin_elementwise_maximum(M, dchk[d]);
          else if (lane == WAVE_LAST) M += dchk[d];  // a wave sum follows: count the column once
        }
      }
    }
    // loss slab layout [row block][order slot][chunk of the block] (p.cpb chunks per block): a
    // workgroup's partials are one contiguous range (its group's slots), so L2 lines fill before
    // write-back
    LAccT<T>* lslab = reinterpret_cast<LAccT<T>*>(p.slab_loss) +
                      ((int64_t)rb * p.ntrees + slot) * __builtin_amdgcn_readfirstlane(p.cpb);
    LAccT<T> csum = 0;  // fused launches: this lane's share of the tree's chunk sums
    int rows_done = 0;  // valid rows this wave evaluated the tree on (the launch's work count)
    if (failed) {
      if (lane == WAVE_LAST)
        for (int c = tile_claims ? tile0 : 0; c < (tile_claims ? tile_end : p.cpb); ++c) lslab[c] = (LAccT<T>)NAN;
      M = (CT)NAN;
      csum = (LAccT<T>)NAN;
    }
    for (int tile = tile0; tile < (failed ? tile0 : tile_end); ++tile) {
      const int64_t row0 = row_base + (int64_t)tile * TILE;
      const int trel = tile * TILE;
      if (trel >= nrel) break;  // whole tile is padding
      rows_done += min(TILE, nrel - trel);
      const T* xt = xsrc + (int64_t)tile * TILE;
      // (cleared per tile: with the registers left undefined or carried over, the allocator moved the
      // accumulator off v0-v15, where the out-of-line operator bodies take and return it)
      RV<T, R> A, S[K];
#if SRHIP_ASM_DEF
      // defined by an empty asm statement: a def the allocator sees at this point, no instruction
      // (every program writes A before reading it and pushes before it pops)
      asm volatile("" : "=v"(A));
      UNR for (int k = 0; k < K; ++k) asm volatile("" : "=v"(S[k]));
#else
      UNR for (int r = 0; r < R; ++r) A[r] = T(0);
      UNR for (int k = 0; k < K; ++k) UNR for (int r = 0; r < R; ++r) S[k][r] = T(0);
#endif
      // The program is read through the constant address space with a wave-uniform pc, so every
      // instruction is one s_load_dwordx4 (scalar cache), prefetched one instruction ahead.
      const CIns* prog = code + pc0;
      Ins nxt = prog[0];
      [[maybe_unused]] uint32_t pord = 0;  // MODE_PRECISE: operators executed so far (precise_hook)
      // bounded: a malformed program ends after max_steps instructions instead of hanging
      for (int step = 0; step < max_steps; ++step) {
        const Ins ins = nxt;
        nxt = prog[step + 1];
        KDBG("[k]   tile=%d step=%d h=%u a=%u\n", tile, step, ins.h, ins.a);
        if (ins.h == H_END) break;
        switch (ins.h) {
          SRHIP_LK case H_LOADF:
            load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, A);
            // (a gradient program's derived-column load carries its operator's ordinal)
            // (a gradient program's derived-column load is an operator: its ordinal field is non-zero)
            if constexpr (MODE == MODE_PRECISE)
              if ((ins.a >> 16) != 0) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);
            break;
          SRHIP_LK case H_LOADC: { const T c = imm_as<T>(ins.imm); UNR for (int r = 0; r < R; ++r) A[r] = c; break; }
#define SRHIP_K_CASES(BASE, ...)                                                            \
  case BASE + 0: if constexpr (0 < K) { constexpr int k = 0; __VA_ARGS__ } break;                 \
  case BASE + 1: if constexpr (1 < K) { constexpr int k = 1; __VA_ARGS__ } break;                 \
  case BASE + 2: if constexpr (2 < K) { constexpr int k = 2; __VA_ARGS__ } break;                 \
  case BASE + 3: if constexpr (3 < K) { constexpr int k = 3; __VA_ARGS__ } break;                 \
  case BASE + 4: if constexpr (4 < K) { constexpr int k = 4; __VA_ARGS__ } break;                 \
  case BASE + 5: if constexpr (5 < K) { constexpr int k = 5; __VA_ARGS__ } break;                 \
  case BASE + 6: if constexpr (6 < K) { constexpr int k = 6; __VA_ARGS__ } break;                 \
  case BASE + 7: if constexpr (7 < K) { constexpr int k = 7; __VA_ARGS__ } break;
#define SRHIP_K_CASES_H(HOT, BASE, ...)                                                     \
  HOT case BASE + 0: if constexpr (0 < K) { constexpr int k = 0; __VA_ARGS__ } break;             \
  HOT case BASE + 1: if constexpr (1 < K) { constexpr int k = 1; __VA_ARGS__ } break;             \
  case BASE + 2: if constexpr (2 < K) { constexpr int k = 2; __VA_ARGS__ } break;                 \
  case BASE + 3: if constexpr (3 < K) { constexpr int k = 3; __VA_ARGS__ } break;                 \
  case BASE + 4: if constexpr (4 < K) { constexpr int k = 4; __VA_ARGS__ } break;                 \
  case BASE + 5: if constexpr (5 < K) { constexpr int k = 5; __VA_ARGS__ } break;                 \
  case BASE + 6: if constexpr (6 < K) { constexpr int k = 6; __VA_ARGS__ } break;                 \
  case BASE + 7: if constexpr (7 < K) { constexpr int k = 7; __VA_ARGS__ } break;
          SRHIP_K_CASES_H(SRHIP_LK, H_PUSH0, { UNR for (int r = 0; r < R; ++r) S[k][r] = A[r]; })
          SRHIP_K_CASES_H(SRHIP_LK, H_PUSHLF0, {
            UNR for (int r = 0; r < R; ++r) S[k][r] = A[r];
            load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, A);
          })
          SRHIP_K_CASES_H(SRHIP_LK, H_PUSHLC0, {
            UNR for (int r = 0; r < R; ++r) S[k][r] = A[r];
            const T c = imm_as<T>(ins.imm);
            UNR for (int r = 0; r < R; ++r) A[r] = c;
          })
          SRHIP_K_CASES(H_SLOADF0, { load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, S[k]); })
          SRHIP_K_CASES(H_SLOADC0, { const T c = imm_as<T>(ins.imm); UNR for (int r = 0; r < R; ++r) S[k][r] = c; })

#define SRHIP_SPEC_CASE(NAME, FN)                                                                  \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_AF):                                                \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      RV<T, R> xv;                                                                                     \
      load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, xv);                                    \
      bin_rows_chk<T, R, SB_##NAME, false>(A, xv, M);                                              \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);         \
    }                                                                                              \
    break;                                                                                         \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_FA):                                                \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      RV<T, R> xv;                                                                                     \
      load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, xv);                                    \
      bin_rows_chk<T, R, SB_##NAME, true>(A, xv, M);                                               \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);         \
    }                                                                                              \
    break;                                                                                         \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_AC):                                                \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      bin_rows_c_chk<T, R, SB_##NAME, false>(A, imm_as<T>(ins.imm), M);                            \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);         \
    }                                                                                              \
    break;                                                                                         \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_CA):                                                \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      bin_rows_c_chk<T, R, SB_##NAME, true>(A, imm_as<T>(ins.imm), M);                             \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);         \
    }                                                                                              \
    break;                                                                                         \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_FF):                                              \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      RV<T, R> xv;                                                                                 \
      load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, A);                          \
      load_rows<T, R>(xt + (int64_t)(ins.imm & 0xffff) * xstride, lane, xv);                       \
      bin_rows_chk<T, R, SB_##NAME, false>(A, xv, M);                                              \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);     \
    }                                                                                              \
    break;                                                                                         \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_FC):                                              \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, A);                          \
      bin_rows_c_chk<T, R, SB_##NAME, false>(A, imm_as<T>(ins.imm), M);                            \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);     \
    }                                                                                              \
    break;                                                                                         \
  SRHIP_HOTB_##NAME case h_spec(SB_##NAME, SPEC_CF):                                              \
    if constexpr (sb_ok<T>(SB_##NAME)) {                                                           \
      load_rows<T, R>(xt + (int64_t)(ins.a & 0xffff) * xstride, lane, A);                          \
      bin_rows_c_chk<T, R, SB_##NAME, true>(A, imm_as<T>(ins.imm), M);                             \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);     \
    }                                                                                              \
    break;                                                                                         \
    SRHIP_K_CASES_H(SRHIP_HOTB_##NAME, h_spec(SB_##NAME, SPEC_SA0), if constexpr (sb_ok<T>(SB_##NAME)) {                \
      bin_rows_chk<T, R, SB_##NAME, true>(A, S[k], M);                                             \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);         \
    })                                                                                             \
    SRHIP_K_CASES_H(SRHIP_HOTB_##NAME, h_spec(SB_##NAME, SPEC_AS0), if constexpr (sb_ok<T>(SB_##NAME)) {                \
      bin_rows_chk<T, R, SB_##NAME, false>(A, S[k], M);                                            \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);         \
    })
          SRHIP_SPEC_BINOPS(SRHIP_SPEC_CASE)
#undef SRHIP_SPEC_CASE

#define SRHIP_HEAVY_CASE(NAME, FN)                                                              \
    SRHIP_K_CASES(h_heavy(HB_##NAME, HEAVY_SA0), if constexpr (hb_ok<T>(HB_##NAME)) {           \
      apply_heavy<T, R, HB_##NAME>(A, S[k], A);                                                 \
      chk_update<R>(M, A);                                                                      \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);  \
    })                                                                                          \
    SRHIP_K_CASES(h_heavy(HB_##NAME, HEAVY_AS0), if constexpr (hb_ok<T>(HB_##NAME)) {           \
      apply_heavy<T, R, HB_##NAME>(A, A, S[k]);                                                 \
      chk_update<R>(M, A);                                                                      \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0);  \
    })
          SRHIP_HEAVY_BINOPS(SRHIP_HEAVY_CASE)
#undef SRHIP_HEAVY_CASE

#define SRHIP_UN_CASE(NAME, FN)                                                  \
  SRHIP_HOTU_##NAME case h_un(UN_##NAME):                                        \
    if constexpr (un_ok<T>(UN_##NAME) && (K == K_MAX || !un_wide(UN_##NAME))) {  \
      apply_un<T, R, UN_##NAME>(A);                                              \
      if constexpr (UN_##NAME == UN_COS || UN_##NAME == UN_SIN) {                \
        if (!(ins.a & UN_NC_FLAG)) chk_update<R>(M, A);                          \
      } else {                                                                   \
        chk_update<R>(M, A);                                                     \
      }                                                                          \
      if constexpr (MODE == MODE_PRECISE) precise_hook<T, R>(p, ++pord, A, slot, rb, lane, row0); \
    }                                                                            \
    break;
          SRHIP_UNOPS(SRHIP_UN_CASE)
#undef SRHIP_UN_CASE
#undef SRHIP_K_CASES
          default: break;
        }
      }
      KDBG("[k]   tile %d done\n", tile);
      KMARK(0, 4);
      if constexpr (MODE == MODE_LOSS) {
        loss_tile<T, R>(p, A, ysrc + (int64_t)tile * TILE, wsrc + (int64_t)tile * TILE, lane, row0, trel + TILE <= nrel,
                        lacc);
        const bool flushed = (tile + 1) % TPC == 0 || trel + TILE >= nrel;
        const int ci0 = tile * CPT / TPC;  // the tile's (first) loss chunk
        if (flushed) {  // chunk(s) done (or last valid tile)
          UNR for (int c = 0; c < CPT; ++c) {
            const LAccT<T> s = wave_sum(lacc[c]);
            if (lane == WAVE_LAST) lslab[ci0 + c] = s;
            if (p.fused) {  // reduce_kernel's lane-strided accumulation: lane c % 64 adds chunk c
              const LAccT<T> sb = __shfl(s, WAVE_LAST);
              if (lane == (ci0 + c) % 64) csum += sb;
            }
            lacc[c] = 0;
          }
        }
        if constexpr (!kIsInt<T>) {
          // Early return (DynamicExpressions returns at the first bad array): a non-finite check
          // statistic in any lane means did_succeed = false for the whole tree (the host decision
          // fails every tree whose statistic is non-finite), so its remaining tiles in this row
          // block cannot change any result.  The unwritten loss chunks get NaN (never read: a failed
          // tree's loss is L(Inf)); M keeps the non-finite value the host sees.
          if (p.early_exit && __builtin_amdgcn_ballot_w64(!(M < (CT)INFINITY)) != 0) {
            csum = (LAccT<T>)NAN;
            if (lane == WAVE_LAST) {
              for (int c = ci0 + (flushed ? CPT : 0); c < (tile_claims ? tile_end : p.cpb); ++c)
                lslab[c] = (LAccT<T>)NAN;
              __hip_atomic_store(p.fail_flag + slot, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
          }
        }
      } else if constexpr (MODE == MODE_PRED) {
        store_pred<T, R>(p, A, tree, lane, row0);
      }
    }
    KDBG("[k] tree %d tiles done\n", tree);
    KMARK(0, 5);
    KMARK(8 + wave, 12);
    // ---- wave reduction, one partial per (tree, row block) ----
    if constexpr (!kIsInt<T> && MODE != MODE_PRECISE) {
      M = wave_chk(M);
      CT* chk_at = reinterpret_cast<CT*>(p.slab_chk) + (int64_t)rb * p.ntrees + slot;
      if (lane == WAVE_LAST) {
        if constexpr (sizeof(CT) == 4) {
          if (tile_claims) atomicMax(reinterpret_cast<unsigned*>(chk_at), __builtin_bit_cast(unsigned, __builtin_fabsf(M) == __builtin_fabsf(M) ? __builtin_fabsf(M) : M));
          else *chk_at = M;
        } else {
          *chk_at = M;
        }
      }
    }
    if (p.slab_rows && lane == WAVE_LAST) {
      if (tile_claims) atomicAdd(p.slab_rows + (int64_t)rb * p.ntrees + slot, rows_done);
      else p.slab_rows[(int64_t)rb * p.ntrees + slot] = rows_done;
    }
    if constexpr (MODE != MODE_PRECISE) {
      if (p.fused) {  // the only row block: reduce_kernel's steps for this tree, same order, same bits
        LAccT<T> s = csum;
        CT m = 0;
        if constexpr (!kIsInt<T>) {
          const CT mb = __shfl(M, WAVE_LAST);  // reduce_kernel's lane 0 reads row block 0
          if (lane == 0) {
            if constexpr (sizeof(T) == 4) m = __builtin_elementwise_maximum(m, mb);
            else m += mb;
          }
        }
        UNR for (int o = 32; o > 0; o >>= 1) {
          if (MODE == MODE_LOSS) s += __shfl_xor(s, o);
          if constexpr (!kIsInt<T>) {
            if constexpr (sizeof(T) == 4) m = __builtin_elementwise_maximum(m, __shfl_xor(m, o));
            else m += __shfl_xor(m, o);
          }
        }
        if (lane == 0) {
          if (MODE == MODE_LOSS && p.fused_loss) reinterpret_cast<LAccT<T>*>(p.fused_loss)[tree] = s;
          if (p.fused_chk) reinterpret_cast<CT*>(p.fused_chk)[tree] = m;
          if (p.fused_rows) p.fused_rows[tree] = rows_done;
        }
      }
    }
    KMARK(8 + wave, 13);
    int claim = 0;
    if (lane == 0) claim = atomicAdd(&next_tree, 1);
    cl = __builtin_amdgcn_readfirstlane(claim);
  }
  KMARK(8 + wave, 14);
}

// ------------------------------------------------------------------------------------------------
// The interpreter kernel.
//   grid.x = row blocks (RB rows each), grid.y = tree groups; block = WAVES wavefronts.
//   Persistent launches (p.persistent, one tree group): grid.x workgroups, each claims row blocks
//   block0, block0 + 1, ... from the counter p.block_ctr (zero at the launch) and interprets
//   the whole population over each, until the blocks run out -- every workgroup leaves the loop on
//   the same claimed index, so the grid always drains.
//   MODE_LOSS: fused loss partial + check partial per (tree, row block) -> slabs
//   MODE_PRED: prediction rows -> out_pred[tree][row], check partial -> slab
// ------------------------------------------------------------------------------------------------
template <typename T, int R, int K, int MODE, bool XLDS>
__global__ __launch_bounds__(64 * eval_waves(R, K)) void eval_kernel(EvalArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  KMARK(0, 1);
  if (p.debug_stop == 1) return;
  // items [0, nfull): whole row blocks block0 .. block0 + nfull - 1; then tail_slices items per
  // remaining row block, each an interleaved slice of the population (the last round of a launch
  // in finer pieces: the workgroups end within a slice of each other, not within a block).
  // Grid launches run their one (blockIdx.x, blockIdx.y) item.  One call site: the interpreter
  // body is inlined once.
  __shared__ int claimed;
  if constexpr (MODE == MODE_PRECISE) {
    // device-listed launches: group g takes the listed slots g, g + G, ...; with fewer listed trees
    // its workgroups leave at once (the launch is enqueued whether or not the list holds a tree)
    if (p.dev_count && p.grid_interleave && __builtin_amdgcn_readfirstlane(*p.dev_count) <= (int)blockIdx.y) return;
  }
  if (p.tile_claims && !p.persistent) {
    // the probe's combining entries start from zero (eval_block's first barrier orders these stores
    // before any wave's atomics); no memset launches before the probe.  Only this workgroup's waves
    // combine into its entries, and the later readers are later launches: a workgroup-scope release
    // suffices (an agent-scope fence is an L2 write-back on every workgroup: probe 39 -> 98 us)
    if (p.zero_ctr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
      __hip_atomic_store(p.zero_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int gs = p.grid_interleave ? (int)blockIdx.y : 0, gst = p.grid_interleave ? (int)gridDim.y : 1;
    const int nz = p.grid_interleave ? (p.ntrees - gs + gst - 1) / gst : 0;
    for (int i = threadIdx.x; i < nz; i += blockDim.x) {
      const int64_t at = (int64_t)blockIdx.x * p.ntrees + gs + (int64_t)i * gst;
      if (p.slab_chk) __hip_atomic_store(reinterpret_cast<uint32_t*>(p.slab_chk) + at, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p.slab_rows) __hip_atomic_store(p.slab_rows + at, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  }
  const int nfull = p.nrb - p.block0 - p.tail_blocks;
  const int nitems = nfull + p.tail_blocks * p.tail_slices;
  for (int it = 0;; ++it) {
    int rb, gy = 0, gslice = 0, gstride = 1;
    if (p.persistent) {
      if (threadIdx.x == 0) claimed = atomicAdd(p.block_ctr, 1);
      __syncthreads();
      const int item = __builtin_amdgcn_readfirstlane(claimed);
      if (item >= nitems) {
        // the items this workgroup evaluated, added to block_ctr[1]: the reduction compares the launch's
        // total with its item count (a counter left non-zero would have skipped items) and clears it
        if (threadIdx.x == 0 && it > 0) atomicAdd(p.block_ctr + 1, it);
        // every workgroup ends on one failing claim; the last of them (nitems + grid - 1) leaves the
        // counter at zero for the context's next persistent launch (no memset launch before it)
        if (threadIdx.x == 0 && item == nitems + (int)gridDim.x - 1)
          __hip_atomic_store(p.block_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      const int q = item - nfull;
      const bool whole = item < nfull;
      rb = p.block0 + (whole ? item : nfull + q / p.tail_slices);
      gslice = whole ? 0 : q % p.tail_slices;
      gstride = whole ? 1 : p.tail_slices;
    } else {
      rb = blockIdx.x + it * (int)gridDim.x;
      if (it > 0 && (!p.block_stride || rb >= p.nrb)) break;
      if (p.grid_interleave) {  // grid.y workgroups share the population interleaved (the probe)
        gslice = blockIdx.y;
        gstride = gridDim.y;
      } else {
        gy = blockIdx.y;
      }
    }
    eval_block<T, R, K, MODE, XLDS>(p, smem, rb, gy, gslice, gstride);
    if (!p.persistent && !p.block_stride) break;
    __syncthreads();  // every wave is done with this block's LDS (and has read `claimed`)
  }
}

// ---- launch helpers, instantiated by the per-variant translation units ----
template <typename T, int R, int K, int MODE, bool XLDS>
inline hipError_t launch_eval_t(const EvalArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  auto kern = eval_kernel<T, R, K, MODE, XLDS>;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const int waves = a.wg_waves > 0 ? std::min(a.wg_waves, eval_waves(R, K)) : eval_waves(R, K);
  hipLaunchKernelGGL(kern, grid, dim3(64 * waves), lds, s, a);
  return hipGetLastError();
}

template <typename T, int R, int MODE, bool XLDS>
inline hipError_t launch_eval_k(const EvalArgs& a, int K, dim3 grid, size_t lds, hipStream_t s) {
  if (K <= 2) return launch_eval_t<T, R, 2, MODE, XLDS>(a, grid, lds, s);
  if (K <= 4) return launch_eval_t<T, R, 4, MODE, XLDS>(a, grid, lds, s);
  return launch_eval_t<T, R, 8, MODE, XLDS>(a, grid, lds, s);
}

// one mode of one (T, R): the K variants, with and without LDS staging (MODE_PRECISE: K_MAX, global reads)
template <typename T, int R, int MODE>
inline hipError_t launch_eval_mode(const EvalArgs& a, int K, bool xlds, dim3 grid, size_t lds, hipStream_t s) {
  if constexpr (MODE == MODE_PRECISE) {
    (void)K;
    (void)xlds;
    return launch_eval_t<T, R, K_MAX, MODE_PRECISE, false>(a, grid, lds, s);
  } else {
    return xlds ? launch_eval_k<T, R, MODE, true>(a, K, grid, lds, s) : launch_eval_k<T, R, MODE, false>(a, K, grid, lds, s);
  }
}

}  // namespace srhip
