// srhip_ops.h — scalar operator and elementwise-loss semantics, host+device.
//
// Restated from the reference (src/Operators.jl) and the Julia Base functions it aliases
// (src/Options.jl:92-150 binopmap/unaopmap), including Julia's Bool "strong zero"
// (false * x == copysign(0, x)) used by relu/cond/greater/logical_* (src/Operators.jl:79-96).
// The same source is compiled for the device (OCML math) and for the host compiler's constant
// folding (libm), so folded constant subtrees follow the reference's scalar path
// (DynamicExpressions _eval_constant_tree) with the same formulas.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/srhip_math.h"

#define SRHIP_HD __host__ __device__ __attribute__((always_inline)) inline

namespace srhip {

// ---- small generic helpers -------------------------------------------------------------------
template <typename T> struct FP;
template <> struct FP<float> {
  static SRHIP_HD float nan() { return __builtin_nanf(""); }
  static SRHIP_HD float inf() { return __builtin_inff(); }
  // |x| at or above this rounds to Inf when summed exactly: 2^128 - 2^103
  static constexpr double OVF = 3.4028235677973366e38;
};
template <> struct FP<double> {
  static SRHIP_HD double nan() { return __builtin_nan(""); }
  static SRHIP_HD double inf() { return __builtin_inf(); }
  static constexpr double OVF = 1.7976931348623157e308;  // DBL_MAX (2^1024 - 2^970 is not representable)
};

SRHIP_HD float m_copysign(float a, float b) { return __builtin_copysignf(a, b); }
SRHIP_HD double m_copysign(double a, double b) { return __builtin_copysign(a, b); }
SRHIP_HD float m_abs(float a) { return __builtin_fabsf(a); }
SRHIP_HD double m_abs(double a) { return __builtin_fabs(a); }
SRHIP_HD bool m_isfinite(float a) { return __builtin_isfinite(a); }
SRHIP_HD bool m_isfinite(double a) { return __builtin_isfinite(a); }
SRHIP_HD bool m_isfinite(int32_t) { return true; }
SRHIP_HD bool m_isinf(float a) { return __builtin_isinf(a); }
SRHIP_HD bool m_isinf(double a) { return __builtin_isinf(a); }

// Julia max/min on floats: NaN-propagating, -0.0 < +0.0 (IEEE 754-2019 maximum/minimum).
SRHIP_HD float m_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }
SRHIP_HD double m_max(double a, double b) { return __builtin_elementwise_maximum(a, b); }
SRHIP_HD float m_min(float a, float b) { return __builtin_elementwise_minimum(a, b); }
SRHIP_HD double m_min(double a, double b) { return __builtin_elementwise_minimum(a, b); }

// ---- libm wrappers (float and double) ----------------------------------------------------------
// exp/log/sin/cos/tan come from the shared include/srhip_math.h (bit-identical on the device, in
// the host constant folder and in the oracle).  Every Float32 transcendental widens to Float64
// and rounds once (Julia's Float32 trig and ^ do the same), so the remaining vendor functions
// (OCML here, glibc in the oracle) agree on Float32 results except in double-rounding cases.
#define SRHIP_WRAP1(name, df)                                      \
  SRHIP_HD float m_##name(float x) { return (float)df((double)x); } \
  SRHIP_HD double m_##name(double x) { return df(x); }
SRHIP_HD float m_cos(float x) { return srm_cosf(x); }
SRHIP_HD double m_cos(double x) { return srm_cos(x); }
SRHIP_HD float m_sin(float x) { return srm_sinf(x); }
SRHIP_HD double m_sin(double x) { return srm_sin(x); }
SRHIP_HD float m_tan(float x) { return srm_tanf(x); }
SRHIP_HD double m_tan(double x) { return srm_tan(x); }
SRHIP_HD float m_exp(float x) { return srm_expf(x); }
SRHIP_HD double m_exp(double x) { return srm_exp(x); }
SRHIP_HD float m_log(float x) { return srm_logf(x); }
SRHIP_HD double m_log(double x) { return srm_log(x); }
SRHIP_WRAP1(log2, log2)
SRHIP_WRAP1(log10, log10)
SRHIP_WRAP1(log1p, log1p)
SRHIP_WRAP1(acosh, acosh)
SRHIP_WRAP1(atanh, atanh)
SRHIP_WRAP1(sinh, sinh)
SRHIP_WRAP1(cosh, cosh)
SRHIP_WRAP1(tanh, tanh)
SRHIP_WRAP1(asin, asin)
SRHIP_WRAP1(acos, acos)
SRHIP_WRAP1(atan, atan)
SRHIP_WRAP1(asinh, asinh)
SRHIP_WRAP1(erf, erf)
SRHIP_WRAP1(erfc, erfc)
SRHIP_WRAP1(tgamma, tgamma)
SRHIP_WRAP1(exp2, exp2)
SRHIP_WRAP1(expm1, expm1)
SRHIP_WRAP1(cbrt, cbrt)
#undef SRHIP_WRAP1
// exact in any IEEE implementation: no widening needed
SRHIP_HD float m_sqrt(float x) { return sqrtf(x); }
SRHIP_HD double m_sqrt(double x) { return sqrt(x); }
SRHIP_HD float m_rint(float x) { return rintf(x); }
SRHIP_HD double m_rint(double x) { return rint(x); }
SRHIP_HD float m_floor(float x) { return floorf(x); }
SRHIP_HD double m_floor(double x) { return floor(x); }
SRHIP_HD float m_ceil(float x) { return ceilf(x); }
SRHIP_HD double m_ceil(double x) { return ceil(x); }
SRHIP_HD float m_trunc(float x) { return truncf(x); }
SRHIP_HD double m_trunc(double x) { return trunc(x); }
SRHIP_HD float m_fmod(float a, float b) { return fmodf(a, b); }
SRHIP_HD double m_fmod(double a, double b) { return fmod(a, b); }
SRHIP_HD float m_atan2(float a, float b) { return (float)atan2((double)a, (double)b); }
SRHIP_HD double m_atan2(double a, double b) { return atan2(a, b); }
// Julia's Float32 ^ Float32 is evaluated by widening to Float64 (base/math.jl); same here.
SRHIP_HD float m_pow(float a, float b) { return (float)pow((double)a, (double)b); }
SRHIP_HD double m_pow(double a, double b) { return pow(a, b); }

// ---- operator semantics, floating point T ------------------------------------------------------
template <typename T> struct FOps {
  // binary (Julia Base + src/Operators.jl)
  static SRHIP_HD T add(T a, T b) { return a + b; }
  static SRHIP_HD T sub(T a, T b) { return a - b; }
  static SRHIP_HD T mul(T a, T b) { return a * b; }
  static SRHIP_HD T div(T a, T b) { return a / b; }
  // src/Operators.jl:82-84  greater(x, y) = (x > y) * one(x)
  static SRHIP_HD T greater(T a, T b) { return (a > b) ? T(1) : T(0); }
  // src/Operators.jl:85-87  cond(x, y) = (x > zero(x)) * y
  static SRHIP_HD T cond(T a, T b) { return (a > T(0)) ? b : m_copysign(T(0), b); }
  // src/Operators.jl:91-96
  static SRHIP_HD T logical_or(T a, T b) { return ((a > T(0)) | (b > T(0))) ? T(1) : T(0); }
  static SRHIP_HD T logical_and(T a, T b) { return ((a > T(0)) & (b > T(0))) ? T(1) : T(0); }
  static SRHIP_HD T max(T a, T b) { return m_max(a, b); }
  static SRHIP_HD T min(T a, T b) { return m_min(a, b); }
  // src/Operators.jl:28-36  safe_pow
  static SRHIP_HD T pow(T x, T y) {
    const bool yint = (y - m_trunc(y)) == T(0);  // isinteger(y): false for Inf/NaN
    if (yint) {
      if (y < T(0) && x == T(0)) return FP<T>::nan();
    } else {
      if (y > T(0) && x < T(0)) return FP<T>::nan();
      if (y < T(0) && x <= T(0)) return FP<T>::nan();
    }
    return m_pow(x, y);
  }
  // Julia Base mod(x::T, y::T) for floats: r = rem(x, y); r == 0 ? copysign(r, y) :
  // ((r > 0) xor (y > 0)) ? r + y : r
  static SRHIP_HD T mod(T x, T y) {
    const T r = m_fmod(x, y);
    if (r == T(0)) return m_copysign(r, y);
    if ((r > T(0)) != (y > T(0))) return r + y;
    return r;
  }
  static SRHIP_HD T atan2(T a, T b) { return m_atan2(a, b); }

  // unary
  static SRHIP_HD T neg(T x) { return -x; }
  static SRHIP_HD T square(T x) { return x * x; }        // src/Operators.jl:65
  static SRHIP_HD T cube(T x) { return (x * x) * x; }    // src/Operators.jl:66
  static SRHIP_HD T abs(T x) { return m_abs(x); }
  static SRHIP_HD T relu(T x) { return (x > T(0)) ? x : m_copysign(T(0), x); }  // :88-90
  static SRHIP_HD T cos(T x) { return m_cos(x); }
  static SRHIP_HD T sin(T x) { return m_sin(x); }
  static SRHIP_HD T tan(T x) { return m_tan(x); }
  static SRHIP_HD T exp(T x) { return m_exp(x); }
  // src/Operators.jl:37-60 safe_log*, safe_log1p, safe_acosh, safe_sqrt
  static SRHIP_HD T log(T x) { return (x <= T(0)) ? FP<T>::nan() : m_log(x); }
  static SRHIP_HD T log2(T x) { return (x <= T(0)) ? FP<T>::nan() : m_log2(x); }
  static SRHIP_HD T log10(T x) { return (x <= T(0)) ? FP<T>::nan() : m_log10(x); }
  static SRHIP_HD T log1p(T x) { return (x <= T(-1)) ? FP<T>::nan() : m_log1p(x); }
  static SRHIP_HD T sqrt(T x) { return (x < T(0)) ? FP<T>::nan() : m_sqrt(x); }
  static SRHIP_HD T acosh(T x) { return (x < T(1)) ? FP<T>::nan() : m_acosh(x); }
  // src/Operators.jl:17 atanh_clip(x) = atanh(mod(x + 1, 2) - 1)
  static SRHIP_HD T atanh_clip(T x) { return m_atanh(mod(x + T(1), T(2)) - T(1)); }
  static SRHIP_HD T sinh(T x) { return m_sinh(x); }
  static SRHIP_HD T cosh(T x) { return m_cosh(x); }
  static SRHIP_HD T tanh(T x) { return m_tanh(x); }
  // Julia throws DomainError for |x| > 1; the device returns NaN (-> did_succeed = false).
  static SRHIP_HD T asin(T x) { return m_asin(x); }
  static SRHIP_HD T acos(T x) { return m_acos(x); }
  static SRHIP_HD T atan(T x) { return m_atan(x); }
  static SRHIP_HD T asinh(T x) { return m_asinh(x); }
  static SRHIP_HD T erf(T x) { return m_erf(x); }
  static SRHIP_HD T erfc(T x) { return m_erfc(x); }
  // src/Operators.jl:11-15  gamma(x) = isinf(out) ? NaN : out
  static SRHIP_HD T gamma(T x) {
    const T g = m_tgamma(x);
    return m_isinf(g) ? FP<T>::nan() : g;
  }
  static SRHIP_HD T round(T x) { return m_rint(x); }  // Julia round: RoundNearest (ties even)
  static SRHIP_HD T floor(T x) { return m_floor(x); }
  static SRHIP_HD T ceil(T x) { return m_ceil(x); }
  // Julia sign: -1 / +1, keeps ±0, NaN -> NaN
  static SRHIP_HD T sign(T x) { return (x < T(0)) ? T(-1) : ((x > T(0)) ? T(1) : x); }
  static SRHIP_HD T exp2(T x) { return m_exp2(x); }
  static SRHIP_HD T expm1(T x) { return m_expm1(x); }
  static SRHIP_HD T cbrt(T x) { return m_cbrt(x); }
};

// ---- Int32 semantics: Julia Int32 wrap-around arithmetic (two's complement) ---------------------
struct IOps {
  using T = int32_t;
  static SRHIP_HD T w(uint32_t v) { return (T)v; }
  static SRHIP_HD T add(T a, T b) { return w((uint32_t)a + (uint32_t)b); }
  static SRHIP_HD T sub(T a, T b) { return w((uint32_t)a - (uint32_t)b); }
  static SRHIP_HD T mul(T a, T b) { return w((uint32_t)a * (uint32_t)b); }
  static SRHIP_HD T greater(T a, T b) { return a > b ? 1 : 0; }
  static SRHIP_HD T cond(T a, T b) { return a > 0 ? b : 0; }
  static SRHIP_HD T logical_or(T a, T b) { return ((a > 0) | (b > 0)) ? 1 : 0; }
  static SRHIP_HD T logical_and(T a, T b) { return ((a > 0) & (b > 0)) ? 1 : 0; }
  static SRHIP_HD T max(T a, T b) { return a > b ? a : b; }
  static SRHIP_HD T min(T a, T b) { return a < b ? a : b; }
  static SRHIP_HD T neg(T x) { return w(0u - (uint32_t)x); }
  static SRHIP_HD T square(T x) { return mul(x, x); }
  static SRHIP_HD T cube(T x) { return mul(mul(x, x), x); }
  static SRHIP_HD T abs(T x) { return x < 0 ? neg(x) : x; }
  static SRHIP_HD T relu(T x) { return x > 0 ? x : 0; }
  static SRHIP_HD T sign(T x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }
};

// ---- elementwise losses (LossFunctions.jl 0.10/0.11 distance losses, diff = output - target) ---
// Restated; the package is not in the container (see DESIGN.md "oracle").
template <typename T>
SRHIP_HD T loss_elem(int kind, T diff, T p0) {
  switch (kind) {
    case SRHIP_LOSS_L2: return diff * diff;                 // abs2(diff)
    case SRHIP_LOSS_L1: return m_abs(diff);
    case SRHIP_LOSS_LP: return m_pow(m_abs(diff), p0);      // abs(diff)^P
    case SRHIP_LOSS_HUBER: {                                // HuberLoss(d)
      const T a = m_abs(diff);
      return (a <= p0) ? T(0.5) * (diff * diff) : p0 * (a - T(0.5) * p0);
    }
    case SRHIP_LOSS_L1_EPS_INS: return m_max(T(0), m_abs(diff) - p0);
    case SRHIP_LOSS_L2_EPS_INS: { const T e = m_max(T(0), m_abs(diff) - p0); return e * e; }
    case SRHIP_LOSS_LOGIT_DIST: {                           // -log(4 e^d / (1 + e^d)^2)
      const T er = m_exp(diff);
      const T den = T(1) + er;
      return -m_log(T(4) * er / (den * den));
    }
    case SRHIP_LOSS_PERIODIC:                               // 1 - cos(2 pi diff / c)
      return T(1) - m_cos(diff * (T(2) * T(3.14159265358979323846)) / p0);
    case SRHIP_LOSS_QUANTILE:                               // diff * (tau - (diff < 0))
      return diff * (p0 - ((diff < T(0)) ? T(1) : T(0)));
    default: return FP<T>::nan();
  }
}
// LossFunctions.jl 0.11 margin losses (src/losses/margin.jl), of the agreement a = target * output.
// Restated from the published definitions (the package is not in the container; parity with it is
// unpinned); evaluated in T.
template <typename T>
SRHIP_HD T margin_loss(int kind, T a, T p0) {
  switch (kind) {
    case SRHIP_LOSS_ZERO_ONE: return a < T(0) ? T(1) : T(0);            // sign(a) < 0
    case SRHIP_LOSS_PERCEPTRON: return m_max(T(0), -a);
    case SRHIP_LOSS_LOGIT_MARGIN: return m_log1p(m_exp(-a));
    case SRHIP_LOSS_L1_HINGE: return m_max(T(0), T(1) - a);
    case SRHIP_LOSS_L2_HINGE: { const T h = T(1) - a; return a >= T(1) ? T(0) : h * h; }
    case SRHIP_LOSS_SMOOTHED_L1_HINGE: {                                // gamma = p0
      if (a >= T(1) - p0) { const T h = m_max(T(0), T(1) - a); return T(0.5) / p0 * (h * h); }
      return T(1) - p0 / T(2) - a;
    }
    case SRHIP_LOSS_MODIFIED_HUBER: {
      if (a >= T(-1)) { const T h = m_max(T(0), T(1) - a); return h * h; }
      return -T(4) * a;
    }
    case SRHIP_LOSS_L2_MARGIN: { const T h = T(1) - a; return h * h; }
    case SRHIP_LOSS_EXP: return m_exp(-a);
    case SRHIP_LOSS_SIGMOID: return T(1) - m_tanh(a);
    case SRHIP_LOSS_DWD_MARGIN: {                                       // q = p0
      if (a <= p0 / (p0 + T(1))) return T(1) - a;
      return (m_pow(p0, p0) / m_pow(p0 + T(1), p0 + T(1))) / m_pow(a, p0);
    }
    default: return FP<T>::nan();
  }
}
SRHIP_HD constexpr bool loss_is_margin(int kind) { return kind >= SRHIP_LOSS_ZERO_ONE && kind <= SRHIP_LOSS_DWD_MARGIN; }
// the elementwise loss of one row: distance losses of output - target, margin losses of
// target * output (LossFunctions' (loss)(output, target) for the two families)
template <typename T>
SRHIP_HD T loss_row(int kind, T output, T target, T p0) {
  return loss_is_margin(kind) ? margin_loss<T>(kind, target * output, p0) : loss_elem<T>(kind, output - target, p0);
}
// Int32 datasets: the elementwise loss is computed in Int32 wrap arithmetic and summed in Int64.
SRHIP_HD int32_t loss_elem_int(int kind, int32_t diff) {
  switch (kind) {
    case SRHIP_LOSS_L2: return IOps::mul(diff, diff);
    case SRHIP_LOSS_L1: return IOps::abs(diff);
    default: return 0;
  }
}

}  // namespace srhip
