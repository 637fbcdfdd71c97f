/* sr_oracle.c — CPU oracle for the srhip parity tests.
 *
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, as the checker or the timed CPU baseline; the product
 * (libsrhip.so, the srhip package) never links or calls it.
 *
 * Restates, independently of the product sources:
 *   - operator semantics: reference src/Operators.jl:11-96 (safe_pow :28-36, safe_log* :37-48,
 *     safe_log1p :49-52, safe_acosh :53-56, safe_sqrt :57-60, square/cube/neg :65-80,
 *     greater/cond/relu/logical_or/logical_and :82-96 with Julia's Bool strong zero),
 *     atanh_clip :17, gamma :11-15, and the Julia Base functions they alias
 *     (src/Options.jl:92-150);
 *   - DynamicExpressions v0.16 eval_tree_array (sr_oracle_impl.h);
 *   - LossFunctions.jl 0.10/0.11 distance losses used by src/LossFunctions.jl:13-33.
 * Pinned by the reference's known-answer tests restated in tests/golden (see
 * tests/golden/make_golden.py) — Julia is not available in this container.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/srhip.h"
#include "../include/srhip_math.h"

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)

/* ---------------- Float32 ----------------
 * Transcendentals widen to Float64 and round once (Julia evaluates Float32 trig through Float64
 * kernels, and Float32 ^ by widening): exp/log/sin/cos/tan from the shared include/srhip_math.h
 * (fdlibm restatement, pinned against glibc in tests/test_math_accuracy.py), the rest from glibc. */
#define W1(fn, x) ((float)fn((double)(x)))
static float julia_modf32(float x, float y) {
  const float r = fmodf(x, y);
  if (r == 0.0f) return copysignf(r, y);
  if ((r > 0.0f) != (y > 0.0f)) return r + y;
  return r;
}
static float bin_f32(int op, float a, float b) {
  switch (op) {
    case SRHIP_OP_ADD: return a + b;
    case SRHIP_OP_SUB: return a - b;
    case SRHIP_OP_MUL: return a * b;
    case SRHIP_OP_DIV: return a / b;
    case SRHIP_OP_POW: {
      const int yint = (b - truncf(b)) == 0.0f;
      if (yint) {
        if (b < 0.0f && a == 0.0f) return NAN;
      } else {
        if (b > 0.0f && a < 0.0f) return NAN;
        if (b < 0.0f && a <= 0.0f) return NAN;
      }
      return (float)pow((double)a, (double)b);
    }
    case SRHIP_OP_GREATER: return (a > b) ? 1.0f : 0.0f;
    case SRHIP_OP_COND: return (a > 0.0f) ? b : copysignf(0.0f, b);
    case SRHIP_OP_LOGICAL_OR: return ((a > 0.0f) || (b > 0.0f)) ? 1.0f : 0.0f;
    case SRHIP_OP_LOGICAL_AND: return ((a > 0.0f) && (b > 0.0f)) ? 1.0f : 0.0f;
    case SRHIP_OP_MAX:
      if (isnan(a) || isnan(b)) return NAN;
      if (a == b) return signbit(a) ? b : a;
      return a > b ? a : b;
    case SRHIP_OP_MIN:
      if (isnan(a) || isnan(b)) return NAN;
      if (a == b) return signbit(a) ? a : b;
      return a < b ? a : b;
    case SRHIP_OP_MOD: return julia_modf32(a, b);
    case SRHIP_OP_ATAN2: return (float)atan2((double)a, (double)b);
    default: return NAN;
  }
}
static float un_f32(int op, float x) {
  switch (op) {
    case SRHIP_OP_NEG: return -x;
    case SRHIP_OP_SQUARE: return x * x;
    case SRHIP_OP_CUBE: return x * x * x;
    case SRHIP_OP_ABS: return fabsf(x);
    case SRHIP_OP_RELU: return x > 0.0f ? x : copysignf(0.0f, x);
    case SRHIP_OP_COS: return srm_cosf(x);
    case SRHIP_OP_SIN: return srm_sinf(x);
    case SRHIP_OP_TAN: return srm_tanf(x);
    case SRHIP_OP_EXP: return srm_expf(x);
    case SRHIP_OP_LOG: return x <= 0.0f ? NAN : srm_logf(x);
    case SRHIP_OP_LOG2: return x <= 0.0f ? NAN : W1(log2, x);
    case SRHIP_OP_LOG10: return x <= 0.0f ? NAN : W1(log10, x);
    case SRHIP_OP_LOG1P: return x <= -1.0f ? NAN : W1(log1p, x);
    case SRHIP_OP_SQRT: return x < 0.0f ? NAN : sqrtf(x);
    case SRHIP_OP_ACOSH: return x < 1.0f ? NAN : W1(acosh, x);
    case SRHIP_OP_ATANH_CLIP: return W1(atanh, julia_modf32(x + 1.0f, 2.0f) - 1.0f);
    case SRHIP_OP_SINH: return W1(sinh, x);
    case SRHIP_OP_COSH: return W1(cosh, x);
    case SRHIP_OP_TANH: return W1(tanh, x);
    case SRHIP_OP_ASIN: return W1(asin, x);
    case SRHIP_OP_ACOS: return W1(acos, x);
    case SRHIP_OP_ATAN: return W1(atan, x);
    case SRHIP_OP_ASINH: return W1(asinh, x);
    case SRHIP_OP_ERF: return W1(erf, x);
    case SRHIP_OP_ERFC: return W1(erfc, x);
    case SRHIP_OP_GAMMA: { const float g = W1(tgamma, x); return isinf(g) ? NAN : g; }
    case SRHIP_OP_ROUND: return rintf(x);
    case SRHIP_OP_FLOOR: return floorf(x);
    case SRHIP_OP_CEIL: return ceilf(x);
    case SRHIP_OP_SIGN: return x < 0.0f ? -1.0f : (x > 0.0f ? 1.0f : x);
    case SRHIP_OP_EXP2: return W1(exp2, x);
    case SRHIP_OP_EXPM1: return W1(expm1, x);
    case SRHIP_OP_CBRT: return W1(cbrt, x);
    default: return NAN;
  }
}
/* Julia's max (the device's v_maximum: NaN-propagating, +0 above -0) */
static float fmaxf_nan(float a, float b) {
  if (a != a || b != b) return NAN;
  if (a == b) return signbit(a) ? b : a;
  return a > b ? a : b;
}
static double fmax_nan(double a, double b) {
  if (a != a || b != b) return NAN;
  if (a == b) return signbit(a) ? b : a;
  return a > b ? a : b;
}
/* LossFunctions.jl 0.11 margin losses of the agreement a = target * output (src/losses/margin.jl;
 * the package is not in the container: restated from its published definitions, parity unpinned) */
static float margin_f32(int kind, float a, float p0) {
  switch (kind) {
    case SRHIP_LOSS_ZERO_ONE: return a < 0.0f ? 1.0f : 0.0f;
    case SRHIP_LOSS_PERCEPTRON: return fmaxf_nan(0.0f, -a);
    case SRHIP_LOSS_LOGIT_MARGIN: return W1(log1p, srm_expf(-a));
    case SRHIP_LOSS_L1_HINGE: return fmaxf_nan(0.0f, 1.0f - a);
    case SRHIP_LOSS_L2_HINGE: { const float h = 1.0f - a; return a >= 1.0f ? 0.0f : h * h; }
    case SRHIP_LOSS_SMOOTHED_L1_HINGE:
      if (a >= 1.0f - p0) { const float h = fmaxf_nan(0.0f, 1.0f - a); return 0.5f / p0 * (h * h); }
      return 1.0f - p0 / 2.0f - a;
    case SRHIP_LOSS_MODIFIED_HUBER:
      if (a >= -1.0f) { const float h = fmaxf_nan(0.0f, 1.0f - a); return h * h; }
      return -4.0f * a;
    case SRHIP_LOSS_L2_MARGIN: { const float h = 1.0f - a; return h * h; }
    case SRHIP_LOSS_EXP: return srm_expf(-a);
    case SRHIP_LOSS_SIGMOID: return 1.0f - W1(tanh, a);
    case SRHIP_LOSS_DWD_MARGIN:
      if (a <= p0 / (p0 + 1.0f)) return 1.0f - a;
      return ((float)pow((double)p0, (double)p0) / (float)pow((double)(p0 + 1.0f), (double)(p0 + 1.0f))) /
             (float)pow((double)a, (double)p0);
    default: return NAN;
  }
}
static float dist_f32(int kind, float d, float p0);
/* one row's elementwise loss: distance losses of output - target, margin losses of target * output */
static float loss_f32(int kind, float out, float y, float p0) {
  return kind >= SRHIP_LOSS_ZERO_ONE ? margin_f32(kind, y * out, p0) : dist_f32(kind, out - y, p0);
}
static float dist_f32(int kind, float d, float p0) {
  switch (kind) {
    case SRHIP_LOSS_L2: return d * d;
    case SRHIP_LOSS_L1: return fabsf(d);
    case SRHIP_LOSS_LP: return (float)pow((double)fabsf(d), (double)p0);
    case SRHIP_LOSS_HUBER: { const float a = fabsf(d); return a <= p0 ? 0.5f * (d * d) : p0 * (a - 0.5f * p0); }
    case SRHIP_LOSS_L1_EPS_INS: { const float e = fabsf(d) - p0; return e > 0.0f ? e : 0.0f; }
    case SRHIP_LOSS_L2_EPS_INS: { const float e = fabsf(d) - p0; const float m = e > 0.0f ? e : 0.0f; return m * m; }
    case SRHIP_LOSS_LOGIT_DIST: { const float er = srm_expf(d); const float den = 1.0f + er; return -srm_logf(4.0f * er / (den * den)); }
    case SRHIP_LOSS_PERIODIC: return 1.0f - srm_cosf(d * (2.0f * 3.14159265358979323846f) / p0);
    case SRHIP_LOSS_QUANTILE: return d * (p0 - (d < 0.0f ? 1.0f : 0.0f));
    default: return NAN;
  }
}

/* ---------------- Float64 ----------------
 * ORACLE_LIBM_GLIBC (the liboracle_glibc64.so variant, oracle/libm_sensitivity.py only): Float64
 * exp / log / sin / cos from glibc instead of the shared header -- a second near-correctly-rounded
 * libm, to measure how far a loss moves when only the transcendental algorithm changes. */
#if ORACLE_LIBM_GLIBC
#define ORC_EXP64(x) exp(x)
#define ORC_LOG64(x) log(x)
#define ORC_SIN64(x) sin(x)
#define ORC_COS64(x) cos(x)
#else
#define ORC_EXP64(x) srm_exp(x)
#define ORC_LOG64(x) srm_log(x)
#define ORC_SIN64(x) srm_sin(x)
#define ORC_COS64(x) srm_cos(x)
#endif
static double julia_modf64(double x, double y) {
  const double r = fmod(x, y);
  if (r == 0.0) return copysign(r, y);
  if ((r > 0.0) != (y > 0.0)) return r + y;
  return r;
}
static double bin_f64(int op, double a, double b) {
  switch (op) {
    case SRHIP_OP_ADD: return a + b;
    case SRHIP_OP_SUB: return a - b;
    case SRHIP_OP_MUL: return a * b;
    case SRHIP_OP_DIV: return a / b;
    case SRHIP_OP_POW: {
      const int yint = (b - trunc(b)) == 0.0;
      if (yint) {
        if (b < 0.0 && a == 0.0) return NAN;
      } else {
        if (b > 0.0 && a < 0.0) return NAN;
        if (b < 0.0 && a <= 0.0) return NAN;
      }
      return pow(a, b);
    }
    case SRHIP_OP_GREATER: return (a > b) ? 1.0 : 0.0;
    case SRHIP_OP_COND: return (a > 0.0) ? b : copysign(0.0, b);
    case SRHIP_OP_LOGICAL_OR: return ((a > 0.0) || (b > 0.0)) ? 1.0 : 0.0;
    case SRHIP_OP_LOGICAL_AND: return ((a > 0.0) && (b > 0.0)) ? 1.0 : 0.0;
    case SRHIP_OP_MAX:
      if (isnan(a) || isnan(b)) return NAN;
      if (a == b) return signbit(a) ? b : a;
      return a > b ? a : b;
    case SRHIP_OP_MIN:
      if (isnan(a) || isnan(b)) return NAN;
      if (a == b) return signbit(a) ? a : b;
      return a < b ? a : b;
    case SRHIP_OP_MOD: return julia_modf64(a, b);
    case SRHIP_OP_ATAN2: return atan2(a, b);
    default: return NAN;
  }
}
static double un_f64(int op, double x) {
  switch (op) {
    case SRHIP_OP_NEG: return -x;
    case SRHIP_OP_SQUARE: return x * x;
    case SRHIP_OP_CUBE: return x * x * x;
    case SRHIP_OP_ABS: return fabs(x);
    case SRHIP_OP_RELU: return x > 0.0 ? x : copysign(0.0, x);
    case SRHIP_OP_COS: return ORC_COS64(x);
    case SRHIP_OP_SIN: return ORC_SIN64(x);
    case SRHIP_OP_TAN: return srm_tan(x);
    case SRHIP_OP_EXP: return ORC_EXP64(x);
    case SRHIP_OP_LOG: return x <= 0.0 ? NAN : ORC_LOG64(x);
    case SRHIP_OP_LOG2: return x <= 0.0 ? NAN : log2(x);
    case SRHIP_OP_LOG10: return x <= 0.0 ? NAN : log10(x);
    case SRHIP_OP_LOG1P: return x <= -1.0 ? NAN : log1p(x);
    case SRHIP_OP_SQRT: return x < 0.0 ? NAN : sqrt(x);
    case SRHIP_OP_ACOSH: return x < 1.0 ? NAN : acosh(x);
    case SRHIP_OP_ATANH_CLIP: return atanh(julia_modf64(x + 1.0, 2.0) - 1.0);
    case SRHIP_OP_SINH: return sinh(x);
    case SRHIP_OP_COSH: return cosh(x);
    case SRHIP_OP_TANH: return tanh(x);
    case SRHIP_OP_ASIN: return asin(x);
    case SRHIP_OP_ACOS: return acos(x);
    case SRHIP_OP_ATAN: return atan(x);
    case SRHIP_OP_ASINH: return asinh(x);
    case SRHIP_OP_ERF: return erf(x);
    case SRHIP_OP_ERFC: return erfc(x);
    case SRHIP_OP_GAMMA: { const double g = tgamma(x); return isinf(g) ? NAN : g; }
    case SRHIP_OP_ROUND: return rint(x);
    case SRHIP_OP_FLOOR: return floor(x);
    case SRHIP_OP_CEIL: return ceil(x);
    case SRHIP_OP_SIGN: return x < 0.0 ? -1.0 : (x > 0.0 ? 1.0 : x);
    case SRHIP_OP_EXP2: return exp2(x);
    case SRHIP_OP_EXPM1: return expm1(x);
    case SRHIP_OP_CBRT: return cbrt(x);
    default: return NAN;
  }
}
static double margin_f64(int kind, double a, double p0) {
  switch (kind) {
    case SRHIP_LOSS_ZERO_ONE: return a < 0.0 ? 1.0 : 0.0;
    case SRHIP_LOSS_PERCEPTRON: return fmax_nan(0.0, -a);
    case SRHIP_LOSS_LOGIT_MARGIN: return log1p(srm_exp(-a));
    case SRHIP_LOSS_L1_HINGE: return fmax_nan(0.0, 1.0 - a);
    case SRHIP_LOSS_L2_HINGE: { const double h = 1.0 - a; return a >= 1.0 ? 0.0 : h * h; }
    case SRHIP_LOSS_SMOOTHED_L1_HINGE:
      if (a >= 1.0 - p0) { const double h = fmax_nan(0.0, 1.0 - a); return 0.5 / p0 * (h * h); }
      return 1.0 - p0 / 2.0 - a;
    case SRHIP_LOSS_MODIFIED_HUBER:
      if (a >= -1.0) { const double h = fmax_nan(0.0, 1.0 - a); return h * h; }
      return -4.0 * a;
    case SRHIP_LOSS_L2_MARGIN: { const double h = 1.0 - a; return h * h; }
    case SRHIP_LOSS_EXP: return srm_exp(-a);
    case SRHIP_LOSS_SIGMOID: return 1.0 - tanh(a);
    case SRHIP_LOSS_DWD_MARGIN:
      if (a <= p0 / (p0 + 1.0)) return 1.0 - a;
      return (pow(p0, p0) / pow(p0 + 1.0, p0 + 1.0)) / pow(a, p0);
    default: return NAN;
  }
}
static double dist_f64(int kind, double d, double p0);
static double loss_f64(int kind, double out, double y, double p0) {
  return kind >= SRHIP_LOSS_ZERO_ONE ? margin_f64(kind, y * out, p0) : dist_f64(kind, out - y, p0);
}
static double dist_f64(int kind, double d, double p0) {
  switch (kind) {
    case SRHIP_LOSS_L2: return d * d;
    case SRHIP_LOSS_L1: return fabs(d);
    case SRHIP_LOSS_LP: return pow(fabs(d), p0);
    case SRHIP_LOSS_HUBER: { const double a = fabs(d); return a <= p0 ? 0.5 * (d * d) : p0 * (a - 0.5 * p0); }
    case SRHIP_LOSS_L1_EPS_INS: { const double e = fabs(d) - p0; return e > 0.0 ? e : 0.0; }
    case SRHIP_LOSS_L2_EPS_INS: { const double e = fabs(d) - p0; const double m = e > 0.0 ? e : 0.0; return m * m; }
    case SRHIP_LOSS_LOGIT_DIST: { const double er = srm_exp(d); const double den = 1.0 + er; return -srm_log(4.0 * er / (den * den)); }
    case SRHIP_LOSS_PERIODIC: return 1.0 - srm_cos(d * (2.0 * 3.14159265358979323846) / p0);
    case SRHIP_LOSS_QUANTILE: return d * (p0 - (d < 0.0 ? 1.0 : 0.0));
    default: return NAN;
  }
}

/* ---------------- Int32 (Julia wrap-around) ---------------- */
static int32_t wrap(uint32_t v) { return (int32_t)v; }
static int32_t bin_i32(int op, int32_t a, int32_t b) {
  switch (op) {
    case SRHIP_OP_ADD: return wrap((uint32_t)a + (uint32_t)b);
    case SRHIP_OP_SUB: return wrap((uint32_t)a - (uint32_t)b);
    case SRHIP_OP_MUL: return wrap((uint32_t)a * (uint32_t)b);
    case SRHIP_OP_GREATER: return a > b;
    case SRHIP_OP_COND: return a > 0 ? b : 0;
    case SRHIP_OP_LOGICAL_OR: return (a > 0) || (b > 0);
    case SRHIP_OP_LOGICAL_AND: return (a > 0) && (b > 0);
    case SRHIP_OP_MAX: return a > b ? a : b;
    case SRHIP_OP_MIN: return a < b ? a : b;
    default: return 0;
  }
}
static int32_t un_i32(int op, int32_t x) {
  switch (op) {
    case SRHIP_OP_NEG: return wrap(0u - (uint32_t)x);
    case SRHIP_OP_SQUARE: return wrap((uint32_t)x * (uint32_t)x);
    case SRHIP_OP_CUBE: return wrap((uint32_t)x * (uint32_t)x * (uint32_t)x);
    case SRHIP_OP_ABS: return x < 0 ? wrap(0u - (uint32_t)x) : x;
    case SRHIP_OP_RELU: return x > 0 ? x : 0;
    case SRHIP_OP_SIGN: return x > 0 ? 1 : (x < 0 ? -1 : 0);
    default: return 0;
  }
}

/* scalar entry points (used by tests to check operator semantics one value at a time) */
float oracle_bin_f32(int op, float a, float b) { return bin_f32(op, a, b); }
/* the shared libm (include/srhip_math.h), vectorised for tests/test_math_accuracy.py */
void oracle_srm_f64(int which, const double* x, double* y, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    switch (which) {
      case 0: y[i] = srm_exp(x[i]); break;
      case 1: y[i] = srm_log(x[i]); break;
      case 2: y[i] = srm_sin(x[i]); break;
      case 3: y[i] = srm_cos(x[i]); break;
      default: y[i] = srm_tan(x[i]); break;
    }
  }
}
void oracle_srm_f32(int which, const float* x, float* y, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    switch (which) {
      case 0: y[i] = srm_expf(x[i]); break;
      case 1: y[i] = srm_logf(x[i]); break;
      case 2: y[i] = srm_sinf(x[i]); break;
      case 3: y[i] = srm_cosf(x[i]); break;
      case 5: y[i] = srm_jtrigf(1, x[i]); break; /* Julia's Float32 sin (SRHIP_JULIA_TRIG restatement) */
      case 6: y[i] = srm_jtrigf(0, x[i]); break; /* Julia's Float32 cos */
      default: y[i] = srm_tanf(x[i]); break;
    }
  }
}
float oracle_un_f32(int op, float x) { return un_f32(op, x); }
double oracle_bin_f64(int op, double a, double b) { return bin_f64(op, a, b); }
double oracle_un_f64(int op, double x) { return un_f64(op, x); }
int32_t oracle_bin_i32(int op, int32_t a, int32_t b) { return bin_i32(op, a, b); }
int32_t oracle_un_i32(int op, int32_t x) { return un_i32(op, x); }

#define T float
#define SFX f32
#define IS_INT 0
#define OVF_T (ldexpl(1.0L, 128) - ldexpl(1.0L, 103))
#include "sr_oracle_impl.h"
#undef T
#undef SFX
#undef IS_INT
#undef OVF_T

#define T double
#define SFX f64
#define IS_INT 0
#define OVF_T (ldexpl(1.0L, 1024) - ldexpl(1.0L, 970))
#include "sr_oracle_impl.h"
#undef T
#undef SFX
#undef IS_INT
#undef OVF_T

#define T int32_t
#define SFX i32
#define IS_INT 1
#define OVF_T 0
static int32_t loss_i32(int kind, int32_t d, int32_t p0) { (void)p0; return kind == SRHIP_LOSS_L1 ? (d < 0 ? wrap(0u - (uint32_t)d) : d) : wrap((uint32_t)d * (uint32_t)d); }
#include "sr_oracle_impl.h"
#undef T
#undef SFX
#undef IS_INT
#undef OVF_T

#include "sr_oracle_grad.h"
