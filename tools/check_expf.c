/* Exhaustive check of the Float32 exp (include/srhip_math.h srm_expf) over all 2^32 inputs:
 *  (1) the device formulation (srhip_eval_impl.h expf2_dev: NaN-propagating clamp to [-104, 89] instead
 *      of the branches, v_cvt_i32_f32 semantics, v_ldexp_f32) returns the same bits as srm_expf;
 *      and so does the range-free form of waves whose inputs all lie in [-87, 87] (dev_expf_fast);
 *  (2) accuracy against glibc's double exp rounded to Float32: max ULP distance and the share of
 *      inputs whose result differs.
 * Build: gcc -O2 -march=x86-64-v3 -ffp-contract=off -fopenmp tools/check_expf.c -lm -o /tmp/check_expf */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/srhip_math.h"

static float from_u(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t to_u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float nmax(float a, float b) { return (a != a || b != b) ? a + b : (a > b ? a : b); }
static float nmin(float a, float b) { return (a != a || b != b) ? a + b : (a < b ? a : b); }
static int cvt_i32(float x) { /* v_cvt_i32_f32: NaN -> 0, saturating */
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (int)0x80000000;
  return (int)x;
}
static float dev_expf(float x0) {
  const float x = nmin(nmax(x0, -104.0f), 89.0f);
  const float n = rintf(x * SRM_EXPF_LOG2E);
  float r = fmaf(n, SRM_EXPF_NLN2_HI, x);
  r = fmaf(n, SRM_EXPF_NLN2_LO, r);
  float p = SRM_EXPF_C6;
  p = fmaf(r, p, SRM_EXPF_C5);
  p = fmaf(r, p, SRM_EXPF_C4);
  p = fmaf(r, p, SRM_EXPF_C3);
  p = fmaf(r, p, 0.5f);
  p = fmaf(r, p, 1.0f);
  p = fmaf(r, p, 1.0f);
  return ldexpf(p, cvt_i32(n));
}
/* the device's range-free form for waves whose every |x| <= SRM_EXPF_FAST_MAX (srhip_eval_impl.h
 * expf2_fast): n by adding and subtracting 1.5 * 2^23 (the same ties-to-even rounding of the same
 * product as rintf), 2^n built in the exponent field from the low bits of the rounded sum, one
 * multiply instead of ldexp (both round the exact p 2^n once) */
#define SRM_EXPF_FAST_MAX 87.0f
static float dev_expf_fast(float x) {
  const float prod = x * SRM_EXPF_LOG2E;
  const float t = prod + 12582912.0f;
  const float n = t - 12582912.0f;
  float r = fmaf(n, SRM_EXPF_NLN2_HI, x);
  r = fmaf(n, SRM_EXPF_NLN2_LO, r);
  float p = SRM_EXPF_C6;
  p = fmaf(r, p, SRM_EXPF_C5);
  p = fmaf(r, p, SRM_EXPF_C4);
  p = fmaf(r, p, SRM_EXPF_C3);
  p = fmaf(r, p, 0.5f);
  p = fmaf(r, p, 1.0f);
  p = fmaf(r, p, 1.0f);
  const float scale = from_u((to_u(t) << 23) + 0x3F800000u);
  return p * scale;
}
static int64_t ordered(float f) {
  const int32_t i = (int32_t)to_u(f);
  return i < 0 ? (int64_t)INT32_MIN - i : i;
}
int main(void) {
  long long mism = 0, differ = 0, over1 = 0, total = 0;
  long long maxulp = 0;
#pragma omp parallel for reduction(+ : mism, differ, over1, total) reduction(max : maxulp) schedule(static)
  for (int64_t i = 0; i < (1LL << 32); ++i) {
    const float x = from_u((uint32_t)i);
    const float a = srm_expf(x), d = dev_expf(x);
    if (x != x) {
      if (a == a || d == d) ++mism;
      continue;
    }
    if (to_u(a) != to_u(d)) ++mism;
    if (fabsf(x) <= SRM_EXPF_FAST_MAX && to_u(a) != to_u(dev_expf_fast(x))) ++mism;
    const float cr = (float)exp((double)x);
    const long long u = llabs(ordered(a) - ordered(cr));
    ++total;
    if (u) ++differ;
    if (u > 1) ++over1;
    if (u > maxulp) maxulp = u;
  }
  printf("device-vs-scalar mismatches %lld; non-NaN inputs %lld, differ from rounded glibc %lld (%.4f%%), >1 ULP %lld, max %lld ULP\n",
         mism, total, differ, 100.0 * differ / total, over1, maxulp);
  return mism != 0 || maxulp > 1;
}
