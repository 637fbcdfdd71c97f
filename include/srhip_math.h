/*
 * srhip_math.h — the scalar libm of the srhip evaluator: exp, log, sin, cos (and tan) in Float64,
 * written with IEEE-754 basic operations and fma only, so that the gfx950 kernels (hipcc) and the
 * CPU parity oracle (gcc) compute bit-identical values from this one source.
 *
 * Why it exists.  The reference evaluates operators with Julia Base.Math (pure-Julia libm derived
 * from FreeBSD msun / fdlibm).  Vendor libms (OCML on the device, glibc on the host) are each
 * within ~1 ULP of it but not bit-identical, and symbolic-regression trees routinely amplify a
 * 1-ULP difference chaotically (cos(exp(x) * c) at large arguments), so parity at 1e-6 / 1e-12
 * relative loss needs the device and the oracle to share the function values.  This file restates
 * the fdlibm algorithms (e_exp.c reduction, e_log.c, k_sin.c, k_cos.c, e_rem_pio2.c, with a
 * Payne-Hanek reduction written for 64-bit limbs); every constant is the fdlibm one (reduction
 * constants regenerated with mpmath and checked bit-for-bit, see tests/test_math_accuracy.py,
 * which also pins every function against glibc: <= 1 ULP in Float64, and Float32 values that are
 * the correctly rounded results in all but double-rounding cases).
 *
 * Float32 sin / cos / tan / log widen to Float64 and round once (srm_*f below), as Julia does for
 * Float32 trigonometry (DoubleFloat32 kernels) and for Float32 `^`; Float32 exp is Julia's own
 * Float32 algorithm (srm_expf).
 *
 * Usable from C99 (oracle, gcc) and HIP C++ (host and device).  Compile WITHOUT fp contraction
 * (-ffp-contract=off): the explicit fma() calls are the only fused operations.
 */
#ifndef SRHIP_MATH_H
#define SRHIP_MATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SRM_FN __host__ __device__ static inline __attribute__((always_inline))
#define SRM_NOINLINE __host__ __device__ static __attribute__((noinline))
#else
#define SRM_FN static inline
#define SRM_NOINLINE static
#endif

/* ---- bit helpers ---------------------------------------------------------------------------- */
SRM_FN uint64_t srm_bits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
SRM_FN double srm_from_bits(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }
SRM_FN double srm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
SRM_FN double srm_rint(double x) { return __builtin_rint(x); }
SRM_FN double srm_inf(void) { return __builtin_inf(); }
SRM_FN double srm_nan(void) { return __builtin_nan(""); }

/* ---- exp ------------------------------------------------------------------------------------ */
/* fdlibm e_exp.c argument reduction x = k ln2 + r, |r| <= ln2/2, with ln2 split so that k*ln2HI is
 * exact; e^r by a degree-13 Taylor polynomial (truncation < 2^-57 on |r| <= 0.3466) instead of
 * fdlibm's rational form, which would need a division (a ~10-instruction sequence on gfx950). */
SRM_FN double srm_exp(double x) {
  const double o_threshold = 7.09782712893383973096e+02;  /* 0x40862E42 FEFA39EF */
  const double u_threshold = -7.45133219101941108420e+02; /* 0xc0874910 D52D3051 */
  const double invln2 = 1.44269504088896338700e+00;
  const double ln2HI = 6.93147180369123816490e-01; /* 0x3fe62e42 fee00000 */
  const double ln2LO = 1.90821492927058770002e-10; /* 0x3dea39ef 35793c76 */
  if (!(x == x)) return x + x;
  if (x > o_threshold) return srm_inf();
  if (x < u_threshold) return 0.0;
  const double k = srm_rint(x * invln2);
  const double hi = srm_fma(-k, ln2HI, x); /* exact product, one rounding (== fdlibm x - k*ln2HI) */
  const double lo = k * ln2LO;
  const double r = hi - lo;
  /* q = sum_{n=2}^{13} r^(n-2) / n! */
  double q = 1.6059043836821613e-10;          /* 1/13! */
  q = srm_fma(q, r, 2.08767569878681e-09);  /* 1/12! */
  q = srm_fma(q, r, 2.505210838544172e-08);  /* 1/11! */
  q = srm_fma(q, r, 2.755731922398589e-07);  /* 1/10! */
  q = srm_fma(q, r, 2.7557319223985893e-06);  /* 1/9!  */
  q = srm_fma(q, r, 2.48015873015873e-05);  /* 1/8!  */
  q = srm_fma(q, r, 1.984126984126984e-04);  /* 1/7!  */
  q = srm_fma(q, r, 1.388888888888889e-03);  /* 1/6!  */
  q = srm_fma(q, r, 8.333333333333333e-03);  /* 1/5!  */
  q = srm_fma(q, r, 4.1666666666666664e-02);  /* 1/4!  */
  q = srm_fma(q, r, 1.6666666666666666e-01);  /* 1/3!  */
  q = srm_fma(q, r, 0.5);                         /* 1/2!  */
  /* r as hi - lo: e^r = 1 + (hi - lo) + r^2 q, with the lo correction kept out of the rounding of r */
  const double s = srm_fma(r * r, q, -lo) + hi;
  const double y = 1.0 + s;
  /* y 2^k in two exact steps (k1, k2 in the normal range); a subnormal result rounds once */
  const int ki = (int)k, k1 = ki / 2, k2 = ki - k1;
  return (y * srm_from_bits((uint64_t)(k1 + 1023) << 52)) * srm_from_bits((uint64_t)(k2 + 1023) << 52);
}

/* ---- log ------------------------------------------------------------------------------------ */
/* fdlibm e_log.c: x = 2^k (1+f), 1+f in [sqrt(2)/2, sqrt(2)); s = f/(2+f); log(1+f) = f - hfsq +
 * s (hfsq + R(s^2)) with fdlibm's Lg1..Lg7.  Caller handles the reference's safe_log domain. */
SRM_FN double srm_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  uint64_t u = srm_bits(x);
  int32_t hx = (int32_t)(u >> 32);
  int k = 0;
  if (hx < 0x00100000) {                                   /* x < 2^-1022 (or negative) */
    if ((u & 0x7fffffffffffffffULL) == 0) return -srm_inf(); /* log(+-0) = -inf */
    if (hx < 0) return srm_nan();                            /* log(-x) = NaN */
    k -= 54;
    x *= 1.80143985094819840000e+16;                         /* 2^54: subnormal, scale up */
    u = srm_bits(x);
    hx = (int32_t)(u >> 32);
  }
  if (hx >= 0x7ff00000) return x + x; /* Inf or NaN */
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  x = srm_from_bits(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (u & 0xffffffffULL)); /* x or x/2 */
  k += (i >> 20);
  const double f = x - 1.0;
  const double dk = (double)k;
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const int32_t ii = (hx - 0x6147a) | (0x6b851 - hx);
  if (f == 0.0) return dk * ln2_hi + dk * ln2_lo;
  if (ii > 0) {
    const double hfsq = 0.5 * f * f;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* ---- sin / cos kernels on [-pi/4, pi/4] (fdlibm k_sin.c / k_cos.c), x + y the reduced arg ---- */
SRM_FN double srm_ksin(double x, double y) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x;
  const double w = z * z;
  const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  const double v = z * x;
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
SRM_FN double srm_kcos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = x * x;
  double w = z * z;
  const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* ---- argument reduction x = n pi/2 + (y0 + y1) ------------------------------------------------ */
/* 2/pi, 64 bits per word, most significant first (regenerated with mpmath in tests). */
#define SRM_TWO_OVER_PI_WORDS                                                                     \
  {0xA2F9836E4E441529ULL, 0xFC2757D1F534DDC0ULL, 0xDB6295993C439041ULL, 0xFE5163ABDEBBC561ULL,    \
   0xB7246E3A424DD2E0ULL, 0x06492EEA09D1921CULL, 0xFE1DEB1CB129A73EULL, 0xE88235F52EBB4484ULL,    \
   0xE99C7026B45F7E41ULL, 0x3991D639835339F4ULL, 0x9C845F8BBDF9283BULL, 0x1FF897FFDE05980FULL,    \
   0xEF2F118B5A0A6D1FULL, 0x6D367ECF27CB09B7ULL, 0x4F463F669E5FEA2DULL, 0x7527BAC7EBE5F17BULL,    \
   0x3D0739F78A5292EAULL, 0x6BFB5FB11F8D5D08ULL, 0x56033046FC7B6BABULL, 0xF0CFBC209AF4361DULL}
#if defined(__HIPCC__)
__device__ __constant__ static const uint64_t srm_2opi_dev[20] = SRM_TWO_OVER_PI_WORDS;
#endif
static const uint64_t srm_2opi_host[20] = SRM_TWO_OVER_PI_WORDS;

/* 64 bits of 2/pi starting at fraction bit `pos` (1 = the first bit after the binary point);
 * bits at positions <= 0 are zero (2/pi < 1). */
SRM_FN uint64_t srm_2opi_bits(int pos) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t* T = srm_2opi_dev;
#else
  const uint64_t* T = srm_2opi_host;
#endif
  const int b = pos - 1;
  if (b <= -64) return 0;
  if (b < 0) return T[0] >> (-b);
  const int k = b >> 6, sh = b & 63;
  return sh ? ((T[k] << sh) | (T[k + 1] >> (64 - sh))) : T[k];
}

/* Payne-Hanek for |x| >= 2^20 pi/2: x = M 2^E (M the 53-bit significand); x 2/pi mod 4 from a
 * 192-bit window of 2/pi starting at fraction bit E-1 (bits of weight >= 4 dropped), as a
 * 192-bit fixed-point product; the fraction is rounded to the nearest quadrant. */
SRM_NOINLINE int srm_rem_pio2_large(double x, double* y0, double* y1) {
  const uint64_t u = srm_bits(x);
  const int e = (int)((u >> 52) & 0x7ff) - 1023;
  const uint64_t M = (u & 0x000fffffffffffffULL) | 0x0010000000000000ULL;
  const int E = e - 52;
  const uint64_t w2 = srm_2opi_bits(E - 1), w1 = srm_2opi_bits(E - 1 + 64), w0 = srm_2opi_bits(E - 1 + 128);
  /* P = M * [w2:w1:w0] mod 2^192 */
  const unsigned __int128 q0 = (unsigned __int128)M * w0;
  const unsigned __int128 q1 = (unsigned __int128)M * w1 + (uint64_t)(q0 >> 64);
  const uint64_t p0 = (uint64_t)q0, p1 = (uint64_t)q1;
  const uint64_t p2 = (uint64_t)M * w2 + (uint64_t)(q1 >> 64);
  /* value = P 2^-190: quadrant = bits 190..191, fraction = bits 0..189 */
  int n = (int)(p2 >> 62);
  const uint64_t T1 = (p2 << 2) | (p1 >> 62); /* top 64 fraction bits */
  const uint64_t T2 = (p1 << 2) | (p0 >> 62); /* next 64 */
  const int64_t Ts = (int64_t)T1;             /* fraction >= 1/2 reads negative: f - 1 */
  if (Ts < 0) n += 1;
  /* f = Ts 2^-64 + T2 2^-128, split into a 53-bit head and a tail */
  const double fhi = (double)(Ts >> 11) * 1.1102230246251565404e-16;                      /* 2^-53 */
  const double flo = (double)(T1 & 0x7ff) * 5.42101086242752217004e-20                     /* 2^-64 */
                     + (double)T2 * 2.93873587705571876992e-39;                            /* 2^-128 */
  const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
  const double rhi = fhi * pio2_hi;
  const double rlo = srm_fma(fhi, pio2_hi, -rhi) + (fhi * pio2_lo + flo * pio2_hi);
  const double s = rhi + rlo;
  *y0 = (x < 0.0) ? -s : s;
  const double t = rlo - (s - rhi);
  *y1 = (x < 0.0) ? -t : t;
  return (x < 0.0) ? -n : n;
}

/* fdlibm e_rem_pio2.c for |x| < 2^20 pi/2 (three Cody-Waite rounds with 33-bit pieces of pi/2). */
SRM_FN int srm_rem_pio2(double x, double* y0, double* y1) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const uint32_t ix = (uint32_t)(srm_bits(x) >> 32) & 0x7fffffff;
  if (ix <= 0x3fe921fb) { /* |x| ~<= pi/4 */
    *y0 = x;
    *y1 = 0.0;
    return 0;
  }
  if (ix >= 0x413921fb) return srm_rem_pio2_large(x, y0, y1);
  const double fn = srm_rint(x * invpio2);
  const int n = (int)fn;
  double r = x - fn * pio2_1;
  double w = fn * pio2_1t;
  const int j = (int)(ix >> 20);
  double yy = r - w;
  int i = j - (int)((srm_bits(yy) >> 52) & 0x7ff);
  if (i > 16) { /* 2nd round, good to 118 bits */
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    yy = r - w;
    i = j - (int)((srm_bits(yy) >> 52) & 0x7ff);
    if (i > 49) { /* 3rd round, good to 151 bits */
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      yy = r - w;
    }
  }
  *y0 = yy;
  *y1 = (r - yy) - w;
  return n;
}

SRM_FN double srm_cos(double x) {
  if (!(x - x == 0.0)) return srm_nan(); /* Inf or NaN */
  double y0, y1;
  const int n = srm_rem_pio2(x, &y0, &y1);
  const double c = srm_kcos(y0, y1), s = srm_ksin(y0, y1);
  switch (n & 3) {
    case 0: return c;
    case 1: return -s;
    case 2: return -c;
    default: return s;
  }
}
SRM_FN double srm_sin(double x) {
  if (!(x - x == 0.0)) return srm_nan();
  double y0, y1;
  const int n = srm_rem_pio2(x, &y0, &y1);
  const double c = srm_kcos(y0, y1), s = srm_ksin(y0, y1);
  switch (n & 3) {
    case 0: return s;
    case 1: return c;
    case 2: return -s;
    default: return -c;
  }
}
/* sin and cos over one shared reduction: the same two values srm_sin and srm_cos return (the
 * constant-gradient kernels need both for a cos or sin node) */
SRM_FN void srm_sincos(double x, double* sn, double* cs) {
  if (!(x - x == 0.0)) {
    *sn = *cs = srm_nan();
    return;
  }
  double y0, y1;
  const int n = srm_rem_pio2(x, &y0, &y1);
  const double c = srm_kcos(y0, y1), s = srm_ksin(y0, y1);
  switch (n & 3) {
    case 0: *sn = s; *cs = c; break;
    case 1: *sn = c; *cs = -s; break;
    case 2: *sn = -s; *cs = -c; break;
    default: *sn = -c; *cs = s; break;
  }
}
/* tan = sin/cos over one shared reduction (<= ~1.5 ULP; fdlibm's k_tan is not restated) */
SRM_FN double srm_tan(double x) {
  if (!(x - x == 0.0)) return srm_nan();
  double y0, y1;
  const int n = srm_rem_pio2(x, &y0, &y1);
  const double c = srm_kcos(y0, y1), s = srm_ksin(y0, y1);
  return (n & 1) ? -c / s : s / c;
}

/* ---- Float32 ---------------------------------------------------------------------------------
 * Float32 sin / cos / tan / log evaluate in Float64 and round once (as Julia Base does for Float32
 * trigonometry: Float64 kernels, one rounding), so results are correctly rounded except when the
 * Float64 value lies within the kernel's error (2^-35 sin/cos, 2^-34 tan) of a rounding boundary.
 *   sinf/cosf, |x| < 2^28 pi/2: x = k pi + y with k an integer (sin) or half-integer (cos),
 *     pi as a double pair and two fmas, |y| <= pi/2; then sin y = y P(y^2) with one degree-5
 *     polynomial (relative error < 2^-35) and the sign of (-1)^k.  One polynomial and no quadrant
 *     select: a SIMD lane pays for every branch of a per-row case analysis.
 *   tanf, and sinf/cosf for |x| >= 2^28 pi/2: the FreeBSD s_tanf.c / s_cosf.c scheme (reduction to
 *     [-pi/4, pi/4] by quadrant, Payne-Hanek when large, the degree-4 __kernel_cosdf/sindf
 *     polynomials, |error| < 2^-34).
 *   expf: Julia's own Float32 algorithm (srm_expf below), not a widened one.
 *   logf: srm_log on the widened value (exact: every float is a normal double). */
/* __kernel_cosdf / __kernel_sindf coefficients (FreeBSD k_cosf.c / k_sinf.c, |error| < 2^-34 on
 * [-pi/4, pi/4]), evaluated by fma Horner as cos y = Q_C(z), sin y = y Q_S(z), z = y^2,
 * Q_K(z) = 1 + K0 z + K1 z^2 + K2 z^3 + K3 z^4.  Both polynomials are evaluated and the quadrant
 * selects one: a SIMD lane would otherwise pay a per-row select for every coefficient. */
SRM_FN double srm_qcos(double z) {
  return srm_fma(z, srm_fma(z, srm_fma(z, srm_fma(z, 2.439044879627741e-05, -0.001388676377460993),
                                       0.04166662332373906), -0.499999997251031), 1.0);
}
SRM_FN double srm_qsin(double z) {
  return srm_fma(z, srm_fma(z, srm_fma(z, srm_fma(z, 2.718311493989822e-06, -0.00019839334836096632),
                                       0.008333329385889463), -0.16666666641626524), 1.0);
}
/* Float32 trig in three shared pieces, so a batched caller (the device evaluates R rows per lane)
 * can run the fast reduction for every row and the Payne-Hanek path only when some row needs it,
 * and still produce bit-identical values:
 *   srm_rem_pio2f_fast: |x| < SRM_PIO2F_BIG (2^28 pi/2): n = rint(x 2/pi), y = x - n (pi/2) with
 *     pi/2 as a double pair and two fmas (each one rounding; |y| error < 2^-50 relative for every
 *     float x in range);
 *   srm_rem_pio2f_big: larger |x|, the shared Payne-Hanek;
 *   srm_trigf_finish: quadrant selection of the two polynomials and the one rounding to Float32. */
#define SRM_PIO2F_BIG 421657428.2663131
SRM_FN int srm_rem_pio2f_fast(double x, double* y) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_hi = 1.5707963267948966,
               pio2_lo = 6.123233995736766e-17;
  /* + 0.0: a -0 quotient becomes +0, so y = x - 0 (pi/2) keeps the sign of a zero x (tan(-0) = -0) */
  const double fn = srm_rint(x * invpio2) + 0.0;
  *y = srm_fma(-fn, pio2_lo, srm_fma(-fn, pio2_hi, x));
  return (int)fn;
}
SRM_FN int srm_rem_pio2f_big(double x, double* y) {
  double y0, y1;
  const int n = srm_rem_pio2_large(x, &y0, &y1);
  *y = y0;
  return n;
}
SRM_FN int srm_pio2f_is_big(double x) { return !(__builtin_fabs(x) < SRM_PIO2F_BIG); }
/* returns n (quadrant), *y the reduced argument; x finite */
SRM_FN int srm_rem_pio2f(float xf, double* y) {
  const double x = (double)xf;
  return srm_pio2f_is_big(x) ? srm_rem_pio2f_big(x, y) : srm_rem_pio2f_fast(x, y);
}
/* kind 0: cos, 1: sin, 2: tan of the reduced argument y in quadrant n */
SRM_FN float srm_trigf_finish(int kind, int n, double y) {
  const double z = y * y, c = srm_qcos(z), s = y * srm_qsin(z);
  if (kind == 2) return (float)((n & 1) ? -c / s : s / c);
  const int q = kind == 0 ? n + 1 : n;
  const double r = ((n & 1) ^ kind) ? s : c;
  return (float)((q & 2) ? -r : r);
}
/* sin y / y = P(y^2) on |y| <= pi/2 (+1e-4): degree-5 minimax on relative error, < 2^-35.3 (Remez,
 * regenerated in tests/test_math_accuracy.py) -- the accuracy class of Julia's own Float32 kernels
 * (FreeBSD __kernel_sindf < 2^-37.5, __kernel_cosdf < 2^-34.1).  A Float32 result differs from the
 * correctly rounded one only within ~2^-35 relative of a rounding boundary (< 0.1 % of arguments). */
SRM_FN double srm_psin(double z) {
  double p = -2.388876069481213e-08;
  p = srm_fma(p, z, 2.752537618509206e-06);
  p = srm_fma(p, z, -0.0001984086805341283);
  p = srm_fma(p, z, 0.00833333110744034);
  p = srm_fma(p, z, -0.16666666626122995);
  return srm_fma(p, z, 1.0);
}
SRM_FN uint32_t srm_bitsf(float x) { uint32_t u; __builtin_memcpy(&u, &x, 4); return u; }
SRM_FN float srm_from_bitsf(uint32_t u) { float x; __builtin_memcpy(&x, &u, 4); return x; }
/* kind 0: cos, 1: sin of a finite x with |x| < SRM_PIO2F_BIG.
 *   sin: k = rint(x/pi),       y = x - k pi, sin x = (-1)^k sin y
 *   cos: k = rint(x/pi - 1/2), y = x - (k + 1/2) pi, cos x = (-1)^(k+1) sin y */
SRM_FN float srm_sincosf_fast(int kind, double x) {
  const double invpi = 0.3183098861837907, pi_hi = 3.141592653589793, pi_lo = 1.2246467991473532e-16;
  double k = srm_rint(srm_fma(x, invpi, kind == 0 ? -0.5 : 0.0));
  const int m = (int)k;
  if (kind == 0) k += 0.5;
  const double y = srm_fma(-k, pi_lo, srm_fma(-k, pi_hi, x));
  const float r = (float)(y * srm_psin(y * y));
  return srm_from_bitsf(srm_bitsf(r) ^ ((uint32_t)(m + (kind == 0)) << 31));
}
SRM_FN float srm_trigf(int kind, float x) {
  if (!(x - x == 0.0f)) return x - x; /* Inf / NaN -> NaN */
  const double xd = (double)x;
  if (kind != 2 && !srm_pio2f_is_big(xd)) return srm_sincosf_fast(kind, xd);
  double y;
  const int n = srm_rem_pio2f(x, &y);
  return srm_trigf_finish(kind, n, y);
}
/* ---- Julia's own Float32 sin / cos (SRHIP_JULIA_TRIG builds; DESIGN.md 4 "Float32 trig") --------
 * Julia Base.Math evaluates sin(x::Float32) / cos(x::Float32) (base/special/trig.jl, rem_pio2.jl) as
 * FreeBSD msun's s_sinf.c / s_cosf.c do: |x| < Float32(pi)/4 -> the kernel of x itself (sin: x below
 * sqrt(eps(Float32)); cos: 1 below sqrt(eps(Float32)/2)); otherwise (n, y) = rem_pio2_kernel(x) in
 * Float64 -- n = +-1..+-4 with y = xd -+ k pi/2 (pi/2, pi, pi*3/2, pi*4/2 as Julia computes them in
 * Float64) for |x| <= 9pi/4, Cody-Waite with a 33 + 53-bit pi/2 below 2^28 pi/2, Payne-Hanek above --
 * and the quadrant n & 3 picks __kernel_sindf or __kernel_cosdf (k_sinf.c / k_cosf.c coefficients,
 * evaluated as written: no contraction), rounded once to Float32.  Restated from those published
 * sources; Julia cannot run here, so bits against Julia itself stay unpinned. */
#define SRM_JS1 (-0x15555554cbac77.0p-55)
#define SRM_JS2 0x111110896efbb2.0p-59
#define SRM_JS3 (-0x1a00f9e2cae774.0p-65)
#define SRM_JS4 0x16cd878c3b46a7.0p-71
#define SRM_JC0 (-0x1ffffffd0c5e81.0p-54)
#define SRM_JC1 0x155553e1053a42.0p-57
#define SRM_JC2 (-0x16c087e80f1e27.0p-62)
#define SRM_JC3 0x199342e0ee5069.0p-68
SRM_FN double srm_jsin_kernel(double y) {
  const double z = y * y, w = z * z, r = SRM_JS3 + z * SRM_JS4, s = z * y;
  return (y + s * (SRM_JS1 + z * SRM_JS2)) + s * w * r;
}
SRM_FN double srm_jcos_kernel(double y) {
  const double z = y * y, w = z * z, r = SRM_JC2 + z * SRM_JC3;
  return ((1.0 + z * SRM_JC0) + w * SRM_JC1) + (w * z) * r;
}
/* The same two polynomials at lower cost, with the same Float32 result (round 6).  Julia rounds its
 * Float64 kernel value once to Float32.  Horner's form with fused multiply-adds (srm_jsin_fma: z*y and
 * four fmas; srm_jcos_fma: four fmas -- against 10 and 9 operations in Julia's order) lands within a few
 * Float64 ulps of Julia's value, so both round to the same Float32 unless the fast value lies within
 * SRM_JTIE_K Float64 ulps of a Float32 rounding midpoint: the low 29 bits of its double -- the bits the
 * rounding drops -- within SRM_JTIE_K of 2^28 (srm_jtie).  The device evaluates the fast form, flags
 * such rows and re-evaluates a wave with a flagged row by Julia's own kernels; tools/check_trigf.c
 * proves on every float each tier may see that an unflagged fast value rounds to srm_jtrigf's bits.
 * (A value near a power of two cannot be near a midpoint in both binades: the test on the fast value
 * is exact there too, and the exhaustive check covers it.) */
#define SRM_JTIE_K 64u
SRM_FN double srm_jsin_fma(double y, double z) {
  const double p = srm_fma(z, srm_fma(z, srm_fma(z, SRM_JS4, SRM_JS3), SRM_JS2), SRM_JS1);
  return srm_fma(z * y, p, y);
}
SRM_FN double srm_jcos_fma(double z) {
  return srm_fma(z, srm_fma(z, srm_fma(z, srm_fma(z, SRM_JC3, SRM_JC2), SRM_JC1), SRM_JC0), 1.0);
}
SRM_FN int srm_jtie(double v) {
  /* low 29 bits within K of 2^28: shifted left by 3 (dropping the rest) the midpoint is 2^31, and
   * (lo << 3) + 2^31 + 8K wraps the window [2^31 - 8K, 2^31 + 8K] onto [0, 16K] -- one shift-add and
   * one compare on the device (v_lshl_add_u32) */
  return (uint32_t)(((uint32_t)srm_bits(v) << 3) + (0x80000000u + 8u * SRM_JTIE_K)) <= 16u * SRM_JTIE_K;
}
/* rem_pio2_kernel(x::Float32): n, y for |x| >= Float32(pi)/4, x finite */
SRM_FN int srm_jrem_pio2f(float x, double* y) {
  const double pi = 3.141592653589793;
  const double xd = (double)x, ax = __builtin_fabs(xd);
  if (ax <= pi * 5 / 4) {
    if (ax <= pi * 3 / 4) { *y = x > 0 ? xd - pi / 2 : xd + pi / 2; return x > 0 ? 1 : -1; }
    *y = x > 0 ? xd - pi : xd + pi;
    return x > 0 ? 2 : -2;
  }
  if (ax <= pi * 9 / 4) {
    if (ax <= pi * 7 / 4) { *y = x > 0 ? xd - pi * 3 / 2 : xd + pi * 3 / 2; return x > 0 ? 3 : -3; }
    *y = x > 0 ? xd - pi * 4 / 2 : xd + pi * 4 / 2;
    return x > 0 ? 4 : -4;
  }
  if (ax < 421657440.0) { /* Float32(pi)/2 * 2f0^28 */
    const double pio2_1 = 1.57079631090164184570e+00, pio2_1t = 1.58932547735281966916e-08,
                 inv_pio2 = 6.36619772367581382433e-01;
    const double fn = srm_rint(xd * inv_pio2);
    const double r = xd - fn * pio2_1, w = fn * pio2_1t;
    *y = r - w;
    return (int)fn;
  }
  return srm_rem_pio2f_big(xd, y);
}
/* The same function in the branch-free pieces the device runs per wave (srhip_eval_impl.h
 * jtrigf_rows), each proven equal to srm_jtrigf on every float it may see by tools/check_trigf.c:
 *   tier A, |x| < Float32(pi)/4 (SRM_JPIO4F): no reduction, ONE kernel of xd (sin: the sign of x
 *     copied onto the result -- the kernel returns |x| itself below sqrt(eps(Float32)), and +0 for -0);
 *   tier B, |x| <= pi*9/4 (SRM_J9PIO4F, the largest float below it): fn = rint(xd 2/pi) is Julia's
 *     region index n (0 below Float32(pi)/4, +-1..+-4 above), and fn * (pi/2) rounds to exactly the
 *     constant Julia subtracts (pi/2, pi, pi*3/2, pi*4/2: scaling by 2 commutes with the rounding),
 *     so y = xd - fn (pi/2) is Julia's y; both kernels, the quadrant selects (srm_jtrigf_q);
 *   tier C, |x| < 2^28 pi/2: per row Julia's own choice between that y and its Cody-Waite reduction
 *     (cos: Cody-Waite alone -- it returns the same bits as the +-k pi/2 cases on every float).
 * sin(-0) is the only row tier B / C would get wrong (y = +0): the caller keeps x where x == 0. */
#define SRM_JPIO4F 0.78539819f
#define SRM_J9PIO4F 7.068583f
#define SRM_JINV_PIO2 6.36619772367581382433e-01
#define SRM_JPIO2 1.5707963267948966
#define SRM_JPIO2_1 1.57079631090164184570e+00  /* first 25 bits of pi/2: fn * pio2_1 is exact */
#define SRM_JPIO2_1T 1.58932547735281966916e-08
SRM_FN double srm_jfn(double xd) { return srm_rint(xd * SRM_JINV_PIO2); }
SRM_FN double srm_jred_near(double xd, double fn) { return xd - fn * SRM_JPIO2; }
SRM_FN double srm_jred_cw(double xd, double fn) { return (xd - fn * SRM_JPIO2_1) - fn * SRM_JPIO2_1T; }
/* kind 0: cos, 1: sin of the reduced argument y in quadrant n: both kernels, one select and the sign */
SRM_FN float srm_jtrigf_q(int kind, int n, double y) {
  const float fs = (float)srm_jsin_kernel(y), fc = (float)srm_jcos_kernel(y);
  const float r = ((n & 1) ^ kind) ? fs : fc;
  return (((n + 1 - kind) >> 1) & 1) ? -r : r;
}
/* kind 0: cos, 1: sin (Inf / NaN -> NaN: Julia throws a DomainError for Inf, which the
 * evaluator never reaches -- a non-finite operand fails the tree first) */
SRM_FN float srm_jtrigf(int kind, float x) {
  if (!(x - x == 0.0f)) return x - x;
  const float ax = __builtin_fabsf(x);
  if (ax < 0.78539819f) { /* Float32(pi)/4 */
    if (kind == 1) return ax < 3.4526698e-4f ? x : (float)srm_jsin_kernel((double)x); /* sqrt(eps(Float32)) */
    return ax < 2.44140625e-4f ? 1.0f : (float)srm_jcos_kernel((double)x);             /* sqrt(eps(Float32)/2) */
  }
  double y;
  const int n = srm_jrem_pio2f(x, &y) & 3;
  const int q = kind == 0 ? n : (n + 3) & 3; /* sin in quadrant n = cos in quadrant n - 1 */
  if (q == 0) return (float)srm_jcos_kernel(y);
  if (q == 1) return (float)-srm_jsin_kernel(y);
  if (q == 2) return (float)-srm_jcos_kernel(y);
  return (float)srm_jsin_kernel(y);
}
/* Julia's kernels are the default (round 5: the minimax moved C2 losses by up to 1.6e-6 relative
 * against them, oracle/libm_sensitivity.py); -DSRHIP_JULIA_TRIG=0 builds the minimax form */
#ifndef SRHIP_JULIA_TRIG
#define SRHIP_JULIA_TRIG 1
#endif
#if SRHIP_JULIA_TRIG
SRM_FN float srm_cosf(float x) { return srm_jtrigf(0, x); }
SRM_FN float srm_sinf(float x) { return srm_jtrigf(1, x); }
#else
SRM_FN float srm_cosf(float x) { return srm_trigf(0, x); }
SRM_FN float srm_sinf(float x) { return srm_trigf(1, x); }
#endif
SRM_FN float srm_tanf(float x) { return srm_trigf(2, x); }
/* Float32 exp: Julia Base.Math exp_impl(x::Float32, Val(:e)) (base/special/exp.jl, Julia >= 1.7), a
 * Float32 algorithm (unlike Float32 sin / cos, which Julia evaluates in Float64): N = round(x log2 e)
 * in Float32, r = x - N ln2 with -ln2 split into two Float32 parts (two fmas: Julia's muladd on FMA
 * hardware), e^r by Julia's degree-6 Float32 minimax polynomial (evalpoly = Horner with muladd), and
 * p 2^N with one rounding (Julia's subnormal / N = 128 rescalings are that same single rounding);
 * x > 88.72284 -> Inf, x < -103.97208 -> 0.  Max error 1 ULP (tests/test_math_accuracy.py; every
 * Float32 input is checked by tools/check_expf.c).  The device runs the same operations two rows per
 * packed instruction (srhip_eval_impl.h expf2_dev), proven bit-identical by the same exhaustive check. */
#define SRM_EXPF_LOG2E 1.442695f
#define SRM_EXPF_NLN2_HI (-0.6931472f)
#define SRM_EXPF_NLN2_LO 1.9046542e-9f
#define SRM_EXPF_C6 0.0013956056f
#define SRM_EXPF_C5 0.008375129f
#define SRM_EXPF_C4 0.041666083f
#define SRM_EXPF_C3 0.16666415f
SRM_FN float srm_fmaf(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
SRM_FN float srm_expf(float x) {
  if (!(x == x)) return x + x;
  if (x > 88.72284f) return __builtin_inff();
  if (x < -103.97208f) return 0.0f;
  const float n = __builtin_rintf(x * SRM_EXPF_LOG2E);
  float r = srm_fmaf(n, SRM_EXPF_NLN2_HI, x);
  r = srm_fmaf(n, SRM_EXPF_NLN2_LO, r);
  float p = SRM_EXPF_C6;
  p = srm_fmaf(r, p, SRM_EXPF_C5);
  p = srm_fmaf(r, p, SRM_EXPF_C4);
  p = srm_fmaf(r, p, SRM_EXPF_C3);
  p = srm_fmaf(r, p, 0.5f);
  p = srm_fmaf(r, p, 1.0f);
  p = srm_fmaf(r, p, 1.0f);
  return __builtin_ldexpf(p, (int)n);
}
SRM_FN float srm_logf(float x) { return (float)srm_log((double)x); }

#endif /* SRHIP_MATH_H */
