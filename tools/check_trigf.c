/* Exhaustive proof and study for the device's Float32 sin / cos (include/srhip_math.h), over every
 * finite float with |x| < 2^28 pi/2 (the rest take the scalar path, srm_jtrigf itself):
 *
 *  (0) PROOF: the three per-wave tiers the device evaluates Julia's Float32 sin / cos in
 *      (srm_jfn / srm_jred_near / srm_jred_cw / srm_jtrigf_q) return srm_jtrigf's bits for every
 *      input each tier may see.  Exit status 1 otherwise.
 *  (0') PROOF (round 6): the same tiers with the kernels in Horner form (srm_jsin_fma / srm_jcos_fma)
 *      return srm_jtrigf's bits on every input whose fast value srm_jtie does not flag; prints how
 *      many each tier flags (the device re-evaluates those waves exactly).  The rest runs with an
 *      argument only:
 *
 *  (1) D = max distance, in Float64 units in the last place, between the value the fast degree-5
 *      minimax (srm_sincosf_fast) computes BEFORE its one rounding to Float32 and the value Julia's
 *      own kernels (srm_jtrigf: __kernel_sindf / __kernel_cosdf per quadrant after rem_pio2_kernel)
 *      compute before theirs.  Both round once, so they can round differently only when the minimax
 *      value lies within D of a Float32 rounding midpoint.
 *  (2) a rejected alternative, measured: certify the minimax per row (the low 29 bits of its double --
 *      the bits Float32 rounding drops -- farther than a threshold from the midpoint pattern 2^28
 *      means Float32(minimax) is Julia's value) and re-evaluate the rest with Julia's kernels.  The
 *      distance histogram's tail (Julia's 25+53-bit reduction near the zeros of large arguments)
 *      makes the re-evaluated share too large to pay.  `check_trigf <threshold>`
 *      prints D, the histogram, and the share a threshold flags.
 * Build: gcc -O2 -march=x86-64-v3 -ffp-contract=off -fopenmp tools/check_trigf.c -lm -o /tmp/check_trigf */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/srhip_math.h"

static float from_u(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t to_u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t to_u64(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

/* srm_sincosf_fast before the rounding (sign applied to the double: negation commutes with it) */
static double mm_double(int kind, double x) {
  const double invpi = 0.3183098861837907, pi_hi = 3.141592653589793, pi_lo = 1.2246467991473532e-16;
  double k = rint(fma(x, invpi, kind == 0 ? -0.5 : 0.0));
  const int m = (int)k;
  if (kind == 0) k += 0.5;
  const double y = fma(-k, pi_lo, fma(-k, pi_hi, x));
  const double v = y * srm_psin(y * y);
  return ((m + (kind == 0)) & 1) ? -v : v;
}
/* srm_jtrigf before the rounding */
static double jl_double(int kind, float x) {
  const float ax = fabsf(x);
  if (ax < 0.78539819f) {
    if (kind == 1) return ax < 3.4526698e-4f ? (double)x : srm_jsin_kernel((double)x);
    return ax < 2.44140625e-4f ? 1.0 : srm_jcos_kernel((double)x);
  }
  double y;
  const int n = srm_jrem_pio2f(x, &y) & 3;
  const int q = kind == 0 ? n : (n + 3) & 3;
  if (q == 0) return srm_jcos_kernel(y);
  if (q == 1) return -srm_jsin_kernel(y);
  if (q == 2) return -srm_jcos_kernel(y);
  return srm_jsin_kernel(y);
}

/* the device's tiers (srhip_eval_impl.h jtrigf_rows) as scalar functions of one row */
static float tier_a(int kind, float x) {
  const double xd = (double)x;
  if (kind == 0) return (float)srm_jcos_kernel(xd);
  const float r = (float)srm_jsin_kernel(xd);
  return copysignf(r, x); /* v_bfi_b32: the sign of x, the magnitude of r */
}
static float tier_b(int kind, float x) {
  const double xd = (double)x, fn = srm_jfn(xd);
  const float r = srm_jtrigf_q(kind, (int)fn, srm_jred_near(xd, fn));
  return (kind == 1 && x == 0.0f) ? x : r;
}
static float tier_c(int kind, float x) {
  const double xd = (double)x, fn = srm_jfn(xd);
  /* cos: Cody-Waite for every row (equal to the +-k pi/2 cases on every float); sin: Julia's choice */
  const double y = kind == 0 ? srm_jred_cw(xd, fn)
                             : (fabs(xd) <= 3.141592653589793 * 9 / 4 ? srm_jred_near(xd, fn) : srm_jred_cw(xd, fn));
  const float r = srm_jtrigf_q(kind, (int)fn, y);
  return (kind == 1 && x == 0.0f) ? x : r;
}

/* the device's fast tiers (round 6): Julia's reduction, the kernels in Horner form with fmas, a row
 * whose fast value lies near a Float32 rounding midpoint flagged (the device then re-evaluates the wave
 * by the exact tiers above) */
static float tier_a_fast(int kind, float x, int* flag) {
  const double xd = (double)x, z = xd * xd;
  const double p = kind == 0 ? srm_jcos_fma(z) : srm_jsin_fma(xd, z);
  *flag = srm_jtie(p);
  return kind == 0 ? (float)p : copysignf((float)p, x);
}
static float tier_bc_fast(int kind, float x, int cw, int* flag) {
  const double xd = (double)x, fn = srm_jfn(xd);
  double y = srm_jred_near(xd, fn);
  if (cw) y = kind == 0 ? srm_jred_cw(xd, fn) : (fabsf(x) <= SRM_J9PIO4F ? y : srm_jred_cw(xd, fn));
  const int n = (int)fn;
  const double z = y * y;
  const double p = ((n & 1) ^ kind) ? srm_jsin_fma(y, z) : srm_jcos_fma(z);
  *flag = srm_jtie(p);
  const float r = (float)p;
  const float q = (((n + 1 - kind) >> 1) & 1) ? -r : r;
  return (kind == 1 && x == 0.0f) ? x : q;
}

int main(int argc, char** argv) {
  const uint32_t cert = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : 0;
  /* (0) the tiers: every float each tier may see */
  for (int kind = 0; kind < 2; ++kind) {
    uint64_t na = 0, nb = 0, nc = 0, ba = 0, bb = 0, bc = 0;
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : na, nb, nc, ba, bb, bc)
    for (int64_t i = 0; i < (1LL << 32); ++i) {
      const float x = from_u((uint32_t)i);
      if (!(fabsf(x) < 421657440.0f)) continue;
      const uint32_t want = to_u(srm_jtrigf(kind, x));
      if (fabsf(x) < SRM_JPIO4F) { ++na; ba += to_u(tier_a(kind, x)) != want; }
      if (fabsf(x) <= SRM_J9PIO4F) { ++nb; bb += to_u(tier_b(kind, x)) != want; }
      ++nc;
      bc += to_u(tier_c(kind, x)) != want;
    }
    printf("%s tiers vs srm_jtrigf: A %llu inputs %llu wrong, B %llu inputs %llu wrong, C %llu inputs %llu wrong\n",
           kind ? "sin" : "cos", (unsigned long long)na, (unsigned long long)ba, (unsigned long long)nb,
           (unsigned long long)bb, (unsigned long long)nc, (unsigned long long)bc);
    fflush(stdout);
    if (ba || bb || bc) return 1;
  }
  /* (0') the fast tiers: an unflagged row returns srm_jtrigf's bits on every float the tier may see.
   * SRHIP_TIE_DUMP=<file>: also write every flagged input (uint32 bits, any tier / kind; sorted
   * ascending) -- the fixture tests/golden/trig_tie_inputs.npy, whose rows the GPU test drives through
   * the device's re-evaluation branch. */
  const char* dump = getenv("SRHIP_TIE_DUMP");
  FILE* df = dump && *dump ? fopen(dump, "wb") : NULL;
  if (df) {
    for (int64_t i = 0; i < (1LL << 32); ++i) {
      const float x = from_u((uint32_t)i);
      if (!(fabsf(x) < 421657440.0f)) continue;
      int f = 0, g;
      for (int kind = 0; kind < 2; ++kind) {
        if (fabsf(x) < SRM_JPIO4F) { (void)tier_a_fast(kind, x, &g); f |= g; }
        if (fabsf(x) <= SRM_J9PIO4F) { (void)tier_bc_fast(kind, x, 0, &g); f |= g; }
        (void)tier_bc_fast(kind, x, 1, &g);
        f |= g;
      }
      if (f) { const uint32_t u = (uint32_t)i; fwrite(&u, 4, 1, df); }
    }
    fclose(df);
  }
  for (int kind = 0; kind < 2; ++kind) {
    uint64_t na = 0, nb = 0, nc = 0, ba = 0, bb = 0, bc = 0, fa = 0, fb = 0, fc = 0;
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : na, nb, nc, ba, bb, bc, fa, fb, fc)
    for (int64_t i = 0; i < (1LL << 32); ++i) {
      const float x = from_u((uint32_t)i);
      if (!(fabsf(x) < 421657440.0f)) continue;
      const uint32_t want = to_u(srm_jtrigf(kind, x));
      int f;
      if (fabsf(x) < SRM_JPIO4F) {
        const uint32_t got = to_u(tier_a_fast(kind, x, &f));
        ++na; fa += f; ba += !f && got != want;
      }
      if (fabsf(x) <= SRM_J9PIO4F) {
        const uint32_t got = to_u(tier_bc_fast(kind, x, 0, &f));
        ++nb; fb += f; bb += !f && got != want;
      }
      const uint32_t got = to_u(tier_bc_fast(kind, x, 1, &f));
      ++nc; fc += f; bc += !f && got != want;
    }
    printf("%s fast tiers vs srm_jtrigf (flagged rows / unflagged wrong): A %llu inputs %llu / %llu, "
           "B %llu inputs %llu / %llu, C %llu inputs %llu / %llu\n",
           kind ? "sin" : "cos", (unsigned long long)na, (unsigned long long)fa, (unsigned long long)ba,
           (unsigned long long)nb, (unsigned long long)fb, (unsigned long long)bb, (unsigned long long)nc,
           (unsigned long long)fc, (unsigned long long)bc);
    fflush(stdout);
    if (ba || bb || bc) return 1;
  }
  if (argc < 2) return 0;
  for (int kind = 0; kind < 2; ++kind) {
    uint64_t dmax = 0, n = 0, differ = 0, flagged = 0, bad = 0, incons = 0;
    uint64_t hist[40] = {0};
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(max : dmax) reduction(+ : n, differ, flagged, bad, incons, hist[:40])
    for (int64_t i = 0; i < (1LL << 32); ++i) {
      const float x = from_u((uint32_t)i);
      if (!(fabsf(x) < 421657440.0f)) continue; /* non-finite / large: the scalar path */
      ++n;
      const double vm = mm_double(kind, (double)x), vj = jl_double(kind, x);
      const float fj = srm_jtrigf(kind, x);
      if (to_u((float)vj) != to_u(fj)) ++incons;
      const int64_t a = (int64_t)(to_u64(fabs(vm))), b = (int64_t)(to_u64(fabs(vj)));
      const uint64_t d = (signbit(vm) != signbit(vj) && vm != 0.0) ? UINT64_MAX / 2 : (uint64_t)(a > b ? a - b : b - a);
      if (d > dmax) dmax = d;
      int lg = 0;
      while (lg < 39 && (1ULL << lg) <= d) ++lg;
      hist[lg]++;
      if (to_u((float)vm) != to_u(fj)) ++differ;
      /* the certificate */
      const uint32_t low = (uint32_t)to_u64(vm) & 0x1FFFFFFFu;
      const uint32_t dist = low > 0x10000000u ? low - 0x10000000u : 0x10000000u - low;
      const int near = dist < cert;
      if (near) ++flagged;
      const float res = near ? fj : (float)vm;
      if (to_u(res) != to_u(fj)) ++bad;
    }
    printf("%s: inputs %llu, max |minimax - julia| before rounding %llu double ulps (log2 %.2f); "
           "Float32 results that differ %llu (%.4f %%); certificate %u: flagged %llu (%.4f %%), wrong after "
           "certification %llu; julia double/float inconsistencies %llu\n",
           kind ? "sin" : "cos", (unsigned long long)n, (unsigned long long)dmax, log2((double)dmax + 1),
           (unsigned long long)differ, 100.0 * differ / n, cert, (unsigned long long)flagged, 100.0 * flagged / n,
           (unsigned long long)bad, (unsigned long long)incons);
    printf("  log2 histogram of the distance:");
    for (int k = 0; k < 40; ++k)
      if (hist[k]) printf(" [%d]%llu", k, (unsigned long long)hist[k]);
    printf("\n");
    fflush(stdout);
    if (bad || incons) return 1;
  }
  return 0;
}
