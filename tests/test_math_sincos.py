"""srm_sincos (include/srhip_math.h): the constant-gradient kernels take a cos or sin node's value
and derivative from one shared Float64 reduction; both must be the bits srm_sin and srm_cos return
(the evaluator's values), for ordinary, huge (Payne-Hanek), tiny and non-finite arguments."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r"""
#include <stdio.h>
#include <string.h>
#include <math.h>
#include "srhip_math.h"
static unsigned long long s = 88172645463325252ULL;
static unsigned long long nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static int same(double a, double b) { return memcmp(&a, &b, 8) == 0 || (a != a && b != b); }
int main(void) {
  long bad = 0, n = 0;
  const double fixed[] = {0.0, -0.0, 0.5, -0.7853981633974483, 1.5707963267948966, 3.141592653589793,
                          1e6, -1e22, 1.7976931348623157e308, 5e-324, INFINITY, -INFINITY, NAN};
  for (int i = 0; i < 2000000 + (int)(sizeof(fixed) / 8); ++i) {
    double x;
    if (i < (int)(sizeof(fixed) / 8)) x = fixed[i];
    else {
      const unsigned long long r = nxt();
      const int kind = (int)(r & 3);
      const double u = (double)(r >> 11) * 0x1p-53;
      x = kind == 0 ? (u - 0.5) * 20.0 : kind == 1 ? (u - 0.5) * 1e7 : kind == 2 ? ldexp(u - 0.5, (int)(r % 1000) - 20) : (u - 0.5) * 4.0;
    }
    double sn, cs;
    srm_sincos(x, &sn, &cs);
    ++n;
    if (!same(sn, srm_sin(x)) || !same(cs, srm_cos(x))) {
      if (bad < 5) printf("mismatch x=%a sin %a/%a cos %a/%a\n", x, sn, srm_sin(x), cs, srm_cos(x));
      ++bad;
    }
  }
  printf("%s %ld %ld\n", bad ? "BAD" : "OK", n, bad);
  return bad != 0;
}
"""


def test_sincos_equals_sin_and_cos_bitwise():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        with open(src, "w") as f:
            f.write(PROG)
        try:
            subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                            "-lm"], check=True, capture_output=True)
        except FileNotFoundError:
            pytest.skip("gcc not available")
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout
