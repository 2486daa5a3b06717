/* div_by_S (csrc/pf_kernels.hpp) against IEEE division: fl(a / b) from y = fl(1 / b), q0 = fl(a y) and two fma
   corrections.  Cases: quotients in [0, 1] over wide exponent ranges, decimal-like numerators, sums on the 2^-21
   grid of fp32 scores (the k_resample case), and numerators just below b.  Exit status 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t xr(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}
static double ud(void) { return (double)(xr() >> 11) * 0x1p-53; }
static double div_by_s(double a, double b, double y) {
  const double q0 = a * y;
  const double r0 = fma(-b, q0, a);
  const double q1 = fma(r0, y, q0);
  const double r1 = fma(-b, q1, a);
  return fma(r1, y, q1);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 10000000;
  long bad = 0;
  for (long i = 0; i < n; i++) {
    double a, b;
    switch (i % 4) {
      case 0: b = ldexp(1.0 + ud(), (int)(xr() % 400) - 200); a = b * ud(); break;
      case 1: b = ldexp(1.0 + ud(), (int)(xr() % 60)); a = floor(b * ud() * 1e6) / 1e6; break;
      case 2: {
        b = (double)(xr() % (1ull << 40) + 1) * 0x1p-21;
        a = (double)(xr() % (1ull << 40)) * 0x1p-21;
        if (a > b) a = b;
        break;
      }
      default:
        b = ldexp(1.0, (int)(xr() % 40)) * (1.0 + (double)(xr() % 16) * 0x1p-52);
        a = b * (1.0 - ldexp(1.0, -(int)(xr() % 53)));
        break;
    }
    const double y = 1.0 / b, q = a / b, m = div_by_s(a, b, y);
    if (memcmp(&q, &m, sizeof q) != 0) {
      if (bad < 10) printf("mismatch a=%a b=%a ieee=%a div_by_s=%a\n", a, b, q, m);
      bad++;
    }
  }
  printf("%ld cases, %ld mismatches\n", n, bad);
  return bad != 0;
}
