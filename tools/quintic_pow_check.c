/* tools/quintic_pow_check.c -- how often the engine's reference-form quintic spline
 * (csrc/sph_mp_kernels.h qr_*: correctly rounded powers from double-double products, the
 * expanded polynomials evaluated left to right without contraction) differs from the
 * reference's own sph_kernel_quintic.cpp arithmetic (glibc pow), over s in [0, 3).
 * Also: how often glibc's pow(x, n) is not the correctly rounded power (__float128 check).
 *   gcc -O2 -ffp-contract=off tools/quintic_pow_check.c -o /tmp/qpc -lm -lquadmath && /tmp/qpc 20000000
 * (measurement helper, not part of the product) */
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

/* the engine's forms (same operations as the device code) */
static double qr_pow3(double x) { double h = x * x, l = fma(x, x, -h); double p = x * h, e = fma(x, h, -p); return p + fma(x, l, e); }
static void qr_pow4dd(double x, double *q, double *t) { double h = x * x, l = fma(x, x, -h); *q = h * h; *t = fma(2.0 * h, l, fma(h, h, -*q)); }
static double qr_pow4(double x) { double q, t; qr_pow4dd(x, &q, &t); return q + t; }
static double qr_pow5(double x) { double q, t; qr_pow4dd(x, &q, &t); double p = x * q, e = fma(x, q, -p); return p + fma(x, t, e); }
static double qr_wpoly(double s) {
  double a = s < 3.0 ? qr_pow5(3.0 - s) : 0.0, b = s < 2.0 ? qr_pow5(2.0 - s) : 0.0, c = s < 1.0 ? qr_pow5(1.0 - s) : 0.0;
  return (a - 6.0 * b) + 15.0 * c;
}
static double qr_dwpoly(double s) {
  int p1 = s < 1.0, p2 = s < 2.0, p3 = s < 3.0;
  double c4 = p1 ? -50.0 : p2 ? 25.0 : p3 ? -5.0 : 0.0, c3 = p1 ? 120.0 : p2 ? -180.0 : p3 ? 60.0 : 0.0;
  double c2 = p1 ? 0.0 : p2 ? 450.0 : p3 ? -270.0 : 0.0, c1 = p1 ? -120.0 : p2 ? -420.0 : p3 ? 540.0 : 0.0;
  double c0 = p1 ? 0.0 : p2 ? 75.0 : p3 ? -405.0 : 0.0;
  return (((c4 * qr_pow4(s) + c3 * qr_pow3(s)) + c2 * (s * s)) + c1 * s) + c0;
}
/* the reference's (sph_kernel_quintic.cpp:17-73, norm left out) */
static double ref_w(double s) {
  if (s < 1.0) return pow(3 - s, 5) - 6 * pow(2 - s, 5) + 15 * pow(1 - s, 5);
  if (s < 2.0) return pow(3 - s, 5) - 6 * pow(2 - s, 5);
  if (s < 3.0) return pow(3 - s, 5);
  return 0.0;
}
static double ref_dw(double s) {
  if (s < 1) return -50 * pow(s, 4) + 120 * pow(s, 3) - 120 * s;
  if (s < 2) return 25 * pow(s, 4) - 180 * pow(s, 3) + 450 * pow(s, 2) - 420 * s + 75;
  if (s < 3.0) return -5 * pow(s, 4) + 60 * pow(s, 3) - 270 * pow(s, 2) + 540 * s - 405;
  return 0.0;
}
int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 1000000;
  uint64_t z = 88172645463325252ull;
  long wdiff = 0, dwdiff = 0, gbad = 0, mbad = 0, calls = 0;
  double worst_dw = 0.0;
  for (long i = 0; i < n; i++) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    double s = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 3.0;
    if (i & 1) s = 3.0 - s * 1e-3;  /* half the samples near the cutoff (cancellation) */
    if (qr_wpoly(s) != ref_w(s)) wdiff++;
    double a = qr_dwpoly(s), b = ref_dw(s);
    if (a != b) {
      dwdiff++;
      double d = fabs(a - b);
      if (d > worst_dw) worst_dw = d;
    }
    for (int k = 3; k <= 5; k++) {
      double x = k == 5 ? 3.0 - s : s;
      __float128 X = x, E = X * X * X;
      if (k >= 4) E *= X;
      if (k == 5) E *= X;
      double ex = (double)E, g = pow(x, k), m = k == 3 ? qr_pow3(x) : k == 4 ? qr_pow4(x) : qr_pow5(x);
      calls++;
      if (g != ex) gbad++;
      if (m != ex) mbad++;
    }
  }
  printf("samples %ld: W differs %ld (%.4f %%), dW differs %ld (%.4f %%), worst |dW diff| %.3e (norm left out)\n",
         n, wdiff, 100.0 * wdiff / n, dwdiff, 100.0 * dwdiff / n, worst_dw);
  printf("powers %ld: glibc pow not correctly rounded %ld (%.4f %%), engine's not correctly rounded %ld\n", calls, gbad,
         100.0 * gbad / calls, mbad);
  return 0;
}
