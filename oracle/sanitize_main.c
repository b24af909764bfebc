/*
 * sanitize_main.c -- drives every routine of the CPU oracle (sph_oracle.c) on small
 * systems under AddressSanitizer + UndefinedBehaviorSanitizer (TEST INFRASTRUCTURE ONLY;
 * tests/test_oracle_sanitize.py builds it with -fsanitize=address,undefined and runs it).
 *
 * The systems: a jittered 3-D lattice with two types (C2/C3 shapes: rhosum, taitwater,
 * morris, heatconduction, the integrators), a 2-D one, and the bubble_growth slab (the
 * multiphase styles, the colour gradient, surface tension, fix phase_change through
 * orc_pre_exchange_ref over CommBrick's swaps).  Besides memory/UB errors it checks what
 * the reference guarantees: finite results, momentum conservation of the Newton-3 pair
 * forces after reverse comm, positive masses after phase change and atoms actually
 * inserted.  Exit status 0 = clean.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sph_oracle.h"

static int fails = 0;
#define CHECK(c, ...)                                                     \
  do {                                                                    \
    if (!(c)) {                                                           \
      fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__);        \
      fprintf(stderr, __VA_ARGS__);                                       \
      fprintf(stderr, "\n");                                              \
      fails++;                                                            \
    }                                                                     \
  } while (0)

static unsigned long long rng_state = 0x9E3779B97F4A7C15ull;
static double urand(void) { /* xorshift64*, [0,1) */
  rng_state ^= rng_state >> 12;
  rng_state ^= rng_state << 25;
  rng_state ^= rng_state >> 27;
  return (double)((rng_state * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}

static void *xcalloc(size_t n, size_t sz) {
  void *p = calloc(n ? n : 1, sz);
  if (!p) {
    fprintf(stderr, "out of memory\n");
    exit(2);
  }
  return p;
}

static int all_finite(const double *a, long n) {
  for (long i = 0; i < n; i++)
    if (!isfinite(a[i])) return 0;
  return 1;
}

/* lattice n^dim (dx 1), jitter 0.1, types 1/2 alternating by a hash when nt == 2 */
static int lattice(int dim, int n, int nt, int nmax, double *x, int *type) {
  int k = 0;
  for (int iz = 0; iz < (dim == 3 ? n : 1); iz++)
    for (int iy = 0; iy < n; iy++)
      for (int ix = 0; ix < n; ix++) {
        if (k >= nmax) return k;
        x[3 * k] = ix + 0.5 + 0.2 * (urand() - 0.5);
        x[3 * k + 1] = iy + 0.5 + 0.2 * (urand() - 0.5);
        x[3 * k + 2] = dim == 3 ? iz + 0.5 + 0.2 * (urand() - 0.5) : 0.0;
        type[k] = nt == 2 ? 1 + ((ix * 7 + iy * 3 + iz) % 2) : 1;
        k++;
      }
  return k;
}

static void single_phase(int dim, int n, int nt) {
  const double h = dim == 3 ? 3.0 : 2.5, skin = 0.3;
  orc_domain d = {dim, {0, 0, 0}, {n, n, dim == 3 ? n : 1.0}, {1, 1, dim == 3 ? 1 : 0}};
  const int nlocal0 = dim == 3 ? n * n * n : n * n, nmax = 8 * nlocal0;
  double *x = xcalloc(3 * (size_t)nmax, sizeof(double));
  int *type = xcalloc(nmax, sizeof(int));
  const int nlocal = lattice(dim, n, nt, nmax, x, type);
  const int n1 = nt + 1;
  double cut[9], cutsq[9], cns[9], mass[3] = {0, 1.0, 0.5}, rho0[3] = {0, 1.0, 0.5};
  double c0[3] = {0, 10.0, 10.0}, B[3], visc[9], alpha[9], cmax;
  for (int i = 0; i < n1 * n1; i++) {
    cut[i] = h;
    cutsq[i] = h * h;
    visc[i] = 0.1;
    alpha[i] = 0.1;
  }
  for (int t = 0; t < n1; t++) B[t] = c0[t] * c0[t] * rho0[t] / 7.0;
  orc_cutneighsq(nt, cut, skin, cns, &cmax);
  orc_pbc(&d, nlocal, x);
  int *gown = xcalloc(nmax, sizeof(int)), *gimg = xcalloc(3 * (size_t)nmax, sizeof(int));
  const int ng = orc_borders(&d, cmax, nlocal, x, type, nmax, gown, gimg);
  CHECK(ng > 0, "borders: %d ghosts", ng);
  if (ng <= 0) return;
  const int nall = nlocal + ng;
  long *foff = xcalloc(nlocal + 1, sizeof(long)), *hoff = xcalloc(nlocal + 1, sizeof(long));
  const long nf = orc_neigh_full(dim, nlocal, nall, x, type, nt, cns, foff, NULL, 0);
  int *fnb = xcalloc(nf, sizeof(int)), *hnb = xcalloc(nf, sizeof(int));
  CHECK(orc_neigh_full(dim, nlocal, nall, x, type, nt, cns, foff, fnb, nf) == nf, "full list");
  const long nh = orc_neigh_half_from_full(nlocal, x, foff, fnb, hoff, hnb);
  CHECK(nh > 0 && 2 * nh >= nf - nlocal && nh <= nf, "half list %ld of %ld", nh, nf);

  double *rho = xcalloc(nall, sizeof(double)), *e = xcalloc(nall, sizeof(double));
  double *v = xcalloc(3 * (size_t)nall, sizeof(double)), *vest = xcalloc(3 * (size_t)nall, sizeof(double));
  for (int i = 0; i < nlocal; i++) {
    e[i] = 1.0 + 0.1 * urand();
    for (int k = 0; k < dim; k++) v[3 * i + k] = 0.01 * (urand() - 0.5);
  }
  orc_meso_setup(nlocal, v, vest);
  orc_rhosum(dim, nlocal, x, type, nt, mass, cut, cutsq, foff, fnb, rho);
  CHECK(all_finite(rho, nlocal), "rhosum finite");
  orc_forward_comm(&d, nlocal, ng, gown, gimg, x, rho, e, vest);
  double *f = xcalloc(3 * (size_t)nall, sizeof(double)), *drho = xcalloc(nall, sizeof(double));
  double *de = xcalloc(nall, sizeof(double)), vir[6] = {0};
  for (int variant = 0; variant < 2; variant++) {
    memset(f, 0, 3 * (size_t)nall * sizeof(double));
    memset(drho, 0, nall * sizeof(double));
    memset(de, 0, nall * sizeof(double));
    if (variant == 0)
      orc_taitwater(dim, nlocal, 1, x, vest, rho, type, nt, mass, rho0, c0, B, visc, cut, cutsq,
                    hoff, hnb, f, drho, de, vir);
    else
      orc_taitwater_morris(dim, nlocal, 1, x, vest, rho, type, nt, mass, rho0, c0, B, visc, cut,
                           cutsq, hoff, hnb, f, drho, de, vir);
    orc_heatconduction(dim, nlocal, 1, x, e, rho, type, nt, mass, alpha, cut, cutsq, hoff, hnb, de);
    orc_reverse_comm(nlocal, ng, gown, f, drho, de);
    CHECK(all_finite(f, 3 * (long)nlocal) && all_finite(de, nlocal) && all_finite(drho, nlocal),
          "forces finite");
    double sf[3] = {0, 0, 0}, af = 0;
    for (int i = 0; i < nlocal; i++)
      for (int k = 0; k < 3; k++) {
        sf[k] += f[3 * i + k];
        af += fabs(f[3 * i + k]);
      }
    for (int k = 0; k < 3; k++)
      CHECK(fabs(sf[k]) <= 1e-10 * (af + 1e-300), "momentum %d: %g of %g", k, sf[k], af);
  }
  orc_meso_initial(nlocal, 1e-3, 5e-4, type, mass, NULL, x, v, f, vest, rho, drho, e, de);
  orc_meso_final(nlocal, 5e-4, type, mass, NULL, v, f, rho, drho, e, de);
  orc_meso_stationary(nlocal, 5e-4, type, 1 << 2, rho, drho, e, de);
  const double acc[3] = {0, -9.81, 0};
  orc_gravity(nlocal, type, 1 << 1, mass, NULL, acc, f);
  CHECK(all_finite(x, 3 * (long)nlocal) && all_finite(rho, nlocal), "integrated finite");
  free(x), free(type), free(gown), free(gimg), free(foff), free(hoff), free(fnb), free(hnb);
  free(rho), free(e), free(v), free(vest), free(f), free(drho), free(de);
}

/* the bubble_growth slab (tests/scenarios.py bubble_system(nx, slab=True)) */
static void multiphase(int dim, int nx) {
  const double dx = 1.0 / nx, h = 3.0 * dx;
  orc_domain d = {dim, {0, 0, 0}, {1, 1, dim == 3 ? 1.0 : dx}, {1, 1, dim == 3 ? 1 : 0}};
  const int nlocal0 = dim == 3 ? nx * nx * nx : nx * nx, nmax = 10 * nlocal0;
  double *x = xcalloc(3 * (size_t)nmax, sizeof(double));
  int *type = xcalloc(nmax, sizeof(int));
  int nlocal = 0;
  for (int iz = 0; iz < (dim == 3 ? nx : 1); iz++)
    for (int iy = 0; iy < nx; iy++)
      for (int ix = 0; ix < nx; ix++) {
        double *p = x + 3 * nlocal;
        p[0] = (ix + 0.5 + 0.2 * (urand() - 0.5)) * dx;
        p[1] = (iy + 0.5 + 0.2 * (urand() - 0.5)) * dx;
        p[2] = dim == 3 ? (iz + 0.5 + 0.2 * (urand() - 0.5)) * dx : 0.0;
        type[nlocal++] = p[0] > 1.0 - dx ? 2 : 1;
      }
  const int nt = 2, n1 = 3;
  double cut[9], cutsq[9], cns[9], cmax, rho0[3] = {0, 1.0, 0.1}, c0[3], B[3], gam[3] = {0, 1, 1};
  double rbg[3] = {0, 0, 0}, visc[9], alpha[9], cga[9], tc[9] = {0};
  int ff[9] = {0};
  ff[1 * 3 + 2] = 2;
  for (int i = 0; i < 9; i++) {
    cut[i] = h;
    cutsq[i] = h * h;
    visc[i] = 0.8;
    alpha[i] = 0.3;
    cga[i] = 0.0;
  }
  cga[1 * 3 + 2] = cga[2 * 3 + 1] = 500.0;
  for (int t = 1; t < n1; t++) {
    c0[t] = 200.0 / sqrt(rho0[t]);
    B[t] = c0[t] * c0[t] * rho0[t] / gam[t];
  }
  c0[0] = B[0] = 0.0;
  orc_cutneighsq(nt, cut, 0.0, cns, &cmax);
  orc_pbc(&d, nlocal, x);
  int *gown = xcalloc(nmax, sizeof(int)), *gimg = xcalloc(3 * (size_t)nmax, sizeof(int));
  int *gsrc = xcalloc(nmax, sizeof(int)), swf[64], nswap = 0;
  const int ng = orc_borders_ex(&d, cmax, nlocal, x, type, nmax, gown, gimg, gsrc, swf, &nswap);
  CHECK(ng > 0 && nswap > 0, "borders_ex: %d ghosts %d swaps", ng, nswap);
  if (ng <= 0) return;
  const int nall = nlocal + ng;
  long *foff = xcalloc(nlocal + 1, sizeof(long)), *hoff = xcalloc(nlocal + 1, sizeof(long));
  const long nf = orc_neigh_full(dim, nlocal, nall, x, type, nt, cns, foff, NULL, 0);
  int *fnb = xcalloc(nf, sizeof(int)), *hnb = xcalloc(nf, sizeof(int));
  orc_neigh_full(dim, nlocal, nall, x, type, nt, cns, foff, fnb, nf);
  orc_neigh_half_from_full(nlocal, x, foff, fnb, hoff, hnb);
  double *rho = xcalloc(nmax, sizeof(double)), *rm = xcalloc(nmax, sizeof(double));
  double *e = xcalloc(nmax, sizeof(double)), *cv = xcalloc(nmax, sizeof(double));
  double *v = xcalloc(3 * (size_t)nmax, sizeof(double)), *vest = xcalloc(3 * (size_t)nmax, sizeof(double));
  double *cg = xcalloc(3 * (size_t)nmax, sizeof(double)), *f = xcalloc(3 * (size_t)nmax, sizeof(double));
  double *de = xcalloc(nmax, sizeof(double)), *dm = xcalloc(nmax, sizeof(double));
  for (int i = 0; i < nall; i++) {
    const int o = i < nlocal ? i : gown[i - nlocal];
    const int t = type[o];
    rho[i] = t == 2 ? 0.1 : 1.0;
    rm[i] = rho[i] * pow(dx, dim);
    cv[i] = t == 2 ? 0.06 : 0.04;
    e[i] = t == 2 ? 0.0 : 0.04 * 1.2;
  }
  orc_rhosum_multiphase(dim, nlocal, x, type, nt, rm, cut, cutsq, foff, fnb, rho);
  orc_colorgradient(dim, nlocal, x, rho, rm, type, nt, cga, cut, cutsq, foff, fnb, cg);
  CHECK(all_finite(rho, nlocal) && all_finite(cg, 3 * (long)nlocal), "rho/cg finite");
  orc_taitwater_multiphase(dim, nlocal, 1, x, vest, rho, type, nt, rm, rho0, c0, B, gam, rbg,
                           visc, cut, cutsq, hoff, hnb, f);
  orc_surfacetension(dim, nlocal, 1, x, rho, rm, type, nt, cg, cut, cutsq, hoff, hnb, f);
  orc_heatconduction_phasechange(dim, nlocal, 1, x, e, cv, rho, rm, type, nt, alpha, ff, tc, cut,
                                 cutsq, hoff, hnb, de);
  CHECK(all_finite(f, 3 * (long)nall) && all_finite(de, nall), "multiphase forces finite");
  for (int k = 0; k < 6; k++) {
    const double r = (k + 0.5) / 6.0;
    CHECK(isfinite(orc_kernel_quintic2d(r)) && isfinite(orc_kernel_quintic3d(r)) &&
              isfinite(orc_dw_quintic2d(r)) && isfinite(orc_dw_quintic3d(r)), "quintic");
  }
  orc_pc_params p;
  memset(&p, 0, sizeof(p));
  p.dim = dim;
  p.Tc = 0.0;
  p.Tt = -1.0;
  p.Hwv = 8.0;
  p.dr = 0.5 * dx;
  p.to_mass = pow(dx, dim) * 0.1;
  p.cutoff = h;
  p.from_type = 1;
  p.to_type = 2;
  p.change_chance = 0.3;
  p.dt = 1e-6;
  p.maxattempt = 10;
  for (int k = 0; k < 3; k++) {
    p.sublo[k] = d.boxlo[k];
    p.subhi[k] = d.boxhi[k];
    p.boxhi[k] = d.boxhi[k];
    p.top[k] = 1;
  }
  int seed = 123456;
  const int nnew = orc_pre_exchange_ref(&p, &seed, nlocal, ng, nmax, x, v, vest, cg, e, rm, rho,
                                        cv, type, foff, fnb, nswap, swf, gsrc, dm);
  CHECK(nnew > nlocal, "pre_exchange_ref: %d (nlocal %d): nothing inserted", nnew, nlocal);
  printf("multiphase %dD nx %d: %d ghosts, %ld full entries, %d atoms inserted\n", dim, nx, ng,
         nf, nnew - nlocal);
  if (nnew >= nlocal) {
    CHECK(all_finite(rm, nnew) && all_finite(e, nnew) && all_finite(x, 3 * (long)nnew),
          "phase change finite");
    for (int i = 0; i < nnew; i++) CHECK(rm[i] > 0.0, "rmass[%d] = %g", i, rm[i]);
  }
  /* the candidate-list form (orc_phasechange + orc_phasechange_finish) */
  double *rec = xcalloc(13 * (size_t)nlocal, sizeof(double));
  int *par = xcalloc(nlocal, sizeof(int));
  memset(dm, 0, nmax * sizeof(double));
  seed = 123456;
  const int ni = orc_phasechange(&p, &seed, nlocal, nall, x, v, vest, cg, e, rm, rho, cv, type,
                                 foff, fnb, dm, nlocal, rec, par);
  CHECK(ni >= 0 && ni <= nlocal, "phasechange: %d", ni);
  orc_phasechange_finish(nlocal, dm, rm, e);
  double u = 0.0;
  int s2 = 7;
  for (int k = 0; k < 1000; k++) u += orc_park_uniform(&s2);
  CHECK(u > 400 && u < 600, "RanPark mean %g", u / 1000);
  free(x), free(type), free(gown), free(gimg), free(gsrc), free(foff), free(hoff), free(fnb);
  free(hnb), free(rho), free(rm), free(e), free(cv), free(v), free(vest), free(cg), free(f);
  free(de), free(dm), free(rec), free(par);
}

int main(void) {
  single_phase(3, 7, 1);
  single_phase(3, 8, 2);
  single_phase(2, 14, 1);
  multiphase(3, 8);
  multiphase(2, 12);
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("sanitize_main: all oracle routines clean\n");
  return 0;
}
