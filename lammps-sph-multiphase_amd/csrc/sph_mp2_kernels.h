// sph_mp2_kernels.h -- the engine's multiphase passes (C5, bubble_growth stack), written for
// the issue rate: the row kernels of sph_mp_kernels.h spend ~300 VALU instructions per pair
// in the fused gather (profiles/r03: 543 M wave-instructions for 1M rows) on branchy quintic
// pieces, per-pair coefficient loads with lane-varying indices and the swaps that put each
// pair in its half-list orientation.  Here
//   * the quintic kernel and its derivative are the reference's own expanded polynomials
//     (sph_kernel_quintic.cpp:17-73) in its arithmetic -- rsq without contraction, IEEE
//     sqrt, s = 3 (r / h), correctly rounded powers, no contraction (sph_mp_kernels.h qr_*) --
//     branch-free (the pieces as selected coefficients); round 5's factored form sat up to
//     ~1e-13 absolute from the reference's dW where its polynomial cancels near the cutoff;
//   * the per-pair-type coefficients sit in LDS, loaded once per workgroup;
//   * when every style is symmetric under exchanging the pair's atoms (all gamma equal, so
//     the p_j-with-gamma[itype] quirk is moot, and no type pinned to its own type's Tc) a
//     pair is evaluated with i as the row atom whatever its half-list orientation: the
//     orientation then only selects the fresh or stale rho / colour gradient of each side
//     (k_mp_gather's comment); otherwise the engine keeps k_mp_gather;
//   * the surface stress S = (|c|^2/ndim e - (c.e) c)/|c| (pair_sph_surfacetension.cpp:
//     135-168, same vector, the reference's terms collected) reads w = c/sqrt(|c|) from the
//     records (|w|^2 = |c|, (w.e) w = (c.e) c/|c|): no square root or division per pair.
// The fields agree with the reference restatement to rounding (~1e-15 relative per pair);
// the parity bar of the C5 tests is 1e-10.
#pragma once
#include <hip/hip_runtime.h>

#include "sph_kernels.h"
#include "sph_mp_kernels.h"

namespace sph {

// list entries per lane whose loads are issued together (study builds: -DSPH_MP2_NU=n)
// (colorgradient at C5 4M, round 5: 1.362 vs 1.471 ms with 2; round 6, its terms in the
// reference's operation order: 4 -> 120 VGPRs = 4 waves, 2 -> 96 VGPRs = 5 waves, 1.406 vs
// 1.451 ms, profiles/r06/cg_nu/ -- the same entries per lane in the same order either way)
#ifndef SPH_MP2_NU
#define SPH_MP2_NU 2
#endif
// ... in the fused gather: one (its three records per entry; 128 VGPRs = 4 waves per SIMD
// with gamma = 1, against 156 = 3 waves with two: 4.36 vs 4.53 ms per C5 step,
// profiles/r04/c5)
#ifndef SPH_MP2_GNU
#define SPH_MP2_GNU 1
#endif
// ... or software-pipelined (records of the next entry loaded while this one is evaluated)
#ifndef SPH_MP2_PIPE
#define SPH_MP2_PIPE 0
#endif
// study builds: -DSPH_MP2_WPE=n asks the compiler for n waves per SIMD in the gather
#if defined(SPH_MP2_WPE) && SPH_MP2_WPE > 0
#define SPH_MP2_OCC __attribute__((amdgpu_waves_per_eu(SPH_MP2_WPE, SPH_MP2_WPE)))
#else
#define SPH_MP2_OCC
#endif

// r = sqrt(rsq) as the reference takes it, correctly rounded (s = 3 (r / h) then feeds the
// reference-form quintic, sph_mp_kernels.h qr_*, bit for bit), and 1/r: LLVM's f64 sqrt
// sequence (a v_rsq_f64 seed, one Goldschmidt step, two residual corrections) without its
// rescaling of tiny arguments (rsq > 1e-300 here: x + 1e-300 makes a coincident pair give a
// huge 1/r times a zero weight instead of NaN); 1/r = 2 h from the same refinement (~1e-15
// relative: it only scales well-conditioned products)
__device__ __forceinline__ void mp2_r_ir(double x, double &r, double &ir) {
  double h;
  r = cr_sqrt(x + 1e-300, &h);
  ir = 2.0 * h;
}

// per pair type: the stack's cutoffs (squared), 1/h and the coefficients the pair terms use
struct Mp2Pair {
  double rcsq, rih;           // rhosum/multiphase
  double ccsq, cih, calpha;   // colorgradient
  double tcsq, tih, tvisc;    // taitwater/multiphase
  double scsq, sih;           // surfacetension
  double hcsq, hih, halpha2;  // heatconduction/phasechange (2 alpha)
  double htc;
  int hfix, pad;
  // the gather's per-pair-type constants: the dW/dr norms (mp2_dwnorm)
  double tdn, sdn, hdn;
};
struct Mp2Type {
  double B, rho0i, gamma, rbg;
};

// stage the tables of pair types and types into LDS (every thread of the block calls it)
__device__ __forceinline__ double mp2_dwnorm(int dim, double ih);
__device__ __forceinline__ void mp2_tables(const MpCoefs *c, Mp2Pair *sp, Mp2Type *st,
                                           int dim) {
  const int nt1 = c->ntypes + 1;
  for (int p = threadIdx.x; p < nt1 * nt1; p += blockDim.x) {
    Mp2Pair q;
    q.rcsq = c->rcutsq[p];
    q.rih = c->rcut_inv[p];
    q.ccsq = c->ccutsq[p];
    q.cih = c->ccut_inv[p];
    q.calpha = c->calpha[p];
    q.tcsq = c->tcutsq[p];
    q.tih = c->tcut_inv[p];
    q.tvisc = c->tvisc[p];
    q.scsq = c->scutsq[p];
    q.sih = c->scut_inv[p];
    q.hcsq = c->hcutsq[p];
    q.hih = c->hcut_inv[p];
    q.halpha2 = 2.0 * c->halpha[p];
    q.htc = c->htc[p];
    q.hfix = c->hfix[p];
    q.pad = 0;
    q.tdn = mp2_dwnorm(dim, q.tih);
    q.sdn = mp2_dwnorm(dim, q.sih);
    q.hdn = mp2_dwnorm(dim, q.hih);
    sp[p] = q;
  }
  for (int t = threadIdx.x; t < nt1; t += blockDim.x)
    st[t] = Mp2Type{c->B[t], c->rho0_inv[t], c->gamma[t], c->rbg[t]};
  __syncthreads();
}

// h^-dim (W) and h^-(dim+1) (dW) with the norms of sph_kernel_quintic.cpp
__device__ __forceinline__ double mp2_wnorm(int dim, double ih) {
  return dim == 3 ? 0.0716197243913529 * (ih * ih * ih) : 0.04195297663091802 * (ih * ih);
}
__device__ __forceinline__ double mp2_dwnorm(int dim, double ih) {
  const double ih2 = ih * ih;
  return dim == 3 ? 3.0 * 0.0716197243913529 * (ih2 * ih2) : 3.0 * 0.04195297663091802 * (ih2 * ih);
}

// rhosum/multiphase (pair_sph_rhosum_multiphase.cpp:118-167) over the engine's strided /
// CSR full rows: rho_i = rmass_i (W(0)/h^dim + sum_j W(r/h)/h^dim), two entries per lane and
// round with both loads issued first
template <int G>
__global__ void __launch_bounds__(256) k_mp2_rhosum(MpArgs a) {
  __shared__ Mp2Pair s_p[NT2];
  __shared__ Mp2Type s_t[MAXT + 1];
  mp2_tables(a.mc, s_p, s_t, a.dim);
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const int nt1 = a.mc->ntypes + 1, dim = a.dim;
  const int i = a.ilist ? a.ilist[row] : row;
  const double4 xi = a.xf[i];
  const int it = a.ty[i];
  const Mp2Pair *const pi = s_p + it * nt1;
  double acc = 0.0;
  const MpRow rw(a.off, a.cnt, a.stride, row);
  constexpr int NU = SPH_MP2_NU;
  for (long long k0 = rw.beg + lane; k0 < rw.end; k0 += NU * G) {
    double4 xj[NU];
    int tj[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int e = k0 + u * G < rw.end ? a.nbr[k0 + u * G] : a.nbr[rw.beg], j = e & MP_NMASK;
      xj[u] = a.xf[j];
      tj[u] = a.typed ? mp_etype(e) : a.ty[j];
    }
#pragma unroll
    for (int u = 0; u < NU; u++) {
      if (k0 + u * G >= rw.end) break;
      const Mp2Pair &q = pi[tj[u]];
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = rsq_ref(dx, dy, dz);
      if (rsq < q.rcsq) acc += qr_wpoly(3.0 * (cr_sqrt(rsq + 1e-300) * q.rih)) * mp2_wnorm(dim, q.rih);
    }
  }
  acc = group_sum<G>(acc);
  if (lane == 0) {
    const Mp2Pair &q = pi[it];
    a.rho[i] = (qr_wpoly(0.0) * mp2_wnorm(dim, q.rih) + acc) * a.rm[i];
  }
}

// one colorgradient term in the reference's own operation order and rounding
// (pair_sph_colorgradient.cpp:151-179: e_ij = del / r, IEEE divisions, nothing contracted):
// on the bubble lattice the reference's sums cancel pairwise to ~1e-6 of the field's largest
// element, so a term's last bits show there (round 5: reciprocals and 1/r products moved such
// elements by ~1e-9 relative, beyond how far the reference moves between its own builds)
__device__ __forceinline__ void mp2_cg_term(int dim, double dx, double dy, double dz, double r,
                                            double ih, double alpha, double sigmaj,
                                            double sigmai, double &gx, double &gy, double &gz) {
#pragma clang fp contract(off)
  const double ex = dx / r, ey = dy / r;
  double wfd;
  if (dim == 3) {
    wfd = (3.0 * 0.0716197243913529) * qr_dwpoly(3.0 * (r * ih));
    wfd = wfd * ih * ih * ih * ih;
  } else {
    wfd = (3.0 * 0.04195297663091802) * qr_dwpoly(3.0 * (r * ih));
    wfd = wfd * ih * ih * ih;
  }
  const double sigmaj2 = sigmaj * sigmaj;
  const double dphi = -wfd * alpha / sigmaj2 * sigmai;
  gx += dphi * ex;
  gy += dphi * ey;
  if (dim == 3) gz += dphi * (dz / r);
}

// colorgradient (pair_sph_colorgradient.cpp:139-181) over the same rows: records (x, sigma)
// study builds: -DSPH_MP2_CGWPE=n asks for at least n waves per SIMD in colorgradient
#if defined(SPH_MP2_CGWPE) && SPH_MP2_CGWPE > 0
#define SPH_MP2_CGOCC __attribute__((amdgpu_waves_per_eu(SPH_MP2_CGWPE)))
#else
#define SPH_MP2_CGOCC
#endif
template <int G>
__global__ void __launch_bounds__(256) SPH_MP2_CGOCC k_mp2_colorgradient(MpArgs a) {
  __shared__ Mp2Pair s_p[NT2];
  __shared__ Mp2Type s_t[MAXT + 1];
  mp2_tables(a.mc, s_p, s_t, a.dim);
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const int nt1 = a.mc->ntypes + 1, dim = a.dim;
  const int i = a.ilist ? a.ilist[row] : row;
  const double4 xi = a.xs[i];
  const int it = a.ty[i];
  const Mp2Pair *const pi = s_p + it * nt1;
  const double sigmai = xi.w;
  double gx = 0.0, gy = 0.0, gz = 0.0;
  const MpRow rw(a.off, a.cnt, a.stride, row);
  constexpr int NU = SPH_MP2_NU;
  int jn[NU];  // (next round's entries in flight, as k_mp2_gather)
#pragma unroll
  for (int u = 0; u < NU; u++) {
    const long long k = rw.beg + lane + u * G;
    jn[u] = k < rw.end ? a.nbr[k] : 0;
  }
  for (long long k0 = rw.beg + lane; k0 < rw.end; k0 += NU * G) {
    double4 xj[NU];
    int tj[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int e = k0 + u * G < rw.end ? jn[u] : jn[0], j = e & MP_NMASK;
      xj[u] = a.xs[j];
      tj[u] = a.typed ? mp_etype(e) : a.ty[j];
    }
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const long long k = k0 + (NU + u) * G;
      jn[u] = k < rw.end ? a.nbr[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < NU; u++) {
      if (k0 + u * G >= rw.end) break;
      const Mp2Pair &q = pi[tj[u]];
      if (q.calpha == 0.0) continue;
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = rsq_ref(dx, dy, dz);
      if (!(rsq < q.ccsq)) continue;
      double r, ir;
      mp2_r_ir(rsq, r, ir);
      mp2_cg_term(dim, dx, dy, dz, r, q.cih, q.calpha, xj[u].w, sigmai, gx, gy, gz);
    }
  }
  gx = group_sum<G>(gx);
  gy = group_sum<G>(gy);
  gz = group_sum<G>(gz);
  if (lane == 0) a.cg[i] = make_double4(gx, gy, gz, 0.0);
}

// the gather's fresh / stale records of (colour gradient, rho): w = c / sqrt(|c|), zero where
// |c| <= EPSILON = 1e-12 (pair_sph_surfacetension.cpp:29) -- see the header
__device__ __forceinline__ double4 mp2_wrec(const double4 c, double rho, int dim) {
  const double c2 = dim == 3 ? c.x * c.x + c.y * c.y + c.z * c.z : c.x * c.x + c.y * c.y;
  const double ac = sqrt(c2);
  if (!(ac > 1.0e-12)) return make_double4(0.0, 0.0, 0.0, rho);
  const double f = 1.0 / sqrt(ac);
  return make_double4(c.x * f, c.y * f, dim == 3 ? c.z * f : 0.0, rho);
}
static __global__ void k_mp2_pack_rec(int nall, int dim, const double4 *__restrict__ xf,
                                      const double4 *__restrict__ vel,
                                      const double *__restrict__ rm, const double *__restrict__ en,
                                      const double *__restrict__ cv,
                                      const double *__restrict__ rhoF,
                                      const double *__restrict__ rhoS,
                                      const double4 *__restrict__ cgF,
                                      const double4 *__restrict__ cgS, int heat,
                                      double4 *__restrict__ A, double4 *__restrict__ K,
                                      double4 *__restrict__ F, double4 *__restrict__ S) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nall) return;
  const double4 x = xf[i], v = vel[i];
  A[i] = make_double4(x.x, x.y, x.z, rm[i]);
  K[i] = make_double4(v.x, v.y, v.z, heat ? en[i] / cv[i] : 0.0);  // (sph_energy2t)
  F[i] = mp2_wrec(cgF[i], rhoF[i], dim);
  S[i] = mp2_wrec(cgS[i], rhoS[i], dim);
}

// S(w, e) V^2 with |w|^2 = |c|: (|c| e / ndim - (c.e) c / |c|) V^2
__device__ __forceinline__ double3 mp2_svec(int dim, const double4 &w, double3 e, double v2) {
  const double w2 = w.x * w.x + w.y * w.y + w.z * w.z;
  const double we = w.x * e.x + w.y * e.y + w.z * e.z;
  const double a = (dim == 3 ? (1.0 / 3.0) : 0.5) * w2 * v2, b = we * v2;
  return make_double3(a * e.x - b * w.x, a * e.y - b * w.y, dim == 3 ? a * e.z - b * w.z : 0.0);
}

// taitwater/multiphase + surfacetension + heatconduction/phasechange fused over the full
// rows, symmetric styles only (see the header; k_mp_gather otherwise).  Per pair (i = row,
// j = entry; bit 31 = the pair is i's in the half list): i's values fresh unless j is a ghost
// whose image pair belongs to j's owner, j's fresh if owned or if the pair is not i's -- the
// pair terms themselves with i first.
// (108 VGPRs, 4 waves per SIMD: asking for 5 or 6 spills -- 32 / 40 ms per C5 step instead
// of 12.8, profiles/r03/README.md)
// POW = false: every gamma is 1 (bubble.lmp), the pressures are linear in rho and the pow()
// code (and its registers) is not instantiated.
template <int G, bool TAIT, bool SURF, bool HEAT, bool POW = true>
__device__ __forceinline__ void mp2_gather_body(const MpArgs &a) {
  __shared__ Mp2Pair s_p[NT2];
  __shared__ Mp2Type s_t[MAXT + 1];
  mp2_tables(a.mc, s_p, s_t, a.dim);
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const int nt1 = a.mc->ntypes + 1, dim = a.dim;
  const int i = a.ilist ? a.ilist[row] : row;
  const double4 xi = a.pA[i], v4i = a.pK[i];
  const int ti = a.ty[i];
  const Mp2Pair *const pi = s_p + ti * nt1;
  const Mp2Type tyi = s_t[ti];
  const double mi = xi.w, Ti = v4i.w;
  const double4 cFi = a.pF[i], cSi = a.pS[i];
  const double irFi = mp_rcp(cFi.w), irSi = mp_rcp(cSi.w);
  double fx = 0.0, fy = 0.0, fz = 0.0, dE = 0.0;
  const MpRow rw(a.off, a.cnt, a.stride, row);
  const long long kend = rw.end;
  // one pair (i = row, jr = its entry) on the records x_j, v_j (k), c_j (fresh or stale)
  auto pair = [&](int jr, int tj, const double4 &xj, const double4 &v4j, const double4 &cj) {
    const int j = jr & MP_NMASK;
    const bool fi = !(j >= a.nlocal && jr >= 0);
    const double4 ci = fi ? cFi : cSi;
    const Mp2Pair &q = pi[tj];
    const double rhoi = ci.w, rhoj = cj.w, mj = xj.w;
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = rsq_ref(dx, dy, dz);
    const bool ct = TAIT && rsq < q.tcsq, cs = SURF && rsq < q.scsq, ch = HEAT && rsq < q.hcsq;
    if (!(ct || cs || ch)) return;
    double r, ir;
    mp2_r_ir(rsq, r, ir);
    const double qt = ct ? qr_dwpoly(3.0 * (r * q.tih)) * q.tdn : 0.0;
    const double qs = !cs ? 0.0 : (ct && q.sih == q.tih) ? qt : qr_dwpoly(3.0 * (r * q.sih)) * q.sdn;
    const double qh = !ch ? 0.0 : (ct && q.hih == q.tih) ? qt : qr_dwpoly(3.0 * (r * q.hih)) * q.hdn;
    const double iri = fi ? irFi : irSi, irj = mp_rcp(rhoj);
    const double Vi = mi * iri, Vj = mj * irj;
    const double Vi2 = Vi * Vi, Vj2 = Vj * Vj;
    if (ct) {  // pair_sph_taitwater_multiphase.cpp:128-170
      const Mp2Type tyj = s_t[tj];
      const double pI = tyi.B * ((!POW || tyi.gamma == 1.0 ? rhoi * tyi.rho0i
                                                            : pow(rhoi * tyi.rho0i, tyi.gamma)) -
                                 tyi.rbg);
      const double pJ = tyj.B * ((!POW || tyi.gamma == 1.0 ? rhoj * tyj.rho0i
                                                            : pow(rhoj * tyj.rho0i, tyi.gamma)) -
                                 tyj.rbg);
      const double pij = (rhoj * pI + rhoi * pJ) * mp_rcp(rhoi + rhoj);
      const double wfd = qt * ir, V2 = Vi2 + Vj2;
      const double fvisc = V2 * q.tvisc * wfd, fpair = -V2 * pij * wfd;
      fx += dx * fpair + (v4i.x - v4j.x) * fvisc;
      fy += dy * fpair + (v4i.y - v4j.y) * fvisc;
      fz += dz * fpair + (v4i.z - v4j.z) * fvisc;
    }
    if (SURF && cs) {  // pair_sph_surfacetension.cpp:100-190
      // S_i + S_j = (a_i + a_j) e - (b_i w_i + b_j w_j), a = |w|^2 V^2 / ndim, b = (w.e) V^2
      // (mp2_svec of both sides, collected)
      const double3 e = make_double3(dx * ir, dy * ir, dim == 3 ? dz * ir : 0.0);
      const double kd = dim == 3 ? (1.0 / 3.0) : 0.5;
      const double wi2 = ci.x * ci.x + ci.y * ci.y + ci.z * ci.z;
      const double wj2 = cj.x * cj.x + cj.y * cj.y + cj.z * cj.z;
      const double A = kd * fma(wi2, Vi2, wj2 * Vj2);
      const double bi = (ci.x * e.x + ci.y * e.y + ci.z * e.z) * Vi2;
      const double bj = (cj.x * e.x + cj.y * e.y + cj.z * e.z) * Vj2;
      fx = fma(fma(A, e.x, -fma(bi, ci.x, bj * cj.x)), qs, fx);
      fy = fma(fma(A, e.y, -fma(bi, ci.y, bj * cj.y)), qs, fy);
      if (dim == 3) fz = fma(fma(A, e.z, -fma(bi, ci.z, bj * cj.z)), qs, fz);
    }
    if (HEAT && ch) {  // pair_sph_heatconduction_phasechange.cpp:101-136
      double Tp = Ti, Tq = v4j.w;
      if (q.hfix == ti && Tp < Tq) Tp = q.htc;
      if (q.hfix == tj && Tq < Tp) Tq = q.htc;
      dE += q.halpha2 * (Tp - Tq) * (qh * ir) * (iri * Vj);  // (m_j / rho_j = V_j)
    }
  };
  // the records of entry jr: x (with the mass), v (with T), and j's colour-gradient record,
  // fresh if j is owned or the pair is not i's (else as communicated)
  auto fetch = [&](int jr, double4 &xj, double4 &v4j, double4 &cj, int &tj) {
    const int j = jr & MP_NMASK;
    const bool fj = j < a.nlocal || jr >= 0;
    xj = a.pA[j];
    v4j = (TAIT || HEAT) ? a.pK[j] : make_double4(0, 0, 0, 0);
    cj = (fj ? a.pF : a.pS)[j];
    tj = a.typed ? mp_etype(jr) : a.ty[j];
  };
#if SPH_MP2_PIPE
  // software-pipelined walk: entry values two rounds ahead, records one round ahead -- the
  // records of the next entry are in flight while this one is evaluated (the rows stream
  // from L2: one round's latency is covered by the previous round's pair)
  long long k = rw.beg + lane;
  int jc = k < kend ? a.nbr[k] : 0;
  int jn = k + G < kend ? a.nbr[k + G] : 0;
  double4 xc, vc, cc;
  int tc;
  fetch(jc, xc, vc, cc, tc);
  for (; k < kend; k += G) {
    const int jn2 = k + 2 * G < kend ? a.nbr[k + 2 * G] : 0;
    double4 xn, vn, cn;
    int tn;
    fetch(jn, xn, vn, cn, tn);
    pair(jc, tc, xc, vc, cc);
    jc = jn;
    jn = jn2;
    xc = xn;
    vc = vn;
    cc = cn;
    tc = tn;
  }
#else
  constexpr int NU = SPH_MP2_GNU;
  // the next round's entries are read while this round computes (the rows stream from HBM:
  // one dependent miss per round instead of two)
  int jn[NU];
#pragma unroll
  for (int u = 0; u < NU; u++) {
    const long long k = rw.beg + lane + u * G;
    jn[u] = k < kend ? a.nbr[k] : 0;
  }
  for (long long k0 = rw.beg + lane; k0 < kend; k0 += NU * G) {
    int jrs[NU], tjs[NU];
    double4 xjs[NU], v4js[NU], cjs[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) jrs[u] = k0 + u * G < kend ? jn[u] : jn[0];
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const long long k = k0 + (NU + u) * G;
      jn[u] = k < kend ? a.nbr[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < NU; u++) fetch(jrs[u], xjs[u], v4js[u], cjs[u], tjs[u]);
#pragma unroll
    for (int u = 0; u < NU; u++) {
      if (k0 + u * G >= kend) break;
      pair(jrs[u], tjs[u], xjs[u], v4js[u], cjs[u]);
    }
  }
#endif
  fx = group_sum<G>(fx);
  fy = group_sum<G>(fy);
  fz = group_sum<G>(fz);
  dE = group_sum<G>(dE);
  if (lane == 0) {
    if (TAIT || SURF) a.fo[i] = make_double4(fx, fy, fz, 0.0);
    if (HEAT) a.de[i] = dE;
  }
}
template <int G, bool TAIT, bool SURF, bool HEAT, bool POW = true>
__global__ void __launch_bounds__(256) SPH_MP2_OCC k_mp2_gather(MpArgs a) {
  mp2_gather_body<G, TAIT, SURF, HEAT, POW>(a);
}
// ... with at least four waves per SIMD (<= 128 VGPRs): the C5 stack's variant (every gamma
// 1, all three styles) otherwise takes 138 VGPRs = 3 waves since its quintic and sqrt are
// the reference's own (section a6); asked for 4 it keeps one 8-B value in scratch (one
// reload per entry): gather 4.79 vs 5.00 ms per C5 step (profiles/r06/gather_w4/).  The
// gamma != 1 variants (170-196 VGPRs) would spill 24-60 and stay on k_mp2_gather.
template <int G, bool TAIT, bool SURF, bool HEAT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_mp2_gather_w4(MpArgs a) {
  mp2_gather_body<G, TAIT, SURF, HEAT, false>(a);
}

// the styles are symmetric under exchanging a pair's atoms (k_mp2_gather applies): every
// gamma equal, and no type pinned to Tc against its own type
inline bool mp2_gamma1(const MpCoefs &c) {
  for (int t = 1; t <= c.ntypes; t++)
    if (c.gamma[t] != 1.0) return false;
  return true;
}
inline bool mp2_symmetric(const MpCoefs &c) {
  const int nt1 = c.ntypes + 1;
  for (int t = 2; t <= c.ntypes; t++)
    if (c.gamma[t] != c.gamma[1]) return false;
  for (int t = 1; t <= c.ntypes; t++)
    if (c.hfix[t * nt1 + t] == t) return false;
  return true;
}

}  // namespace sph
