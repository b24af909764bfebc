// sph_mp_kernels.h -- gfx950 kernels of the multiphase USER-SPH styles (atom_style
// meso/multiphase: per-atom rmass; quintic spline kernel):
//   sph/rhosum/multiphase          pair_sph_rhosum_multiphase.cpp:112-167      (full list)
//   sph/taitwater/multiphase       pair_sph_taitwater_multiphase.cpp:95-183    (half list)
//   sph/heatconduction/phasechange pair_sph_heatconduction_phasechange.cpp:81-138 (half)
//   sph/colorgradient              pair_sph_colorgradient.cpp:118-187          (full list)
//   sph/surfacetension             pair_sph_surfacetension.cpp:50-192          (half list)
// Same walk as sph_kernels.h: G lanes per list row, register accumulation, xor-shuffle
// group reduction; half lists scatter the Newton-3 share onto j with fp64 atomics, as the
// reference does.  The two half-list styles are NOT pair-symmetric in the reference
// (p_j takes gamma[itype], pair_sph_taitwater_multiphase.cpp:148; the fixed-temperature
// clamp depends on which atom is i, pair_sph_heatconduction_phasechange.cpp:124-129), so
// they follow the caller's half list exactly instead of being rewritten as gathers.
#pragma once
#include <hip/hip_runtime.h>

#include "sph_kernels.h"

namespace sph {

// Engine full lists carry the half list's orientation of each pair, frozen at the build as
// the reference's half list is, in bit 31 of the entry, and the neighbour's type - 1 in bits
// 28-30 (MpArgs::typed; written by k_neigh3's fill): mask with MP_NMASK (LAMMPS' NEIGHMASK
// idiom).  Lists from the pair-style layer set neither; every multiphase list indexes fewer
// than 2^28 atoms (MP_MAXALL, checked where lists are staged or built).
constexpr int MP_NMASK = 0x0fffffff;
// type - 1 in bits 28-30: three bits, so at most 8 types (the self-exclusion test xj.w != di
// and the j decode would alias otherwise)
static_assert(SPH_MAXTYPES <= 8, "packed list entries hold type - 1 in three bits");
constexpr long long MP_MAXALL = 1ll << 28;
__device__ __forceinline__ int mp_etype(int e) { return ((e >> 28) & 7) + 1; }

struct MpCoefs {
  int ntypes, dim;
  // rhosum/multiphase: h = cut[it][jt]
  double rcut[NT2], rcutsq[NT2];
  // taitwater/multiphase: per type rho0, B = c^2 rho0 / gamma, gamma, rbackground
  double rho0[MAXT + 1], B[MAXT + 1], gamma[MAXT + 1], rbg[MAXT + 1];
  double tvisc[NT2], tcut[NT2], tcutsq[NT2];
  // heatconduction/phasechange
  double halpha[NT2], hcut[NT2], hcutsq[NT2], htc[NT2];
  int hfix[NT2];
  // colorgradient
  double calpha[NT2], ccut[NT2], ccutsq[NT2];
  // surfacetension: h = cut[it][jt]
  double scut[NT2], scutsq[NT2];
  // 1/h of every style and 1/rho0 (mp_inverses: the reference's own 1.0/h, taken once)
  double rcut_inv[NT2], tcut_inv[NT2], hcut_inv[NT2], ccut_inv[NT2], scut_inv[NT2];
  double rho0_inv[MAXT + 1];
};

// the reciprocal tables of MpCoefs from its cut / rho0 tables (host, before every upload)
inline void mp_inverses(MpCoefs &m) {
  auto inv = [](double h) { return h != 0.0 ? 1.0 / h : 0.0; };
  for (int k = 0; k < NT2; k++) {
    m.rcut_inv[k] = inv(m.rcut[k]);
    m.tcut_inv[k] = inv(m.tcut[k]);
    m.hcut_inv[k] = inv(m.hcut[k]);
    m.ccut_inv[k] = inv(m.ccut[k]);
    m.scut_inv[k] = inv(m.scut[k]);
  }
  for (int t = 0; t <= MAXT; t++) m.rho0_inv[t] = inv(m.rho0[t]);
}

// the quintic kernel's dW/dr scaled by h^-(dim+1) (the styles' wfd before any 1/r)
__device__ __forceinline__ double quintic_dw(int dim, double r);
__device__ __forceinline__ double mp_qdw(int dim, double r, double ih);

// 1/b for the pair terms' divisions: v_rcp_f64 seed + one Newton step (~1 ulp; the fp64
// IEEE division sequence costs ~3x the issue slots, and the 1e-10 parity bar is kept)
__device__ __forceinline__ double mp_rcp(double b) {
  const double y = __builtin_amdgcn_rcp(b);
  return fma(y, fma(-b, y, 1.0), y);
}

// Quintic spline, sph_kernel_quintic.cpp:17-73 (s = 3r), in the reference's own arithmetic:
// its expanded piecewise polynomials through pow(x, n), evaluated left to right with every
// product and sum rounded (its x86-64 build has no FMA, so nothing is contracted).  Near the
// cutoff those polynomials cancel (dW ~ -5 s^4 + 60 s^3 - ... - 405 with terms ~1e3 for a
// result ~1e-6), so their rounding errors ARE the reference's dW there; a factored form
// (exact to ~1 ulp) sits up to ~1e-13 absolute away from it, which a small colour-gradient or
// force element shows at ~1e-9 relative (the round-5 C5 tests).  pow(x, n) for n = 2..5 is
// evaluated correctly rounded (double-double products, one final rounding): glibc's pow
// agrees with the correctly rounded power except in ~0.08 % of calls (1 ulp, tools/
// quintic_pow_check.c), so dW matches the reference bit for bit except there.
__device__ __forceinline__ double qr_pow3(double x) {  // x^3, correctly rounded
  const double h = x * x, l = fma(x, x, -h);
  const double p = x * h, e = fma(x, h, -p);
  return p + fma(x, l, e);
}
__device__ __forceinline__ void qr_pow4dd(double x, double &q, double &t) {  // x^4 = q + t
  const double h = x * x, l = fma(x, x, -h);
  q = h * h;
  t = fma(2.0 * h, l, fma(h, h, -q));
}
__device__ __forceinline__ double qr_pow4(double x) {
  double q, t;
  qr_pow4dd(x, q, t);
  return q + t;
}
__device__ __forceinline__ double qr_pow5(double x) {
  double q, t;
  qr_pow4dd(x, q, t);
  const double p = x * q, e = fma(x, q, -p);
  return p + fma(x, t, e);
}
// the reference's W(s) / norm: pow(3-s,5) - 6 pow(2-s,5) + 15 pow(1-s,5) on [0,1), the first two
// on [1,2), the first on [2,3), 0 beyond -- the pieces as zero terms (x - 0 and x + 0 are x)
__device__ __forceinline__ double qr_wpoly(double s) {
#pragma clang fp contract(off)
  const double a = s < 3.0 ? qr_pow5(3.0 - s) : 0.0;
  const double b = s < 2.0 ? qr_pow5(2.0 - s) : 0.0;
  double c = 0.0;
  if (__any(s < 1.0)) c = s < 1.0 ? qr_pow5(1.0 - s) : 0.0;  // (rare: s = r / dx >= ~1)
  return (a - 6.0 * b) + 15.0 * c;
}
// the reference's dW/ds / norm: c4 pow(s,4) + c3 pow(s,3) + c2 pow(s,2) + c1 s + c0 with the
// piece's integer coefficients (a missing term is + 0 * s^2 or + 0: exact), left to right.
// Pairs sit at s >= ~1 (h = 3 dx, s = r / dx): the [1,2) / [2,3) coefficients are one select
// each, the rare [0,1) piece a wave-uniform branch
__device__ __forceinline__ double qr_dwpoly(double s) {
#pragma clang fp contract(off)
  const bool p2 = s < 2.0;
  double c4 = p2 ? 25.0 : -5.0, c3 = p2 ? -180.0 : 60.0, c2 = p2 ? 450.0 : -270.0;
  double c1 = p2 ? -420.0 : 540.0, c0 = p2 ? 75.0 : -405.0;
  if (__any(s < 1.0)) {
    const bool p1 = s < 1.0;
    c4 = p1 ? -50.0 : c4;
    c3 = p1 ? 120.0 : c3;
    c2 = p1 ? 0.0 : c2;
    c1 = p1 ? -120.0 : c1;
    c0 = p1 ? 0.0 : c0;
  }
  const double w = (((c4 * qr_pow4(s) + c3 * qr_pow3(s)) + c2 * (s * s)) + c1 * s) + c0;
  return s < 3.0 ? w : 0.0;
}
__device__ __forceinline__ double quintic_w(int dim, double r) {
#pragma clang fp contract(off)
  const double norm = (dim == 3) ? 0.0716197243913529 : 0.04195297663091802;
  return norm * qr_wpoly(3.0 * r);
}
__device__ __forceinline__ double quintic_dw(int dim, double r) {
#pragma clang fp contract(off)
  const double norm = (dim == 3) ? 3.0 * 0.0716197243913529 : 3.0 * 0.04195297663091802;
  return norm * qr_dwpoly(3.0 * r);
}

__device__ __forceinline__ double mp_qdw(int dim, double r, double ih) {
  return dim == 3 ? quintic_dw(3, r * ih) * ih * ih * ih * ih
                  : quintic_dw(2, r * ih) * ih * ih * ih;
}

struct MpArgs {
  int inum, nlocal, newton, dim, half;
  const int *ilist, *off, *nbr;
  const double4 *xf;  // x, y, z, (unused)
  const double4 *vr;  // vest, rho
  const int *ty;
  const double *rm, *en, *cv;
  const MpCoefs *mc;
  double *rho;    // rhosum out (nall)
  double4 *fo;    // taitwater out (nall, x y z used)
  double *de;     // heat out (nall)
  double4 *cg;    // colorgradient out (nall)
  const double4 *cgi;  // surfacetension: colorgradient of every atom (nall, x y z used)
  int exp;             // study (SPH_MPX): 1 = skip the Newton-3 atomics onto j
  int typed;           // entries carry the neighbour's type (engine lists, mp_etype)
  int rev;             // half list with its reverse list: j share gathered (k_mp_half REV)
  const int *roff, *rnbr;  // reverse half list: row j holds the atoms whose half row has j
  int nrows;               // reverse rows (nall with newton_pair, else nlocal)
  // k_mp_gather: v of every atom, and rho / colorgradient in two versions -- S (stale: the
  // values the atoms' ghost copies carry, i.e. before this step's rhosum / colorgradient)
  // and F (fresh: after them, forwarded to the ghosts too)
  const double4 *vel;
  const double *rhoS, *rhoF;
  const double4 *cgS, *cgF;
  // ... packed per atom (k_mp_pack_rec): (x, rmass), (v, T), (cg, rho) fresh / stale
  const double4 *pA, *pK, *pF, *pS;
  // colorgradient: (x, y, z, sigma = rho / rmass) per atom, rho as it stands (nullptr: the
  // kernel reads xf, vr, rm)
  const double4 *xs;
  // stride > 0: fixed-stride rows (row r at r*stride, cnt[r] entries) instead of CSR off
  int stride;
  const int *cnt;
};
// a list row's entries [beg, end): CSR (off) or fixed-stride rows (stride, cnt)
struct MpRow {
  long long beg, end;  // (64-bit: fixed-stride rows of any system size)
  __device__ __forceinline__ MpRow(const int *off, const int *cnt, int stride, int row) {
    if (stride > 0) {
      beg = (long long)row * stride;
      end = beg + cnt[row];
    } else {
      beg = off[row];
      end = off[row + 1];
    }
  }
};

template <int G>
__global__ void __launch_bounds__(256) k_mp_rhosum(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int i = a.ilist ? a.ilist[row] : row;
  const double4 xi = a.xf[i];
  const int it = a.ty[i];
  const int dim = a.dim;
  double acc = 0.0;
  const MpRow rw(a.off, a.cnt, a.stride, row);
  for (long long k = rw.beg + lane; k < rw.end; k += G) {
    const int j = a.nbr[k] & MP_NMASK;
    const double4 xj = a.xf[j];
    const int jt = a.ty[j];
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = rsq_ref(dx, dy, dz);
    if (rsq < c->rcutsq[it * nt1 + jt]) {
      const double ih = c->rcut_inv[it * nt1 + jt];
      const double r = sqrt(rsq) * ih;
      acc += (dim == 3) ? quintic_w(3, r) * ih * ih * ih : quintic_w(2, r) * ih * ih;
    }
  }
  acc = group_sum<G>(acc);
  if (lane == 0) {
    const double h = c->rcut[it * nt1 + it];
    const double self = (dim == 3) ? quintic_w(3, 0.0) / (h * h * h) : quintic_w(2, 0.0) / (h * h);
    a.rho[i] = (self + acc) * a.rm[i];
  }
}

// p = B (pow(rho/rho0, gamma) - rbackground), pair_sph_taitwater_multiphase.cpp:289-292.
// pow(x, 1) == x exactly (C99 F.9.4.4), and gamma = 1 is the bubble_growth value: the
// library pow runs only for other exponents
__device__ __forceinline__ double mp_pressure(double B, double rho0, double gamma, double rbg,
                                              double rho) {  // (rho0 = 1/rho0)
  const double x = rho * rho0;  // (rho0: 1/rho0 from the table)
  return B * ((gamma == 1.0 ? x : pow(x, gamma)) - rbg);
}


// ---- half-list styles: taitwater/multiphase, heatconduction/phasechange, surfacetension ----
// The reference's per-pair arithmetic as device functions of the pair (i = the list row's
// atom, j = the entry), so the same value can be added to i and subtracted from j.
enum { MP_TAIT = 0, MP_HEAT = 1, MP_SURF = 2 };

// taitwater/multiphase (pair_sph_taitwater_multiphase.cpp:128-170): force on i
__device__ __forceinline__ bool mp_tait_pair(const MpCoefs *c, int dim, double4 xi, double4 vi,
                                             int it, double mi, double4 xj, double4 vj, int jt,
                                             double mj, double3 &F) {
  const int p = it * (c->ntypes + 1) + jt;
  const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
  const double rsq = rsq_ref(dx, dy, dz);
  if (!(rsq < c->tcutsq[p])) return false;
  const double ih = c->tcut_inv[p];
  const double r = sqrt(rsq);
  double wfd;
  if (dim == 3) wfd = quintic_dw(3, r * ih) * ih * ih * ih * ih * mp_rcp(r);
  else wfd = quintic_dw(2, r * ih) * ih * ih * ih * mp_rcp(r);
  const double rhoi = vi.w, rhoj = vj.w;
  const double Vi = mi * mp_rcp(rhoi), Vj = mj * mp_rcp(rhoj);
  const double Vi2 = Vi * Vi, Vj2 = Vj * Vj;
  const double pi = mp_pressure(c->B[it], c->rho0_inv[it], c->gamma[it], c->rbg[it], rhoi);
  // reference quirk kept: p_j with gamma[itype] (pair_sph_taitwater_multiphase.cpp:148)
  const double pj = mp_pressure(c->B[jt], c->rho0_inv[jt], c->gamma[it], c->rbg[jt], rhoj);
  const double pij = (rhoj * pi + rhoi * pj) * mp_rcp(rhoi + rhoj);
  const double velx = vi.x - vj.x, vely = vi.y - vj.y, velz = vi.z - vj.z;
  const double fvisc = (Vi2 + Vj2) * c->tvisc[p] * wfd;
  const double fpair = -(Vi2 + Vj2) * pij * wfd;
  F = make_double3(dx * fpair + velx * fvisc, dy * fpair + vely * fvisc, dz * fpair + velz * fvisc);
  return true;
}

// heatconduction/phasechange (pair_sph_heatconduction_phasechange.cpp:101-136): deltaE;
// de_i += deltaE m_j, de_j -= deltaE m_i
__device__ __forceinline__ bool mp_heat_pair(const MpCoefs *c, int dim, double4 xi, int it,
                                             double rhoi, double Ti0, double4 xj, int jt,
                                             double rhoj, double Tj0, double &deltaE) {
  const int p = it * (c->ntypes + 1) + jt;
  const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
  const double rsq = rsq_ref(dx, dy, dz);
  if (!(rsq < c->hcutsq[p])) return false;
  const double ih = c->hcut_inv[p];
  const double r = sqrt(rsq);
  double wfd;
  if (dim == 3) {
    wfd = quintic_dw(3, r * ih);
    wfd = wfd * ih * ih * ih * ih * mp_rcp(r);
  } else {
    wfd = quintic_dw(2, r * ih);
    wfd = wfd * ih * ih * ih * mp_rcp(r);
  }
  double Ti = Ti0, Tj = Tj0;
  const int ff = c->hfix[p];
  if (ff == it && Ti < Tj) Ti = c->htc[p];
  if (ff == jt && Tj < Ti) Tj = c->htc[p];
  deltaE = 2.0 * c->halpha[p] * (Ti - Tj) * wfd * mp_rcp(rhoi * rhoj);
  return true;
}

template <int G>
__global__ void __launch_bounds__(256) k_mp_colorgradient(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int i = a.ilist ? a.ilist[row] : row;
  const double4 xi = a.xs ? a.xs[i] : a.xf[i];
  const int it = a.ty[i];
  const double sigmai = a.xs ? xi.w : a.vr[i].w / a.rm[i];
  double gx = 0.0, gy = 0.0, gz = 0.0;
  const MpRow rw(a.off, a.cnt, a.stride, row);
  for (long long k = rw.beg + lane; k < rw.end; k += G) {
    const int j = a.nbr[k] & MP_NMASK;
    const double4 xj = a.xs ? a.xs[j] : a.xf[j];
    const int jt = a.ty[j];
    const int p = it * nt1 + jt;
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = rsq_ref(dx, dy, dz);
    if (!(rsq < c->ccutsq[p])) continue;
    const double r = sqrt(rsq);
    const double ih = c->ccut_inv[p];
    double wfd;
    if (a.dim == 3) wfd = quintic_dw(3, r * ih) * ih * ih * ih * ih;
    else wfd = quintic_dw(2, r * ih) * ih * ih * ih;
    const double sigmaj = a.xs ? xj.w : a.vr[j].w / a.rm[j];
    const double dphi = -wfd * c->calpha[p] * mp_rcp(sigmaj * sigmaj) * sigmai;
    const double ir = mp_rcp(r);
    gx += dphi * (dx * ir);
    gy += dphi * (dy * ir);
    if (a.dim == 3) gz += dphi * (dz * ir);
  }
  gx = group_sum<G>(gx);
  gy = group_sum<G>(gy);
  gz = group_sum<G>(gz);
  if (lane == 0) a.cg[i] = make_double4(gx, gy, gz, 0.0);
}

// Surface stress vector S = (|c|^2/ndim I - c c^T) e / |c| of colorgradient c along the
// pair direction e (pair_sph_surfacetension.cpp:135-168; zero for |c| <= EPSILON = 1e-12,
// :29), written term by term as the reference does.
__device__ __forceinline__ double3 st_vector(int dim, double4 c, double absc, double3 e) {
  if (!(absc > 1.0e-12)) return make_double3(0.0, 0.0, 0.0);
  const double ia = mp_rcp(absc);
  if (dim == 2)
    return make_double3(
        (e.x * ((c.y * c.y + c.x * c.x) / 2 - c.x * c.x) - c.x * e.y * c.y) * ia,
        (e.y * ((c.y * c.y + c.x * c.x) / 2 - c.y * c.y) - e.x * c.x * c.y) * ia, 0.0);
  return make_double3(
      (e.x * (0.3333333333333333 * c.z * c.z + 0.3333333333333333 * c.y * c.y -
              0.6666666666666666 * c.x * c.x) -
       1.0 * c.x * e.z * c.z - 1.0 * c.x * e.y * c.y) * ia,
      (e.y * (0.3333333333333333 * c.z * c.z - 0.6666666666666666 * c.y * c.y +
              0.3333333333333333 * c.x * c.x) -
       1.0 * c.y * e.z * c.z - 1.0 * e.x * c.x * c.y) * ia,
      (e.z * (-0.6666666666666666 * c.z * c.z + 0.3333333333333333 * c.y * c.y +
              0.3333333333333333 * c.x * c.x) -
       1.0 * e.y * c.y * c.z - 1.0 * e.x * c.x * c.z) * ia);
}
__device__ __forceinline__ double st_abs(int dim, double4 c) {
  return dim == 3 ? sqrt(c.x * c.x + c.y * c.y + c.z * c.z) : sqrt(c.x * c.x + c.y * c.y);
}


// surfacetension (pair_sph_surfacetension.cpp:100-190): F = (S_i V_i^2 + S_j V_j^2) dW
__device__ __forceinline__ bool mp_surf_pair(const MpCoefs *c, int dim, double4 xi, int it,
                                             double Vi, double4 cgi, double abscgi, double4 xj,
                                             int jt, double Vj, double4 cgj, double3 &F) {
  const int p = it * (c->ntypes + 1) + jt;
  const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
  const double rsq = rsq_ref(dx, dy, dz);
  if (!(rsq < c->scutsq[p])) return false;
  const double ih = c->scut_inv[p];
  const double r = sqrt(rsq);
  const double wfd = (dim == 3) ? quintic_dw(3, r * ih) * ih * ih * ih * ih
                                : quintic_dw(2, r * ih) * ih * ih * ih;
  const double ir = mp_rcp(r);
  const double3 e = make_double3(dx * ir, dy * ir, dim == 3 ? dz * ir : 0.0);
  const double3 Si = st_vector(dim, cgi, abscgi, e);
  const double3 Sj = st_vector(dim, cgj, st_abs(dim, cgj), e);
  F = make_double3((Si.x * Vi * Vi + Sj.x * Vj * Vj) * wfd, (Si.y * Vi * Vi + Sj.y * Vj * Vj) * wfd,
                   dim == 3 ? (Si.z * Vi * Vi + Sj.z * Vj * Vj) * wfd : 0.0);
  return true;
}

// One pass of a half-list style over list rows (REV = false: rows = the caller's list, the
// pair's share onto i; full lists add into i only, half lists without a reverse list also
// scatter the j share with fp64 atomics, as the reference scatters) or over the REVERSE
// half list (REV = true: row = atom j, entries = the atoms i whose half row holds j; the
// same pair value, recomputed with i as the row atom, is subtracted from j).  With a
// reverse list the j share is gathered: no atomics (device fp64 atomics run at ~35 G/s).
template <int G, int STYLE, bool REV>
__global__ void __launch_bounds__(256) k_mp_half(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  const int nrows = REV ? a.nrows : a.inum;
  if (row >= nrows) return;
  const MpCoefs *c = a.mc;
  const int dim = a.dim;
  const int r = REV ? row : a.ilist[row];  // this row's atom
  const double4 xr = a.xf[r], vrr = a.vr[r];
  const int tr = a.ty[r];
  const double mr = a.rm[r];
  const double Tr = STYLE == MP_HEAT ? a.en[r] / a.cv[r] : 0.0;  // sph_energy2t
  const double4 cgr = STYLE == MP_SURF ? a.cgi[r] : make_double4(0, 0, 0, 0);
  const double abscgr = STYLE == MP_SURF ? st_abs(dim, cgr) : 0.0;
  const double Vr = STYLE == MP_SURF ? mr / vrr.w : 0.0;
  const int *off = REV ? a.roff : a.off;
  const int *nbr = REV ? a.rnbr : a.nbr;
  const bool scatter = !REV && a.half && !a.rev && !(a.exp & 1);
  double sx = 0.0, sy = 0.0, sz = 0.0;
  for (int k = off[row] + lane; k < off[row + 1]; k += G) {
    const int o = nbr[k];  // the other atom of the pair
    const double4 xo = a.xf[o], vo = a.vr[o];
    const int to = a.ty[o];
    const double mo = a.rm[o];
    // pair (i, j): i = row atom for REV = false, the entry for REV = true
    if (STYLE == MP_TAIT) {
      double3 F;
      const bool hit = REV ? mp_tait_pair(c, dim, xo, vo, to, mo, xr, vrr, tr, mr, F)
                           : mp_tait_pair(c, dim, xr, vrr, tr, mr, xo, vo, to, mo, F);
      if (!hit) continue;
      if (REV) {
        sx -= F.x;
        sy -= F.y;
        sz -= F.z;
      } else {
        sx += F.x;
        sy += F.y;
        sz += F.z;
        if (scatter && (a.newton || o < a.nlocal)) {
          atomicAdd(&a.fo[o].x, -F.x);
          atomicAdd(&a.fo[o].y, -F.y);
          atomicAdd(&a.fo[o].z, -F.z);
        }
      }
    } else if (STYLE == MP_SURF) {
      double3 F;
      const double Vo = mo / vo.w;
      const double4 cgo = a.cgi[o];
      const bool hit = REV ? mp_surf_pair(c, dim, xo, to, Vo, cgo, st_abs(dim, cgo), xr, tr, Vr,
                                          cgr, F)
                           : mp_surf_pair(c, dim, xr, tr, Vr, cgr, abscgr, xo, to, Vo, cgo, F);
      if (!hit) continue;
      if (REV) {
        sx -= F.x;
        sy -= F.y;
        sz -= F.z;
      } else {
        sx += F.x;
        sy += F.y;
        sz += F.z;
        if (scatter && (a.newton || o < a.nlocal)) {
          atomicAdd(&a.fo[o].x, -F.x);
          atomicAdd(&a.fo[o].y, -F.y);
          if (dim == 3) atomicAdd(&a.fo[o].z, -F.z);
        }
      }
    } else {
      const double To = a.en[o] / a.cv[o];
      double dE;
      const bool hit = REV ? mp_heat_pair(c, dim, xo, to, vo.w, To, xr, tr, vrr.w, Tr, dE)
                           : mp_heat_pair(c, dim, xr, tr, vrr.w, Tr, xo, to, vo.w, To, dE);
      if (!hit) continue;
      if (REV) {
        sx -= dE * mo;
      } else {
        sx += dE * mo;
        if (scatter && (a.newton || o < a.nlocal)) atomicAdd(&a.de[o], -dE * mr);
      }
    }
  }
  sx = group_sum<G>(sx);
  if (STYLE != MP_HEAT) {
    sy = group_sum<G>(sy);
    sz = group_sum<G>(sz);
  }
  if (lane != 0) return;
  if (STYLE == MP_HEAT) {
    if (scatter) atomicAdd(&a.de[r], sx);
    else a.de[r] += sx;  // one row per atom per pass: plain read-modify-write
  } else if (scatter) {
    atomicAdd(&a.fo[r].x, sx);
    atomicAdd(&a.fo[r].y, sy);
    atomicAdd(&a.fo[r].z, sz);
  } else {
    a.fo[r].x += sx;
    a.fo[r].y += sy;
    a.fo[r].z += sz;
  }
}

// The three half-list styles fused and gathered over the FULL list (the device-resident
// engine): the reference evaluates each pair once, with the half list's row atom first
// (half_from_full_newton: owned j if i < j, ghost j if above i in z, y, x), adds the value
// to that atom and subtracts it from the other (Newton-3, then reverse comm for ghosts).
// Here every owned atom walks its full row and evaluates each pair in that same
// orientation -- F(i,j) when the pair is i's, F(j,i) when it is j's (or, for a ghost j, its
// owner's image pair) -- adding or subtracting it: the same pair values, gather-only, no
// atomics, no reverse comm.  With the stale-ghost quirk (ghosts keep their
// comm-time rho and colorgradient) the reference's value of a pair depends on which side
// is owned where it is evaluated: the pair's row atom uses its fresh values when owned, and
// the other atom its fresh values when owned, stale ones when a ghost.  So for owned i and
// neighbour j: owned j -> both fresh; ghost j in i's half row -> i fresh, j stale; ghost j
// whose image pair belongs to j's owner (evaluated there with the owner fresh and i's ghost
// copy stale) -> j fresh, i stale.  fo[i].xyz and de[i] of the owned rows are overwritten
// (fo.w = drho = 0: none of the styles has a drho term).
template <class T>
__device__ __forceinline__ T mp_sel(bool c, const T &a, const T &b) {
  return c ? a : b;
}

template <int G, bool TAIT, bool SURF, bool HEAT>
__global__ void __launch_bounds__(256) k_mp_gather(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int dim = a.dim;
  const int i = a.ilist ? a.ilist[row] : row;
  // packed records (k_mp_pack_rec): .w of A = rmass, of K = T, of F / S = rho
  const double4 xi = a.pA[i], v4i = a.pK[i];
  const int ti = a.ty[i];
  const double mi = xi.w;
  const double Ti = v4i.w;
  const double4 cFi = a.pF[i], cSi = a.pS[i];
  const double rFi = cFi.w, rSi = cSi.w;
  double fx = 0.0, fy = 0.0, fz = 0.0, dE = 0.0;
  // two entries per lane and round, both entries' records loaded before either is used
  // (the loop is latency-bound on the index -> record chain otherwise)
  constexpr int NU = 2;
  const MpRow rw(a.off, a.cnt, a.stride, row);
  const long long kend = rw.end;
  for (long long k0 = rw.beg + lane; k0 < kend; k0 += NU * G) {
    int jrs[NU];
    double4 xjs[NU], v4js[NU], cjs[NU];
    int tjs[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) jrs[u] = k0 + u * G < kend ? a.nbr[k0 + u * G] : 0;
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int j = jrs[u] & MP_NMASK;
      const bool fj = !(j >= a.nlocal) || !(jrs[u] < 0);
      xjs[u] = a.pA[j];
      v4js[u] = (TAIT || HEAT) ? a.pK[j] : make_double4(0, 0, 0, 0);
      cjs[u] = (fj ? a.pF : a.pS)[j];
      tjs[u] = a.ty[j];
    }
#pragma unroll
  for (int u = 0; u < NU; u++) {
    if (k0 + u * G >= kend) break;
    const int jr = jrs[u];
    const int j = jr & MP_NMASK;
    const bool own = jr < 0;  // (bit 31: the pair is i's in the half list, k_neigh3)
    const bool gj = j >= a.nlocal;
    const bool fi = !(gj && !own);  // fresh or stale values of i (see above; j's: cjs)
    const double4 xj = xjs[u];
    const double4 v4j = v4js[u];
    const double4 cj = cjs[u];  // (colorgradient, rho) of j as used here
    const int tj = tjs[u];
    const double mj = xj.w;
    const double rhoi = fi ? rFi : rSi;
    const double rhoj = cj.w;
    const double sg = own ? 1.0 : -1.0;
    // the pair's row atom (p) and neighbour (q) in the half list
    const double4 xp = mp_sel(own, xi, xj), xq = mp_sel(own, xj, xi);
    const int tp = own ? ti : tj, tq = own ? tj : ti;
    const double mp = own ? mi : mj, mq = own ? mj : mi;
    const double rp = own ? rhoi : rhoj, rq = own ? rhoj : rhoi;
    // the three styles' pair terms (mp_tait_pair, mp_surf_pair, mp_heat_pair) sharing the
    // geometry: r, 1/r, and the quintic dW once per distinct cutoff (bubble.lmp: one h)
    const int pc = tp * (c->ntypes + 1) + tq;
    const double dx = xp.x - xq.x, dy = xp.y - xq.y, dz = xp.z - xq.z;
    const double rsq = rsq_ref(dx, dy, dz);
    const bool ct = TAIT && rsq < c->tcutsq[pc], cs = SURF && rsq < c->scutsq[pc],
               ch = HEAT && rsq < c->hcutsq[pc];
    if (!(ct || cs || ch)) continue;
    const double r = sqrt(rsq), ir = mp_rcp(r);
    const double iht = c->tcut_inv[pc], ihs = c->scut_inv[pc], ihh = c->hcut_inv[pc];
    const double qt = ct ? mp_qdw(dim, r, iht) : 0.0;
    const double qs = !cs ? 0.0 : (ct && ihs == iht) ? qt : mp_qdw(dim, r, ihs);
    const double qh = !ch ? 0.0 : (ct && ihh == iht) ? qt : (cs && ihh == ihs) ? qs
                                                                            : mp_qdw(dim, r, ihh);
    if (ct) {  // taitwater/multiphase (pair_sph_taitwater_multiphase.cpp:128-170)
      const double wfd = qt * ir;
      const double4 vp = mp_sel(own, v4i, v4j), vq = mp_sel(own, v4j, v4i);
      const double Vi = mp * mp_rcp(rp), Vj = mq * mp_rcp(rq);
      const double V2 = Vi * Vi + Vj * Vj;
      const double pi = mp_pressure(c->B[tp], c->rho0_inv[tp], c->gamma[tp], c->rbg[tp], rp);
      // reference quirk kept: p_j with gamma[itype] (pair_sph_taitwater_multiphase.cpp:148)
      const double pj = mp_pressure(c->B[tq], c->rho0_inv[tq], c->gamma[tp], c->rbg[tq], rq);
      const double pij = (rq * pi + rp * pj) * mp_rcp(rp + rq);
      const double fvisc = V2 * c->tvisc[pc] * wfd;
      const double fpair = -V2 * pij * wfd;
      fx += sg * (dx * fpair + (vp.x - vq.x) * fvisc);
      fy += sg * (dy * fpair + (vp.y - vq.y) * fvisc);
      fz += sg * (dz * fpair + (vp.z - vq.z) * fvisc);
    }
    if (SURF && cs) {  // surfacetension (pair_sph_surfacetension.cpp:100-190)
      const double4 ci = fi ? cFi : cSi;
      const double4 cp = mp_sel(own, ci, cj), cq = mp_sel(own, cj, ci);
      const double Vp = mp * mp_rcp(rp), Vq = mq * mp_rcp(rq);
      const double3 e = make_double3(dx * ir, dy * ir, dim == 3 ? dz * ir : 0.0);
      const double3 Sp = st_vector(dim, cp, st_abs(dim, cp), e);
      const double3 Sq = st_vector(dim, cq, st_abs(dim, cq), e);
      fx += sg * ((Sp.x * Vp * Vp + Sq.x * Vq * Vq) * qs);
      fy += sg * ((Sp.y * Vp * Vp + Sq.y * Vq * Vq) * qs);
      if (dim == 3) fz += sg * ((Sp.z * Vp * Vp + Sq.z * Vq * Vq) * qs);
    }
    if (HEAT && ch) {  // heatconduction/phasechange (pair_sph_heatconduction_phasechange.cpp:101-136)
      double Tp = own ? Ti : v4j.w, Tq = own ? v4j.w : Ti;
      const int ff = c->hfix[pc];
      if (ff == tp && Tp < Tq) Tp = c->htc[pc];
      if (ff == tq && Tq < Tp) Tq = c->htc[pc];
      const double d = 2.0 * c->halpha[pc] * (Tp - Tq) * (qh * ir) * mp_rcp(rp * rq);
      // de_p += deltaE m_q, de_q -= deltaE m_p (:132-136)
      dE += sg * d * mj;
    }
  }
  }
  fx = group_sum<G>(fx);
  fy = group_sum<G>(fy);
  fz = group_sum<G>(fz);
  dE = group_sum<G>(dE);
  if (lane == 0) {
    if (TAIT || SURF) a.fo[i] = make_double4(fx, fy, fz, 0.0);
    if (HEAT) a.de[i] = dE;
  }
}

// reverse half list: entry owner (the row's atom) of every list entry
static __global__ void __launch_bounds__(256)
k_entry_owner(int inum, const int *__restrict__ off, const int *__restrict__ ilist,
              int *__restrict__ owner) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= inum) return;
  const int i = ilist[row];
  for (int k = off[row]; k < off[row + 1]; k++) owner[k] = i;
}
// reverse CSR offsets: roff[j] = first position of key >= j in the sorted keys
static __global__ void __launch_bounds__(256)
k_rev_offsets(int nrows, int tot, const int *__restrict__ skey, int *__restrict__ roff) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > nrows) return;
  int lo = 0, hi = tot;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (skey[m] < j) lo = m + 1;
    else hi = m;
  }
  roff[j] = lo;
}

}  // namespace sph
