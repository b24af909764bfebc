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
};

// Quintic spline, sph_kernel_quintic.cpp:17-73 (s = 3r).  The reference's pow(x, n) with
// small integer n are evaluated as products (a few ulp apart from libm pow; the golden
// vectors hold at 1e-13), and the branches as selects of one polynomial per piece.
__device__ __forceinline__ double p5(double x) {
  const double x2 = x * x;
  return x2 * x2 * x;
}
__device__ __forceinline__ double quintic_w(int dim, double r) {
  const double norm = (dim == 3) ? 0.0716197243913529 : 0.04195297663091802;
  const double s = 3.0 * r;
  const double a = s < 3.0 ? p5(3 - s) : 0.0;
  const double b = s < 2.0 ? 6 * p5(2 - s) : 0.0;
  const double c = s < 1.0 ? 15 * p5(1 - s) : 0.0;
  return norm * (a - b + c);
}
__device__ __forceinline__ double quintic_dw(int dim, double r) {
  const double norm = 3.0 * ((dim == 3) ? 0.0716197243913529 : 0.04195297663091802);
  const double s = 3.0 * r;
  const double s2 = s * s, s3 = s2 * s, s4 = s2 * s2;
  double wfd;
  if (s < 1) {
    wfd = -50 * s4 + 120 * s3 - 120 * s;
  } else if (s < 2) {
    wfd = 25 * s4 - 180 * s3 + 450 * s2 - 420 * s + 75;
  } else if (s < 3.0) {
    wfd = -5 * s4 + 60 * s3 - 270 * s2 + 540 * s - 405;
  } else {
    wfd = 0.0;
  }
  return norm * wfd;
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
};

template <int G>
__global__ void __launch_bounds__(256) k_mp_rhosum(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int i = a.ilist[row];
  const double4 xi = a.xf[i];
  const int it = a.ty[i];
  const int dim = a.dim;
  double acc = 0.0;
  for (int k = a.off[row] + lane; k < a.off[row + 1]; k += G) {
    const int j = a.nbr[k];
    const double4 xj = a.xf[j];
    const int jt = a.ty[j];
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    if (rsq < c->rcutsq[it * nt1 + jt]) {
      const double ih = 1.0 / c->rcut[it * nt1 + jt];
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

// p = B (pow(rho/rho0, gamma) - rbackground), pair_sph_taitwater_multiphase.cpp:289-292
__device__ __forceinline__ double mp_pressure(double B, double rho0, double gamma, double rbg,
                                              double rho) {
  return B * (pow(rho / rho0, gamma) - rbg);
}

template <int G>
__global__ void __launch_bounds__(256) k_mp_tait(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int i = a.ilist[row];
  const double4 xi = a.xf[i], vi = a.vr[i];
  const int it = a.ty[i];
  const double rhoi = vi.w;
  const double pi = mp_pressure(c->B[it], c->rho0[it], c->gamma[it], c->rbg[it], rhoi);
  const double Vi = a.rm[i] / rhoi;
  const double Vi2 = Vi * Vi;
  double fx = 0.0, fy = 0.0, fz = 0.0;
  for (int k = a.off[row] + lane; k < a.off[row + 1]; k += G) {
    const int j = a.nbr[k];
    const double4 xj = a.xf[j], vj = a.vr[j];
    const int jt = a.ty[j];
    const int p = it * nt1 + jt;
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    if (!(rsq < c->tcutsq[p])) continue;
    const double ih = 1.0 / c->tcut[p];
    const double r = sqrt(rsq);
    double wfd;
    if (a.dim == 3) wfd = quintic_dw(3, r * ih) * ih * ih * ih * ih / r;
    else wfd = quintic_dw(2, r * ih) * ih * ih * ih / r;
    const double rhoj = vj.w;
    const double Vj = a.rm[j] / rhoj;
    const double Vj2 = Vj * Vj;
    // reference quirk kept: p_j with gamma[itype] (pair_sph_taitwater_multiphase.cpp:148)
    const double pj = mp_pressure(c->B[jt], c->rho0[jt], c->gamma[it], c->rbg[jt], rhoj);
    const double pij = (rhoj * pi + rhoi * pj) / (rhoi + rhoj);
    const double velx = vi.x - vj.x, vely = vi.y - vj.y, velz = vi.z - vj.z;
    const double fvisc = (Vi2 + Vj2) * c->tvisc[p] * wfd;
    const double fpair = -(Vi2 + Vj2) * pij * wfd;
    const double tx = dx * fpair + velx * fvisc;
    const double ty_ = dy * fpair + vely * fvisc;
    const double tz = dz * fpair + velz * fvisc;
    fx += tx;
    fy += ty_;
    fz += tz;
    if (a.half && (a.newton || j < a.nlocal) && !(a.exp & 1)) {
      atomicAdd(&a.fo[j].x, -tx);
      atomicAdd(&a.fo[j].y, -ty_);
      atomicAdd(&a.fo[j].z, -tz);
    }
  }
  fx = group_sum<G>(fx);
  fy = group_sum<G>(fy);
  fz = group_sum<G>(fz);
  if (lane == 0) {
    if (a.half) {
      atomicAdd(&a.fo[i].x, fx);
      atomicAdd(&a.fo[i].y, fy);
      atomicAdd(&a.fo[i].z, fz);
    } else {
      a.fo[i].x += fx;
      a.fo[i].y += fy;
      a.fo[i].z += fz;
    }
  }
}

template <int G>
__global__ void __launch_bounds__(256) k_mp_heat(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int i = a.ilist[row];
  const double4 xi = a.xf[i];
  const int it = a.ty[i];
  const double rhoi = a.vr[i].w;
  const double mi = a.rm[i];
  const double Ti0 = a.en[i] / a.cv[i];   // sph_energy2t, sph_energy_equation.cpp:16-18
  double dE = 0.0;
  for (int k = a.off[row] + lane; k < a.off[row + 1]; k += G) {
    const int j = a.nbr[k];
    const double4 xj = a.xf[j];
    const int jt = a.ty[j];
    const int p = it * nt1 + jt;
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    if (!(rsq < c->hcutsq[p])) continue;
    const double ih = 1.0 / c->hcut[p];
    double wfd;
    if (a.dim == 3) {
      wfd = quintic_dw(3, sqrt(rsq) * ih);
      wfd = wfd * ih * ih * ih * ih / sqrt(rsq);
    } else {
      wfd = quintic_dw(2, sqrt(rsq) * ih);
      wfd = wfd * ih * ih * ih / sqrt(rsq);
    }
    double Ti = Ti0;
    double Tj = a.en[j] / a.cv[j];
    const int ff = c->hfix[p];
    if (ff == it && Ti < Tj) Ti = c->htc[p];
    if (ff == jt && Tj < Ti) Tj = c->htc[p];
    const double deltaE = 2.0 * c->halpha[p] * (Ti - Tj) * wfd / (rhoi * a.vr[j].w);
    dE += deltaE * a.rm[j];
    if (a.half && (a.newton || j < a.nlocal)) atomicAdd(&a.de[j], -deltaE * mi);
  }
  dE = group_sum<G>(dE);
  if (lane == 0) {
    if (a.half) atomicAdd(&a.de[i], dE);
    else a.de[i] += dE;
  }
}

template <int G>
__global__ void __launch_bounds__(256) k_mp_colorgradient(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int i = a.ilist[row];
  const double4 xi = a.xf[i];
  const int it = a.ty[i];
  const double sigmai = a.vr[i].w / a.rm[i];
  double gx = 0.0, gy = 0.0, gz = 0.0;
  for (int k = a.off[row] + lane; k < a.off[row + 1]; k += G) {
    const int j = a.nbr[k];
    const double4 xj = a.xf[j];
    const int jt = a.ty[j];
    const int p = it * nt1 + jt;
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    if (!(rsq < c->ccutsq[p])) continue;
    const double r = sqrt(rsq);
    const double ih = 1.0 / c->ccut[p];
    double wfd;
    if (a.dim == 3) wfd = quintic_dw(3, r * ih) * ih * ih * ih * ih;
    else wfd = quintic_dw(2, r * ih) * ih * ih * ih;
    const double sigmaj = a.vr[j].w / a.rm[j];
    const double dphi = -wfd * c->calpha[p] / (sigmaj * sigmaj) * sigmai;
    gx += dphi * (dx / r);
    gy += dphi * (dy / r);
    if (a.dim == 3) gz += dphi * (dz / r);
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
  if (dim == 2)
    return make_double3(
        (e.x * ((c.y * c.y + c.x * c.x) / 2 - c.x * c.x) - c.x * e.y * c.y) / absc,
        (e.y * ((c.y * c.y + c.x * c.x) / 2 - c.y * c.y) - e.x * c.x * c.y) / absc, 0.0);
  return make_double3(
      (e.x * (0.3333333333333333 * c.z * c.z + 0.3333333333333333 * c.y * c.y -
              0.6666666666666666 * c.x * c.x) -
       1.0 * c.x * e.z * c.z - 1.0 * c.x * e.y * c.y) / absc,
      (e.y * (0.3333333333333333 * c.z * c.z - 0.6666666666666666 * c.y * c.y +
              0.3333333333333333 * c.x * c.x) -
       1.0 * c.y * e.z * c.z - 1.0 * e.x * c.x * c.y) / absc,
      (e.z * (-0.6666666666666666 * c.z * c.z + 0.3333333333333333 * c.y * c.y +
              0.3333333333333333 * c.x * c.x) -
       1.0 * e.y * c.y * c.z - 1.0 * e.x * c.x * c.z) / absc);
}
__device__ __forceinline__ double st_abs(int dim, double4 c) {
  return dim == 3 ? sqrt(c.x * c.x + c.y * c.y + c.z * c.z) : sqrt(c.x * c.x + c.y * c.y);
}

// sph/surfacetension: F = (S_i V_i^2 + S_j V_j^2) dW_quintic, V = rmass/rho; i gets +F, j
// gets -F on a half list (newton_pair or j < nlocal), like the reference.
template <int G>
__global__ void __launch_bounds__(256) k_mp_surface(MpArgs a) {
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= a.inum) return;
  const MpCoefs *c = a.mc;
  const int nt1 = c->ntypes + 1;
  const int dim = a.dim;
  const int i = a.ilist[row];
  const double4 xi = a.xf[i];
  const int it = a.ty[i];
  const double4 cgi = a.cgi[i];
  const double abscgi = st_abs(dim, cgi);
  const double Vi = a.rm[i] / a.vr[i].w;
  double fx = 0.0, fy = 0.0, fz = 0.0;
  for (int k = a.off[row] + lane; k < a.off[row + 1]; k += G) {
    const int j = a.nbr[k];
    const double4 xj = a.xf[j];
    const int jt = a.ty[j];
    const int p = it * nt1 + jt;
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    if (!(rsq < c->scutsq[p])) continue;
    const double ih = 1.0 / c->scut[p];
    const double r = sqrt(rsq);
    const double wfd = (dim == 3) ? quintic_dw(3, r * ih) * ih * ih * ih * ih
                                  : quintic_dw(2, r * ih) * ih * ih * ih;
    const double3 e = make_double3(dx / r, dy / r, dim == 3 ? dz / r : 0.0);
    const double4 cgj = a.cgi[j];
    const double3 Si = st_vector(dim, cgi, abscgi, e);
    const double3 Sj = st_vector(dim, cgj, st_abs(dim, cgj), e);
    const double Vj = a.rm[j] / a.vr[j].w;
    const double tx = (Si.x * Vi * Vi + Sj.x * Vj * Vj) * wfd;
    const double ty_ = (Si.y * Vi * Vi + Sj.y * Vj * Vj) * wfd;
    const double tz = dim == 3 ? (Si.z * Vi * Vi + Sj.z * Vj * Vj) * wfd : 0.0;
    fx += tx;
    fy += ty_;
    fz += tz;
    if (a.half && (a.newton || j < a.nlocal) && !(a.exp & 1)) {
      atomicAdd(&a.fo[j].x, -tx);
      atomicAdd(&a.fo[j].y, -ty_);
      if (dim == 3) atomicAdd(&a.fo[j].z, -tz);
    }
  }
  fx = group_sum<G>(fx);
  fy = group_sum<G>(fy);
  fz = group_sum<G>(fz);
  if (lane == 0) {
    if (a.half) {
      atomicAdd(&a.fo[i].x, fx);
      atomicAdd(&a.fo[i].y, fy);
      atomicAdd(&a.fo[i].z, fz);
    } else {
      a.fo[i].x += fx;
      a.fo[i].y += fy;
      a.fo[i].z += fz;
    }
  }
}

}  // namespace sph
