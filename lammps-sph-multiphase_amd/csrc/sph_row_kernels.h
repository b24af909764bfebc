// sph_row_kernels.h -- the engine's CSR-row pair passes (full list, gather only).
//
// Same arithmetic as k_rhosum / k_force in sph_kernels.h (which also serve the pair-style
// layer's half lists, virial and accumulate modes), specialised for the device-resident
// engine: full list, no virial, no accumulate, gravity fused.  The pair body is
// branch-free -- a pair outside the cutoff (or a padding lane past the row's end) gets
// its kernel-derivative weight selected to 0, which zeroes every term it feeds -- so the
// U unrolled pairs of a lane form one basic block whose dependency chains (v_rsq/v_rcp
// seeds + Newton steps) the scheduler can interleave, instead of U branch-separated
// blocks executed one after the other.
#pragma once
#include <hip/hip_runtime.h>

#include "sph_kernels.h"

namespace sph {

template <int G, int U, bool NT1>
__global__ void __launch_bounds__(256)
k_row_rhosum(int n, const int *__restrict__ off, const int *__restrict__ nbr,
             double4 *__restrict__ xf, const int *__restrict__ ty, double4 *__restrict__ vr,
             const Coefs *__restrict__ cf) {
  __shared__ RhoPair s_c[NT1 ? 1 : NT2];
  const int nt1 = cf->ntypes + 1;
  if (!NT1) {
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_c[t] = cf->rho[t];
    __syncthreads();
  }
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= n) return;
  const double4 xi = xf[row];
  const int it = NT1 ? 1 : ty[row];
  const RhoPair c1 = NT1 ? cf->rho[3] : RhoPair{};
  const int beg = off[row], end = off[row + 1];
  double acc = 0.0;
  for (int k0 = beg + lane; k0 < end; k0 += G * U) {
    int jv[U];
#pragma unroll
    for (int u = 0; u < U; u++) jv[u] = nbr[min(k0 + u * G, end - 1)];
    double4 xj[U];
    int tj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      xj[u] = xf[jv[u]];
      tj[u] = NT1 ? 1 : ty[jv[u]];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const RhoPair c = NT1 ? c1 : s_c[it * nt1 + tj[u]];
      double wf = 1.0 - rsq * c.ihsq;
      wf = wf * wf;
      wf = wf * wf;
      acc += (k0 + u * G < end && rsq < c.cutsq) ? c.mK * wf : 0.0;
    }
  }
  acc = group_sum<G>(acc);
  if (lane == 0) {
    const double rho = cf->self_rho[it] + acc;
    vr[row].w = rho;
    xf[row].w = tait_p_over_rho2(rho, cf->rho0[it], cf->B[it]);
  }
}

template <int G, int U, int VISC, int MODE, bool NT1>
__global__ void __launch_bounds__(256)
k_row_force(int n, const int *__restrict__ off, const int *__restrict__ nbr,
            const double4 *__restrict__ xf, const double4 *__restrict__ vr,
            const int *__restrict__ ty, const double *__restrict__ en,
            const Coefs *__restrict__ cf, double4 *__restrict__ fo, double *__restrict__ de,
            double gx, double gy, double gz) {
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  __shared__ TaitPair s_t[(TAIT && !NT1) ? NT2 : 1];
  __shared__ HeatPair s_h[(HEAT && !NT1) ? NT2 : 1];
  const int nt1 = cf->ntypes + 1;
  if (!NT1) {
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
      if (TAIT) s_t[t] = cf->tait[t];
      if (HEAT) s_h[t] = cf->heat[t];
    }
    __syncthreads();
  }
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= n) return;
  const double4 xi = xf[row];
  const double4 vi = vr[row];
  const double ei = HEAT ? en[row] : 0.0;
  const int it = NT1 ? 1 : ty[row];
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  const int beg = off[row], end = off[row + 1];
  double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
  for (int k0 = beg + lane; k0 < end; k0 += G * U) {
    int jv[U];
#pragma unroll
    for (int u = 0; u < U; u++) jv[u] = nbr[min(k0 + u * G, end - 1)];
    double4 xj[U], vj[U];
    double ej[U];
    int tj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      xj[u] = xf[jv[u]];
      vj[u] = vr[jv[u]];
      ej[u] = HEAT ? en[jv[u]] : 0.0;
      tj[u] = NT1 ? 1 : ty[jv[u]];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const int pidx = NT1 ? 3 : it * nt1 + tj[u];
      const bool ok = k0 + u * G < end;
      const double r = fast_sqrt(rsq);
      if (TAIT) {
        const TaitPair c = NT1 ? t1 : s_t[pidx];
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        wfd = (ok && rsq < c.cutsq) ? wfd : 0.0;   // zeroes every term below
        const double velx = vi.x - vj[u].x, vely = vi.y - vj[u].y, velz = vi.z - vj[u].z;
        const double dvdr = dx * velx + dy * vely + dz * velz;
        if (VISC == SPH_VISC_MONAGHAN) {
          const double q = (c.viscC * dvdr) * fast_rcp((rsq + c.eps) * (vi.w + vj[u].w));
          const double fvisc = dvdr < 0. ? q : 0.0;
          const double fpair = c.mm * (xi.w + xj[u].w + fvisc) * wfd;
          fx += dx * fpair;
          fy += dy * fpair;
          fz += dz * fpair;
          dE += -0.5 * fpair * dvdr;
        } else {
          double fvisc = c.viscC * fast_rcp(vi.w * vj[u].w);
          fvisc *= (-c.mm) * wfd;
          const double fpair = c.mm * (xi.w + xj[u].w) * wfd;
          fx += dx * fpair + velx * fvisc;
          fy += dy * fpair + vely * fvisc;
          fz += dz * fpair + velz * fvisc;
          dE += -0.5 * (fpair * dvdr + fvisc * (velx * velx + vely * vely + velz * velz));
        }
        drho += c.mj * dvdr * wfd;
      }
      if (HEAT) {
        const HeatPair c = NT1 ? h1 : s_h[pidx];
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        wfd = (ok && rsq < c.cutsq) ? wfd : 0.0;
        double deltaE = c.hmD;
        deltaE *= (vi.w + vj[u].w) * fast_rcp(vi.w * vj[u].w);
        deltaE *= (ei - ej[u]) * wfd;
        dE += deltaE;
      }
    }
  }
  if (TAIT) {
    fx = group_sum<G>(fx);
    fy = group_sum<G>(fy);
    fz = group_sum<G>(fz);
    drho = group_sum<G>(drho);
  }
  dE = group_sum<G>(dE);
  if (lane == 0) {
    if (TAIT) {
      const double m = cf->mass[it];
      fo[row] = make_double4(fx + m * gx, fy + m * gy, fz + m * gz, drho);
    }
    de[row] = dE;
  }
}

}  // namespace sph

namespace sph {

// (G lanes per row, U unrolled pairs per lane) of the engine's row kernels; SPH_ROWTILE
// env var (tuning) picks one of the instantiated shapes, default 8x4.
int row_tile();

struct RowArgs {
  int n;
  const int *off, *nbr;
  double4 *xf, *vr;
  const int *ty;
  const double *en;
  const Coefs *cf;
  double4 *fo;
  double *de;
  double gx, gy, gz;
};

template <int G, int U>
inline void row_rhosum_gu(bool nt1, hipStream_t s, const RowArgs &a) {
  const int grid = (int)(((long long)a.n * G + 255) / 256);
  if (grid == 0) return;
  if (nt1)
    hipLaunchKernelGGL((k_row_rhosum<G, U, true>), dim3(grid), dim3(256), 0, s, a.n, a.off,
                       a.nbr, a.xf, a.ty, a.vr, a.cf);
  else
    hipLaunchKernelGGL((k_row_rhosum<G, U, false>), dim3(grid), dim3(256), 0, s, a.n, a.off,
                       a.nbr, a.xf, a.ty, a.vr, a.cf);
}

template <int G, int U, int VISC, int MODE, bool NT1>
inline void row_force_t(hipStream_t s, const RowArgs &a) {
  const int grid = (int)(((long long)a.n * G + 255) / 256);
  if (grid == 0) return;
  hipLaunchKernelGGL((k_row_force<G, U, VISC, MODE, NT1>), dim3(grid), dim3(256), 0, s, a.n,
                     a.off, a.nbr, a.xf, a.vr, a.ty, a.en, a.cf, a.fo, a.de, a.gx, a.gy, a.gz);
}

template <int G, int U, bool NT1>
inline void row_force_n(int visc, int mode, hipStream_t s, const RowArgs &a) {
  const bool mor = visc == SPH_VISC_MORRIS;
  switch (mode) {
    case M_TAIT:
      if (mor) row_force_t<G, U, 1, M_TAIT, NT1>(s, a);
      else row_force_t<G, U, 0, M_TAIT, NT1>(s, a);
      break;
    case M_TAIT | M_HEAT:
      if (mor) row_force_t<G, U, 1, M_TAIT | M_HEAT, NT1>(s, a);
      else row_force_t<G, U, 0, M_TAIT | M_HEAT, NT1>(s, a);
      break;
    default: row_force_t<G, U, 0, M_HEAT, NT1>(s, a); break;
  }
}

template <int G, int U>
inline void row_force_gu(bool nt1, int visc, int mode, hipStream_t s, const RowArgs &a) {
  if (nt1) row_force_n<G, U, true>(visc, mode, s, a);
  else row_force_n<G, U, false>(visc, mode, s, a);
}

#define SPH_ROW_TILES(X) X(0, 8, 4) X(1, 4, 4) X(2, 8, 2) X(3, 16, 2) X(4, 4, 8) X(5, 8, 8)

inline void row_rhosum(bool nt1, hipStream_t s, const RowArgs &a) {
  switch (row_tile()) {
#define SPH_CASE(k, G, U) \
  case k: row_rhosum_gu<G, U>(nt1, s, a); break;
    SPH_ROW_TILES(SPH_CASE)
#undef SPH_CASE
    default: row_rhosum_gu<8, 4>(nt1, s, a); break;
  }
}

inline void row_force(bool nt1, int visc, int mode, hipStream_t s, const RowArgs &a) {
  switch (row_tile()) {
#define SPH_CASE(k, G, U) \
  case k: row_force_gu<G, U>(nt1, visc, mode, s, a); break;
    SPH_ROW_TILES(SPH_CASE)
#undef SPH_CASE
    default: row_force_gu<8, 4>(nt1, visc, mode, s, a); break;
  }
}

}  // namespace sph
