// sph_kernels.h -- gfx950 kernels of the USER-SPH pair engine.
//
// Layout in HBM (all fp64; one record per atom, owned atoms first, ghosts after):
//   xt[i]  = {x, y, z, type}   double4 (type stored as the integer bit pattern of .w)
//   vr[i]  = {vx, vy, vz, rho} double4 (v = atom->vest, the extrapolated velocity)
//   aux[i] = {p/rho^2, e}      double2 (Tait pressure term of i, internal energy)
// Output of the force pass (owned rows): fo[i] = {fx, fy, fz, drho} double4, de[i].
//
// Every pair kernel walks a CSR neighbor list with a G-lane group per row (G in
// {1,2,4,8,16,32,64}, a power of two dividing the 64-lane wave), accumulates the row in
// registers and reduces across the group with xor-shuffles.  A FULL list is walked
// gather-only: each pair is evaluated from both sides, so no atomics and no reverse
// communication are needed and results are deterministic.  A HALF list (LAMMPS' default
// request) is walked with the reference's Newton-3 scatter onto j, done with fp64
// hardware atomics.  No MFMA: the work is an irregular gather, bounded by memory and
// fp64 VALU, not by dense contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sph_hip.h"

namespace sph {

constexpr int MAXT = SPH_MAXTYPES;
constexpr int NT2 = (MAXT + 1) * (MAXT + 1);

// per type-pair coefficient records (index it*(ntypes+1)+jt)
struct RhoPair {   // sph/rhosum, quadric kernel (pair_sph_rhosum.cpp:172-192)
  double cutsq, ihsq, mK;  // mK = mass[jt] * norm * ihsq * ih (3d) | norm * ihsq (2d)
};
struct TaitPair {  // sph/taitwater[/morris], Lucy kernel (pair_sph_taitwater.cpp:136-191)
  double cutsq, h, wK, mm, mj, mi, viscC, eps;
  // wK = -25.0669..*ihsq^3*ih (3d) | -19.0986..*ihsq^3 (2d); mm = -mass[it]*mass[jt]
  // viscC = -visc*(c_i+c_j) (Monaghan) | 2*visc (Morris); eps = 0.01*h*h
};
struct HeatPair {  // sph/heatconduction (pair_sph_heatconduction.cpp:103-129)
  double cutsq, h, wK, hmD;  // hmD = 2 m_i m_j/(m_i+m_j) * alpha
};

struct Coefs {
  int ntypes, dim;
  double self_rho[MAXT + 1];   // mass[t] * norm / h_tt^3 (pair_sph_rhosum.cpp:116-138)
  double rho0[MAXT + 1], B[MAXT + 1], mass[MAXT + 1];
  RhoPair rho[NT2];
  TaitPair tait[NT2];
  HeatPair heat[NT2];
  double cutneighsq[NT2];
};

__device__ __forceinline__ int type_of(double w) { return (int)__double_as_longlong(w); }
__host__ __device__ __forceinline__ double type_bits(int t) {
#ifdef __HIP_DEVICE_COMPILE__
  return __longlong_as_double((long long)t);
#else
  union { long long l; double d; } u;
  u.l = (long long)t;
  return u.d;
#endif
}

template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
  for (int m = G >> 1; m > 0; m >>= 1) v += __shfl_xor(v, m, G);
  return v;
}
template <int G>
__device__ __forceinline__ int group_sum_i(int v) {
#pragma unroll
  for (int m = G >> 1; m > 0; m >>= 1) v += __shfl_xor(v, m, G);
  return v;
}

// Tait EOS pressure term P/rho^2 with gamma = 7, in the reference's operation order
// (pair_sph_taitwater.cpp:117-120).
__device__ __forceinline__ double tait_p_over_rho2(double rho, double rho0, double B) {
  double tmp = rho / rho0;
  double fi = tmp * tmp * tmp;
  return B * (fi * fi * tmp - 1.0) / (rho * rho);
}

// ------------------------------------------------------------------------------------
// sph/rhosum over a list (gather only, exactly like the reference which never scatters)
// EOS: also store p/rho^2 of i into aux[i].x (engine path, fused epilogue).
// ------------------------------------------------------------------------------------
template <int G, int DIM, bool EOS>
__global__ void __launch_bounds__(256)
k_rhosum(int inum, const int *__restrict__ ilist, const int *__restrict__ off,
         const int *__restrict__ nbr, const double4 *__restrict__ xt,
         double4 *__restrict__ vr, double2 *__restrict__ aux, double *__restrict__ rho_out,
         const Coefs *__restrict__ cf) {
  __shared__ RhoPair s_c[NT2];
  __shared__ double s_self[MAXT + 1], s_rho0[MAXT + 1], s_B[MAXT + 1];
  const int nt1 = cf->ntypes + 1;
  for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_c[t] = cf->rho[t];
  for (int t = threadIdx.x; t < nt1; t += blockDim.x) {
    s_self[t] = cf->self_rho[t];
    s_rho0[t] = cf->rho0[t];
    s_B[t] = cf->B[t];
  }
  __syncthreads();
  const int row = (int)((blockIdx.x * (unsigned)blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= inum) return;
  const int i = ilist ? ilist[row] : row;
  const double4 xi = xt[i];
  const int it = type_of(xi.w);
  const RhoPair *crow = s_c + it * nt1;
  const int beg = off[row], end = off[row + 1];
  double acc = 0.0;
  constexpr int U = 4;
  for (int k0 = beg + lane; k0 < end; k0 += G * U) {
    int jv[U];
#pragma unroll
    for (int u = 0; u < U; u++) jv[u] = nbr[min(k0 + u * G, end - 1)];
    double4 xj[U];
#pragma unroll
    for (int u = 0; u < U; u++) xj[u] = xt[jv[u]];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const RhoPair c = crow[type_of(xj[u].w)];
      if (k0 + u * G < end && rsq < c.cutsq) {
        double wf = 1.0 - rsq * c.ihsq;
        wf = wf * wf;
        wf = wf * wf;
        acc += c.mK * wf;
      }
    }
  }
  acc = group_sum<G>(acc);
  if (lane == 0) {
    const double rho = s_self[it] + acc;
    if (rho_out) rho_out[i] = rho;
    if (EOS) {
      vr[i].w = rho;
      aux[i].x = tait_p_over_rho2(rho, s_rho0[it], s_B[it]);
    }
  }
}

// EOS term for a range of atoms (pair-style layer: rho comes from the host)
static __global__ void k_eos(int n, const double4 *__restrict__ xt, const double4 *__restrict__ vr,
                      double2 *__restrict__ aux, const Coefs *__restrict__ cf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = type_of(xt[i].w);
  aux[i].x = tait_p_over_rho2(vr[i].w, cf->rho0[t], cf->B[t]);
}

// ------------------------------------------------------------------------------------
// Force pass: sph/taitwater (VISC=0 Monaghan, 1 Morris) and/or sph/heatconduction.
// MODE bits: TAIT | HEAT | HALF.  FULL lists: overwrite (accum=0) or add (accum=1) the
// owned row's results.  HALF lists: atomics on both i and j (reference scatter).
// ------------------------------------------------------------------------------------
enum { M_TAIT = 1, M_HEAT = 2, M_HALF = 4 };

// neighbors processed per lane per iteration: all U index loads, then all U gathers are
// issued before the first use, so a row costs ~2 dependent memory round trips per U
// neighbors instead of 3 per neighbor (index -> position -> velocity/rho).
constexpr int UNROLL = 4;

// 1/b to ~1 ulp: v_rcp_f64 seed + two Newton steps (no IEEE fix-up path; operands here
// are positive normal numbers).
__device__ __forceinline__ double fast_rcp(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  return fma(y, e, y);
}
// sqrt(x) for x >= 0 (normal or zero) to ~1 ulp: v_rsq_f64 seed + Goldschmidt step +
// correction, without the denormal rescaling of the libm path.
__device__ __forceinline__ double fast_sqrt(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  const double d = fma(-g, g, x);
  g = fma(d, h, g);
  return x > 0.0 ? g : 0.0;
}

template <int G, int DIM, int VISC, int MODE>
__global__ void __launch_bounds__(256)
k_force(int inum, int nlocal, int newton, const int *__restrict__ ilist,
        const int *__restrict__ off, const int *__restrict__ nbr,
        const double4 *__restrict__ xt, const double4 *__restrict__ vr,
        const double2 *__restrict__ aux, double4 *__restrict__ fo, double *__restrict__ de,
        int accum, const Coefs *__restrict__ cf, double gx, double gy, double gz,
        double *__restrict__ virial) {
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  constexpr bool HALF = (MODE & M_HALF) != 0;
  constexpr int U = UNROLL;
  __shared__ TaitPair s_t[TAIT ? NT2 : 1];
  __shared__ HeatPair s_h[HEAT ? NT2 : 1];
  __shared__ double s_mass[MAXT + 1];
  const int nt1 = cf->ntypes + 1;
  for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
    if (TAIT) s_t[t] = cf->tait[t];
    if (HEAT) s_h[t] = cf->heat[t];
  }
  for (int t = threadIdx.x; t < nt1; t += blockDim.x) s_mass[t] = cf->mass[t];
  __syncthreads();
  const int row = (int)((blockIdx.x * (unsigned)blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= inum) return;
  const int i = ilist ? ilist[row] : row;
  const double4 xi = xt[i];
  const double4 vi = vr[i];
  const double2 ai = aux[i];
  const int it = type_of(xi.w);
  const int beg = off[row], end = off[row + 1];
  double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, v5 = 0.0;
  for (int k0 = beg + lane; k0 < end; k0 += G * U) {
    int jv[U];
#pragma unroll
    for (int u = 0; u < U; u++) jv[u] = nbr[min(k0 + u * G, end - 1)];
    double4 xj[U], vj[U];
    double2 aj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      xj[u] = xt[jv[u]];
      vj[u] = vr[jv[u]];
      aj[u] = aux[jv[u]];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int j = jv[u];
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const int pidx = it * nt1 + type_of(xj[u].w);
      const bool ok = k0 + u * G < end;
      bool hit_t = false, hit_h = false;
      if (TAIT) hit_t = ok && rsq < s_t[pidx].cutsq;
      if (HEAT) hit_h = ok && rsq < s_h[pidx].cutsq;
      if (!(hit_t || hit_h)) continue;
      const double r = fast_sqrt(rsq);
      double jfx = 0.0, jfy = 0.0, jfz = 0.0, jdrho = 0.0, jdE = 0.0;
      if (TAIT && hit_t) {
        const TaitPair c = s_t[pidx];
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        const double velx = vi.x - vj[u].x, vely = vi.y - vj[u].y, velz = vi.z - vj[u].z;
        const double dvdr = dx * velx + dy * vely + dz * velz;
        double fpair, deltaE, fvx = 0.0, fvy = 0.0, fvz = 0.0;
        if (VISC == SPH_VISC_MONAGHAN) {
          // mu = h dvdr/(rsq+0.01h^2); fvisc = -visc (c_i+c_j) mu/(rho_i+rho_j), dvdr < 0
          const double q = (c.viscC * c.h * dvdr) * fast_rcp((rsq + c.eps) * (vi.w + vj[u].w));
          const double fvisc = dvdr < 0. ? q : 0.0;
          fpair = c.mm * (ai.x + aj[u].x + fvisc) * wfd;
          deltaE = -0.5 * fpair * dvdr;
        } else {
          // fvisc = 2 visc/(rho_i rho_j) * m_i m_j wfd
          double fvisc = c.viscC * fast_rcp(vi.w * vj[u].w);
          fvisc *= (-c.mm) * wfd;
          fpair = c.mm * (ai.x + aj[u].x) * wfd;
          deltaE = -0.5 * (fpair * dvdr + fvisc * (velx * velx + vely * vely + velz * velz));
          fvx = velx * fvisc;
          fvy = vely * fvisc;
          fvz = velz * fvisc;
        }
        const double tx = dx * fpair + fvx, ty = dy * fpair + fvy, tz = dz * fpair + fvz;
        fx += tx;
        fy += ty;
        fz += tz;
        drho += c.mj * dvdr * wfd;
        dE += deltaE;
        if (HALF) {
          jfx = -tx;
          jfy = -ty;
          jfz = -tz;
          jdrho = c.mi * dvdr * wfd;
          jdE = deltaE;
        }
        if (virial) {
          const double s = (!HALF || newton || j < nlocal) ? 1.0 : 0.5;
          const double sf = HALF ? s * fpair : 0.5 * fpair;
          v0 += sf * dx * dx;
          v1 += sf * dy * dy;
          v2 += sf * dz * dz;
          v3 += sf * dx * dy;
          v4 += sf * dx * dz;
          v5 += sf * dy * dz;
        }
      }
      if (HEAT && hit_h) {
        // 2 m_i m_j/(m_i+m_j) (rho_i+rho_j)/(rho_i rho_j) D (e_i-e_j) wfd
        const HeatPair c = s_h[pidx];
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        double deltaE = c.hmD;
        deltaE *= (vi.w + vj[u].w) * fast_rcp(vi.w * vj[u].w);
        deltaE *= (ai.y - aj[u].y) * wfd;
        dE += deltaE;
        if (HALF) jdE -= deltaE;
      }
      if (HALF && (newton || j < nlocal)) {
        if (TAIT) {
          atomicAdd(&fo[j].x, jfx);
          atomicAdd(&fo[j].y, jfy);
          atomicAdd(&fo[j].z, jfz);
          atomicAdd(&fo[j].w, jdrho);
        }
        atomicAdd(&de[j], jdE);
      }
    }
  }
  if (TAIT) {
    fx = group_sum<G>(fx);
    fy = group_sum<G>(fy);
    fz = group_sum<G>(fz);
    drho = group_sum<G>(drho);
    if (virial) {
      v0 = group_sum<G>(v0);
      v1 = group_sum<G>(v1);
      v2 = group_sum<G>(v2);
      v3 = group_sum<G>(v3);
      v4 = group_sum<G>(v4);
      v5 = group_sum<G>(v5);
    }
  }
  dE = group_sum<G>(dE);
  if (lane == 0) {
    if (HALF) {
      if (TAIT) {
        atomicAdd(&fo[i].x, fx);
        atomicAdd(&fo[i].y, fy);
        atomicAdd(&fo[i].z, fz);
        atomicAdd(&fo[i].w, drho);
      }
      atomicAdd(&de[i], dE);
    } else {
      if (TAIT) {
        const double m = s_mass[it];
        double4 o = make_double4(fx + m * gx, fy + m * gy, fz + m * gz, drho);
        if (accum) {
          const double4 p = fo[i];
          o.x += p.x;
          o.y += p.y;
          o.z += p.z;
          o.w += p.w;
        }
        fo[i] = o;
      }
      de[i] = accum ? de[i] + dE : dE;
    }
    if (TAIT && virial) {
      atomicAdd(&virial[0], v0);
      atomicAdd(&virial[1], v1);
      atomicAdd(&virial[2], v2);
      atomicAdd(&virial[3], v3);
      atomicAdd(&virial[4], v4);
      atomicAdd(&virial[5], v5);
    }
  }
}

}  // namespace sph
