// sph_kernels.h -- gfx950 pair kernels of the USER-SPH engine (CSR neighbor-list walk).
//
// Layout in HBM (fp64; owned atoms first, ghosts after; a 64-B position/velocity pair of
// records per atom so a neighbor costs two 32-B gathers):
//   xf[i] = {x, y, z, p/rho^2}   double4   (p/rho^2 = Tait pressure term, written by the
//                                           rhosum epilogue or k_eos)
//   vr[i] = {vx, vy, vz, rho}    double4   (v = atom->vest, the extrapolated velocity)
//   ty[i] = type (int32), en[i] = e (double, heat conduction only)
// Output of the force pass: fo[i] = {fx, fy, fz, drho} double4, de[i].
//
// Every kernel walks a CSR list with a G-lane group per row (G a power of two dividing the
// 64-lane wave), issues UNROLL neighbors' index loads and gathers before first use,
// accumulates in registers and reduces across the group with xor-shuffles.  A FULL list
// is walked gather-only (each pair evaluated from both sides: no atomics, no reverse
// communication, deterministic).  A HALF list (LAMMPS' default request) is walked with
// the reference's Newton-3 scatter onto j via fp64 hardware atomics.  NT1 specialises the
// single-type case (coefficients in registers, no type gathers).  Workgroups are remapped
// so that each XCD (own 4 MB L2) sweeps a contiguous, spatially compact range of rows.
// No MFMA: the work is an irregular gather, bounded by cache bandwidth and fp64 VALU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sph_hip.h"

namespace sph {

constexpr int MAXT = SPH_MAXTYPES;
constexpr int NT2 = (MAXT + 1) * (MAXT + 1);
// typed neighbour-list entries: atom index below bit 28, type-1 in bits 28-30 (row2_fits
// bounds nall by 2^26; SPH_MAXTYPES = 8 needs 3 bits)
#define SPH_TBIT_SHIFT 28
#define SPH_TBIT_MASK 0x0FFFFFFF
static_assert(MAXT - 1 < 8, "type bits hold 3 bits");

// per type-pair coefficient records (index it*(ntypes+1)+jt)
struct RhoPair {   // sph/rhosum, quadric kernel (pair_sph_rhosum.cpp:172-192)
  double cutsq, ihsq, mK;  // mK = mass[jt] * norm * ihsq * ih (3d) | norm * ihsq (2d)
};
struct TaitPair {  // sph/taitwater[/morris], Lucy kernel (pair_sph_taitwater.cpp:136-191)
  double cutsq, h, wK, mm, mj, mi, viscC, eps;
  // wK = -25.0669..*ihsq^3*ih (3d) | -19.0986..*ihsq^3 (2d); mm = -mass[it]*mass[jt]
  // viscC = -visc*(c_i+c_j)*h (Monaghan) | 2*visc (Morris); eps = 0.01*h*h
};
struct HeatPair {  // sph/heatconduction (pair_sph_heatconduction.cpp:103-129)
  double cutsq, h, wK, hmD;  // hmD = 2 m_i m_j/(m_i+m_j) * alpha
};

struct Coefs {
  int ntypes, dim;
  // bit t: sph/rhosum has no coefficients for type t, so under hybrid/overlay its rows are
  // on the skip list (pair_hybrid.cpp:439-471, neigh_derive.cpp:186) and keep their rho
  int rho_keep;
  double self_rho[MAXT + 1];   // mass[t] * norm / h_tt^3 (pair_sph_rhosum.cpp:116-138)
  // mass: the body-force (fix gravity) mass of type t -- 0 for types outside the fix's group
  double rho0[MAXT + 1], B[MAXT + 1], mass[MAXT + 1];
  RhoPair rho[NT2];
  TaitPair tait[NT2];
  HeatPair heat[NT2];
  double cutneighsq[NT2];
  double cutinsq[NT2];     // (cut + inner margin)^2 of the block path's inner rows
  double fcutsq[NT2];  // engine: max cutsq of the enabled force styles (tight-list test)
};

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, dispatch): give
// each XCD a contiguous range of logical blocks so neighboring rows share one L2.
// Bijective for any grid size (cdna_hip_programming.md, "XCD swizzle must be bijective").
__device__ __forceinline__ unsigned xcd_block() {
  const unsigned nwg = gridDim.x, orig = blockIdx.x;
  const unsigned q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Entry slot (0..G-1) of lane l in each G-entry group of a row2 chunk.  pi = 0: slot l.
// pi = 1 (pair-interleaved, for lane-pair gathers): lane 2p takes slot p and lane 2p+1
// slot G/2 + p, so the lane-pair load that fetches the even lanes' records covers the G/2
// CONSECUTIVE entries 0..G/2-1 (mostly consecutive atoms: fewer distinct 128-B lines)
// and the odd lanes' load the next G/2, instead of both striding over all G.
template <int G>
__host__ __device__ __forceinline__ int entry_slot(int l, int pi) {
  return pi ? (l & 1) * (G / 2) + (l >> 1) : l;
}
__host__ __device__ __forceinline__ int slot_lane(int m, int G, int pi) {
  return pi ? 2 * (m % (G / 2)) + m / (G / 2) : m;
}
// Storage position of entry q of a neighbor row in the chunk-transposed layout of the
// strided engine list (chunks of 4G entries; entry u*G + m of a chunk, taken by lane
// l = slot_lane(m), at 4l + u), so the row2 kernels' lane l loads its four entries of a
// chunk with one 16-B load.
__host__ __device__ __forceinline__ int tpos(int q, int G, int pi) {
  const int c = q % (4 * G);
  return q - c + 4 * slot_lane(c % G, G, pi) + c / G;
}

// rsq in the reference's operation order and rounding (its x86-64 build has no FMA, so no
// contraction: neigh_full.cpp:305-312), for the neighbour-list membership test
// rsq <= cutneighsq -- bit-exact also for atoms on a lattice, whose distances tie with the
// cutoff
__device__ __forceinline__ double rsq_ref(double dx, double dy, double dz) {
#pragma clang fp contract(off)
  return dx * dx + dy * dy + dz * dz;
}

// sqrt(x), correctly rounded for normal x > ~1e-290: LLVM's f64 sqrt sequence (a v_rsq_f64
// seed, one Goldschmidt step, two residual corrections) without the rescaling it adds for
// tiny arguments -- r for the quintic's s = 3 r / h, which must be the reference's sqrt(rsq)
// to the last bit; *hh = ~0.5 / sqrt(x) from the same refinement
__device__ __forceinline__ double cr_sqrt(double x, double *hh = nullptr) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double e = fma(-h, g, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  if (hh) *hh = h;
  return fma(d, h, g);
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
template <int G>
__device__ __forceinline__ int group_min_i(int v) {
#pragma unroll
  for (int m = G >> 1; m > 0; m >>= 1) v = min(v, __shfl_xor(v, m, G));
  return v;
}

// Tait EOS pressure term P/rho^2 with gamma = 7, in the reference's operation order
// (pair_sph_taitwater.cpp:117-120).
__device__ __forceinline__ double tait_p_over_rho2(double rho, double rho0, double B) {
  double tmp = rho / rho0;
  double fi = tmp * tmp * tmp;
  return B * (fi * fi * tmp - 1.0) / (rho * rho);
}

// 1/b to ~1 ulp: v_rcp_f64 seed + two Newton steps (operands are positive normals).
__device__ __forceinline__ double fast_rcp(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  return fma(y, e, y);
}
// sqrt(x), x >= 0 normal or zero, to ~1 ulp: v_rsq_f64 seed + Goldschmidt step +
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

constexpr int UNROLL = 4;

// ------------------------------------------------------------------------------------
// sph/rhosum over a list (gather only, as the reference, which never scatters)
// EOS: also store p/rho^2 of i (engine path, fused epilogue) and rho into vr[i].w.
// ------------------------------------------------------------------------------------
template <int G, int DIM, bool EOS, bool NT1>
__global__ void __launch_bounds__(256)
k_rhosum(int inum, const int *__restrict__ ilist, const int *__restrict__ off,
         const int *__restrict__ nbr, double4 *__restrict__ xf, const int *__restrict__ ty,
         double4 *__restrict__ vr, double *__restrict__ rho_out,
         const Coefs *__restrict__ cf) {
  __shared__ RhoPair s_c[NT1 ? 1 : NT2];
  __shared__ double s_self[MAXT + 1], s_rho0[MAXT + 1], s_B[MAXT + 1];
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_c[t] = cf->rho[t];
  for (int t = threadIdx.x; t < nt1; t += blockDim.x) {
    s_self[t] = cf->self_rho[t];
    s_rho0[t] = cf->rho0[t];
    s_B[t] = cf->B[t];
  }
  __syncthreads();
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= inum) return;
  const int i = ilist ? ilist[row] : row;
  const double4 xi = xf[i];
  const int it = NT1 ? 1 : ty[i];
  const RhoPair c1 = NT1 ? cf->rho[3] : RhoPair{};
  const RhoPair *crow = s_c + it * nt1;
  const int beg = off[row], end = off[row + 1];
  double acc = 0.0;
  constexpr int U = UNROLL;
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
      const RhoPair c = NT1 ? c1 : crow[tj[u]];
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
    const double rho = (EOS && ((cf->rho_keep >> it) & 1)) ? vr[i].w : s_self[it] + acc;
    if (rho_out) rho_out[i] = rho;
    if (EOS) {
      vr[i].w = rho;
      xf[i].w = tait_p_over_rho2(rho, s_rho0[it], s_B[it]);
    }
  }
}

// EOS term for a range of atoms (pair-style layer, or steps without rhosum)
static __global__ void k_eos(int n, double4 *__restrict__ xf, const double4 *__restrict__ vr,
                             const int *__restrict__ ty, const Coefs *__restrict__ cf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ty[i];
  xf[i].w = tait_p_over_rho2(vr[i].w, cf->rho0[t], cf->B[t]);
}

// ------------------------------------------------------------------------------------
// Force pass: sph/taitwater (VISC=0 Monaghan, 1 Morris) and/or sph/heatconduction.
// MODE bits: TAIT | HEAT | HALF.  FULL lists: overwrite (accum=0) or add (accum=1) the
// owned row's results.  HALF lists: atomics on both i and j (reference scatter), or, with
// nojside, the i share only, added without atomics (the j share is then gathered by a
// FULL-mode pass over the reverse half list: each pair value seen from j is exactly the
// negated/mirrored j share -- the formulas are symmetric up to the sign of dx and dv).
// ------------------------------------------------------------------------------------
enum { M_TAIT = 1, M_HEAT = 2, M_HALF = 4 };

// Neighbor::half_from_full_newton's test for a ghost j (neigh_derive.cpp:113-121): the pair
// stays in i's half row iff j lies above i in z, then y, then x
__device__ __forceinline__ bool ghost_keep(const double4 &xi, const double4 &xj) {
  if (xj.z < xi.z) return false;
  if (xj.z == xi.z) {
    if (xj.y < xi.y) return false;
    if (xj.y == xi.y && xj.x < xi.x) return false;
  }
  return true;
}

template <int G, int DIM, int VISC, int MODE, bool NT1>
__global__ void __launch_bounds__(256)
k_force(int inum, int nlocal, int newton, const int *__restrict__ ilist,
        const int *__restrict__ off, const int *__restrict__ nbr,
        const double4 *__restrict__ xf, const double4 *__restrict__ vr,
        const int *__restrict__ ty, const double *__restrict__ en, double4 *__restrict__ fo,
        double *__restrict__ de, int accum, const Coefs *__restrict__ cf, double gx,
        double gy, double gz, double *__restrict__ virial, int nojside,
        const double4 *__restrict__ vso, const double4 *__restrict__ vsg) {
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  constexpr bool HALF = (MODE & M_HALF) != 0;
  constexpr int U = UNROLL;
  __shared__ TaitPair s_t[(TAIT && !NT1) ? NT2 : 1];
  __shared__ HeatPair s_h[(HEAT && !NT1) ? NT2 : 1];
  __shared__ double s_mass[MAXT + 1];
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
      if (TAIT) s_t[t] = cf->tait[t];
      if (HEAT) s_h[t] = cf->heat[t];
    }
  for (int t = threadIdx.x; t < nt1; t += blockDim.x) s_mass[t] = cf->mass[t];
  __syncthreads();
  const int row = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (row >= inum) return;
  const int i = ilist ? ilist[row] : row;
  const double4 xi = xf[i];
  const double4 vi = vr[i];
  const double ei = HEAT ? en[i] : 0.0;
  const int it = NT1 ? 1 : ty[i];
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  const int beg = off[row], end = off[row + 1];
  double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, v5 = 0.0;
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
      const int j = jv[u];
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const int pidx = it * nt1 + tj[u];
      const bool ok = k0 + u * G < end;
      bool hit_t = false, hit_h = false;
      if (TAIT) hit_t = ok && rsq < (NT1 ? t1.cutsq : s_t[pidx].cutsq);
      if (HEAT) hit_h = ok && rsq < (NT1 ? h1.cutsq : s_h[pidx].cutsq);
      if (!(hit_t || hit_h)) continue;
      const double r = fast_sqrt(rsq);
      double jfx = 0.0, jfy = 0.0, jfz = 0.0, jdrho = 0.0, jdE = 0.0;
      if (TAIT && hit_t) {
        const TaitPair c = NT1 ? t1 : s_t[pidx];
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        // setup step (vso != nullptr, full list): the reference's half-list pass meets each
        // ghost pair once, on the side half_from_full keeps -- (i, ghost j) with vest_i as
        // setup_pre_force set it and vest_j as borders() left it, else (j, ghost i') with
        // j's new vest and i's old one (Verlet::setup runs borders before setup_pre_force)
        double3 va = make_double3(vi.x, vi.y, vi.z), vb = make_double3(vj[u].x, vj[u].y, vj[u].z);
        if (vso && j >= nlocal) {
          if (ghost_keep(xi, xj[u])) {
            const double4 g = vsg[j - nlocal];
            vb = make_double3(g.x, g.y, g.z);
          } else {
            const double4 o = vso[i];
            va = make_double3(o.x, o.y, o.z);
          }
        }
        const double velx = va.x - vb.x, vely = va.y - vb.y, velz = va.z - vb.z;
        const double dvdr = dx * velx + dy * vely + dz * velz;
        double fpair, deltaE, fvx = 0.0, fvy = 0.0, fvz = 0.0;
        if (VISC == SPH_VISC_MONAGHAN) {
          // mu = h dvdr/(rsq+0.01h^2); fvisc = -visc (c_i+c_j) mu/(rho_i+rho_j), dvdr < 0
          const double q = (c.viscC * dvdr) * fast_rcp((rsq + c.eps) * (vi.w + vj[u].w));
          const double fvisc = dvdr < 0. ? q : 0.0;
          fpair = c.mm * (xi.w + xj[u].w + fvisc) * wfd;
          deltaE = -0.5 * fpair * dvdr;
        } else {
          // fvisc = 2 visc/(rho_i rho_j) * m_i m_j wfd
          double fvisc = c.viscC * fast_rcp(vi.w * vj[u].w);
          fvisc *= (-c.mm) * wfd;
          fpair = c.mm * (xi.w + xj[u].w) * wfd;
          deltaE = -0.5 * (fpair * dvdr + fvisc * (velx * velx + vely * vely + velz * velz));
          fvx = velx * fvisc;
          fvy = vely * fvisc;
          fvz = velz * fvisc;
        }
        const double tx = dx * fpair + fvx, ty_ = dy * fpair + fvy, tz = dz * fpair + fvz;
        fx += tx;
        fy += ty_;
        fz += tz;
        drho += c.mj * dvdr * wfd;
        dE += deltaE;
        if (HALF) {
          jfx = -tx;
          jfy = -ty_;
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
        const HeatPair c = NT1 ? h1 : s_h[pidx];
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        double deltaE = c.hmD;
        deltaE *= (vi.w + vj[u].w) * fast_rcp(vi.w * vj[u].w);
        deltaE *= (ei - ej[u]) * wfd;
        dE += deltaE;
        if (HALF) jdE -= deltaE;
      }
      if (HALF && !nojside && (newton || j < nlocal)) {
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
    if (HALF && nojside) {  // one row per atom: plain read-modify-write
      if (TAIT) {
        double4 o = fo[i];
        o.x += fx;
        o.y += fy;
        o.z += fz;
        o.w += drho;
        fo[i] = o;
      }
      de[i] += dE;
    } else if (HALF) {
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
