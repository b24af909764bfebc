// sph_tile_kernels.h -- LDS-tiled pair passes (engine kernel_path 2).
//
// Why: the CSR-row kernels (sph_row2_kernels.h) are bound by the texture addresser, not by
// HBM or fp64 VALU: rocprofv3 on C2 1M shows TA_TA_BUSY at ~93% of the kernel's cycles for
// both rhosum and taitwater, and a body-free variant (SPH_EXP=1) runs as long as the full
// kernel (0.69 vs 0.70 ms) while the body on register-resident neighbors (SPH_EXP=2)
// takes 0.33 ms.  Every pair costs 2-4 per-lane random 16-B gathers through the TA.
//
// Here one workgroup serves one bin of owned atoms (bins >= cutneighmax, linear order,
// owned atoms sorted by bin): it stages the records of the bin's 27 (2-D: 9) neighbor
// bins into LDS once with coalesced loads, then every pair reads its neighbor from LDS
// (ds_read_b128, no TA).  Ghost atoms are not moved: a bin-sorted ghost index list
// (gidx) supplies the ghost ranges, so the halo/swap bookkeeping of the brick
// decomposition is untouched.
//
// Lists: the CSR full list of the fast builder (global indices, Neighbor::full_bin
// membership) is translated once per rebuild into 16-bit LDS slots, laid out per bin
// thread-major: thread t of the bin's workgroup owns a contiguous chunk of one row
// (chunk length L_b = ceil(E_b / (TB - R_b)) so the R_b rows' chunks fit in TB
// threads) and its k-th slot lives at base_b + k*TB + t, so each list load of a wave is
// one coalesced 128-B access.  Threads sum their chunk in registers and fold into the
// row's LDS accumulator once (fp64 LDS atomics), so summation order differs from the
// CSR kernels only by association (parity bar 1e-10 rel).
//
// LDS image (SoA 16-B chunks: the 16 lanes of a ds_read_b128 group read 16 random slots
// spread over all 16 four-bank groups instead of 8 with 32-B records):
//   c0[s] = (x, y)   c1[s] = (z, p/rho^2)   c2[s] = (vx, vy)   c3[s] = (vz, rho)
//   [e[s] heat]  [type[s] multi-type]
#pragma once
#include <hip/hip_runtime.h>

#include "sph_bin_kernels.h"
#include "sph_row2_kernels.h"

namespace sph {

constexpr int TB = 512;  // threads per tile workgroup

// gpos[gidx[p] - nlocal] = p (position of each ghost in the bin-sorted ghost order)
static __global__ void k_inverse_perm(int ng, int nlocal, const int *__restrict__ gidx,
                                      int *__restrict__ gpos) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < ng) gpos[gidx[p] - nlocal] = p;
}

// ---- rebuild: per-bin chunk length, list capacity ----------------------------------------
// desc.E = list entries of the bin's rows, desc.L = chunk length (<= TILE_LMAX, else the
// host falls back); blen[b] = TB * ceil(L/2) packed slot pairs
static __global__ void k_tile_plan(int nbins, int *__restrict__ desc, const int *__restrict__ off,
                                   long long *__restrict__ blen, int *__restrict__ mx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nbins) return;
  if (b == nbins) {
    blen[b] = 0;
    return;
  }
  int *d = desc + (size_t)b * kDescInts;
  const int row0 = d[offsetof(BinDesc, row0) / 4], R = d[offsetof(BinDesc, nrows) / 4];
  int E = 0, L = 0;
  if (R > 0) {
    E = off[row0 + R] - off[row0];
    L = R < TB ? max(1, (E + (TB - R) - 1) / (TB - R)) : 0;
    if (R >= TB) atomicMax(&mx[2], R);  // host falls back to the CSR path
  }
  d[offsetof(BinDesc, E) / 4] = E;
  d[offsetof(BinDesc, L) / 4] = L;
  blen[b] = (long long)TB * ((L + 1) / 2);
  atomicMax(&mx[3], L);
}

// chunk prefix of the bin's rows: cpre[r] = sum_{r'<r} ceil(len_r' / L), cpre[R] = total.
// One wave; rows in batches of 64.
__device__ __forceinline__ void tile_chunks(const BinDesc &h, const int *__restrict__ off,
                                            int *cpre) {
  if (threadIdx.x < 64) {
    int carry = 0;
    for (int base = 0; base < h.nrows; base += 64) {
      const int r = base + (int)threadIdx.x;
      const int len = r < h.nrows ? off[h.row0 + r + 1] - off[h.row0 + r] : 0;
      const int c0 = (len + h.L - 1) / h.L;
      int v = c0;
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const int u = __shfl_up(v, dd, 64);
        if ((int)threadIdx.x >= dd) v += u;
      }
      if (r < h.nrows) cpre[r] = carry + v - c0;
      carry += __shfl(v, 63, 64);
    }
    if (threadIdx.x == 0) cpre[h.nrows] = carry;
  }
}

// thread -> (row, first entry, count) of its chunk (count 0: idle thread)
struct Chunk {
  int r, e0, n;
};
__device__ __forceinline__ Chunk tile_chunk(const BinDesc &h, const int *__restrict__ off,
                                            const int *cpre) {
  Chunk q{0, 0, 0};
  const int t = threadIdx.x;
  if (t >= cpre[h.nrows]) return q;
  int lo = 0, hi = h.nrows - 1;  // last r with cpre[r] <= t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cpre[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int len = off[h.row0 + lo + 1] - off[h.row0 + lo];
  q.r = lo;
  q.e0 = (t - cpre[lo]) * h.L;
  q.n = min(h.L, len - q.e0);
  return q;
}

// staged range and offset of slot s (ranges in desc order: 2*row + {0 owned, 1 ghost})
__device__ __forceinline__ int slot_range(const BinDesc &h, int s) {
  int r = 0;
#pragma unroll
  for (int k = 1; k < MAXR; k++) r += (s >= h.pre[k]) ? 1 : 0;
  return r;
}

// ---- rebuild: CSR (global indices) -> thread-major 16-bit slot lists --------------------
// Thread t's chunk is stored as ceil(L/2) packed slot pairs at base + k2*TB + t (entries
// 2*k2 in the low half, 2*k2+1 in the high half): each pair pass loads all of a thread's
// slots with ceil(L/2) coalesced dword loads before its first pair, so no global load
// latency sits inside the pair loop.
constexpr int TILE_LMAX = 32;
// gpos[g] = position of ghost nlocal+g in the bin-sorted ghost order (gidx)
static __global__ void __launch_bounds__(TB)
k_tile_translate(int nbins, int nlocal, const int *__restrict__ desc,
                 const int *__restrict__ off, const int *__restrict__ nbr,
                 const int *__restrict__ gpos, const long long *__restrict__ boff,
                 unsigned *__restrict__ nbr32, int *__restrict__ err) {
  __shared__ BinDesc h;
  __shared__ int cpre[TB + 1];
  const int b = xcd_block();
  if (b >= nbins) return;
  load_desc(desc, b, h);
  if (h.nrows == 0 || h.nrows >= TB) return;
  tile_chunks(h, off, cpre);
  __syncthreads();
  const Chunk q = tile_chunk(h, off, cpre);
  unsigned *out = nbr32 + boff[b] + threadIdx.x;
  const int *row = nbr + off[h.row0 + q.r] + q.e0;
  auto slot_of = [&](int k) {
    if (k >= q.n) return 0;
    const int j = row[k];
    const bool ghost = j >= nlocal;
    const int p = ghost ? gpos[j - nlocal] : j;
    int slot = -1;
#pragma unroll
    for (int r = 0; r < MAXR; r++) {
      const int cnt = h.pre[r + 1] - h.pre[r];
      if (((r & 1) != 0) == ghost && p >= h.rs[r] && p < h.rs[r] + cnt)
        slot = h.pre[r] + (p - h.rs[r]);
    }
    if (slot < 0) {
      atomicOr(err, 1);
      slot = 0;
    }
    return slot;
  };
  for (int k2 = 0; 2 * k2 < h.L; k2++)
    out[(size_t)k2 * TB] = (unsigned)slot_of(2 * k2) | ((unsigned)slot_of(2 * k2 + 1) << 16);
}

// ---- staging ------------------------------------------------------------------------------
template <bool VEL, bool EN, bool TY>
__device__ __forceinline__ void tile_stage(const BinDesc &h, const int *__restrict__ gidx,
                                           const double4 *__restrict__ xf,
                                           const double4 *__restrict__ vr,
                                           const double *__restrict__ en,
                                           const int *__restrict__ ty, double2 *c0,
                                           double2 *c1, double2 *c2, double2 *c3, double *se,
                                           int *sty) {
  const int S = h.pre[MAXR];
  constexpr int K = 2;
  for (int s0 = threadIdx.x; s0 < S; s0 += TB * K) {
    int a[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int s = min(s0 + k * TB, S - 1);
      const int r = slot_range(h, s);
      const int p = h.rs[r] + (s - h.pre[r]);
      a[k] = (r & 1) ? gidx[p] : p;
    }
    double4 x[K], v[K];
    double e[K];
    int t[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      x[k] = xf[a[k]];
      if (VEL) v[k] = vr[a[k]];
      if (EN) e[k] = en[a[k]];
      if (TY) t[k] = ty[a[k]];
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int s = s0 + k * TB;
      if (s < S) {
        c0[s] = make_double2(x[k].x, x[k].y);
        c1[s] = make_double2(x[k].z, x[k].w);
        if (VEL) {
          c2[s] = make_double2(v[k].x, v[k].y);
          c3[s] = make_double2(v[k].z, v[k].w);
        }
        if (EN) se[s] = e[k];
        if (TY) sty[s] = t[k];
      }
    }
  }
}

// LDS bytes of a tile pass for S staged atoms and R rows
__host__ __device__ constexpr int tile_fixed_bytes() {
  return align16((int)sizeof(BinDesc)) + align16((TB + 1) * 4);
}
__host__ inline size_t tile_lds_bytes(bool force, bool heat, bool nt1, int S, int R) {
  size_t b = tile_fixed_bytes();
  b += (size_t)align16((force ? 5 : 1) * 8 * (R > 0 ? R : 1));
  if (!nt1) b += force ? (size_t)kForceCoefBytes : (size_t)kRhoCoefBytes;
  b += (size_t)S * (force ? 64 : 32);
  if (force && heat) b += (size_t)S * 8;
  if (!nt1) b += (size_t)align16(S * 4);
  return b;
}

// ---- sph/rhosum (+ fused EOS epilogue) ------------------------------------------------------
template <bool NT1>
__global__ void __launch_bounds__(TB)
k_tile_rhosum(int nbins, int rmax, const int *__restrict__ desc, const int *__restrict__ gidx,
              double4 *__restrict__ xf, const int *__restrict__ ty, double4 *__restrict__ vr,
              const int *__restrict__ off, const long long *__restrict__ boff,
              const unsigned *__restrict__ nbr32, const Coefs *__restrict__ cf) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BinDesc &h = *reinterpret_cast<BinDesc *>(smem);
  int *cpre = reinterpret_cast<int *>(smem + align16((int)sizeof(BinDesc)));
  double *acc = reinterpret_cast<double *>(smem + tile_fixed_bytes());
  unsigned char *p = smem + tile_fixed_bytes() + align16(8 * rmax);
  RhoPair *s_c = reinterpret_cast<RhoPair *>(p);
  if (!NT1) p += kRhoCoefBytes;
  const int b = xcd_block();
  if (b >= nbins) return;
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_c[t] = cf->rho[t];
  load_desc(desc, b, h);
  if (h.nrows == 0) return;
  const int S = h.pre[MAXR];
  double2 *c0 = reinterpret_cast<double2 *>(p);
  double2 *c1 = c0 + S;
  int *sty = reinterpret_cast<int *>(c1 + S);
  tile_chunks(h, off, cpre);
  for (int r = threadIdx.x; r < h.nrows; r += TB) acc[r] = 0.0;
  tile_stage<false, false, !NT1>(h, gidx, xf, nullptr, nullptr, ty, c0, c1, nullptr, nullptr,
                                 nullptr, sty);
  __syncthreads();
  const Chunk q = tile_chunk(h, off, cpre);
  const RhoPair cc1 = NT1 ? cf->rho[3] : RhoPair{};
  const int si = h.slot0 + q.r;
  const double2 a0 = c0[si], a1 = c1[si];
  const int it = NT1 ? 1 : sty[si];
  const unsigned *lst = nbr32 + boff[b] + threadIdx.x;
  const int L2 = (h.L + 1) >> 1;
  unsigned sv[TILE_LMAX / 2];
#pragma unroll
  for (int k2 = 0; k2 < TILE_LMAX / 2; k2++) sv[k2] = k2 < L2 ? lst[(size_t)k2 * TB] : 0u;
  double sum = 0.0;
  auto pair = [&](int sj, bool ok) {
    const double2 b0 = c0[sj], b1 = c1[sj];
    const double dx = a0.x - b0.x, dy = a0.y - b0.y, dz = a1.x - b1.x;
    const double rsq = dx * dx + dy * dy + dz * dz;
    const RhoPair c = NT1 ? cc1 : s_c[it * nt1 + sty[sj]];
    double wf = 1.0 - rsq * c.ihsq;
    wf = wf * wf;
    wf = wf * wf;
    sum += (ok && rsq < c.cutsq) ? c.mK * wf : 0.0;
  };
#pragma unroll
  for (int k2 = 0; k2 < TILE_LMAX / 2; k2++) {
    if (k2 >= L2) break;  // workgroup-uniform
    pair((int)(sv[k2] & 0xffffu), 2 * k2 < q.n);
    pair((int)(sv[k2] >> 16), 2 * k2 + 1 < q.n);
  }
  if (q.n > 0) atomicAdd(&acc[q.r], sum);
  __syncthreads();
  for (int r = threadIdx.x; r < h.nrows; r += TB) {
    const int i = h.row0 + r;
    const int t = NT1 ? 1 : sty[h.slot0 + r];
    const double rho = cf->self_rho[t] + acc[r];
    vr[i].w = rho;
    xf[i].w = tait_p_over_rho2(rho, cf->rho0[t], cf->B[t]);
  }
}

// ---- sph/taitwater[/morris] [+ sph/heatconduction] ----------------------------------------
template <int VISC, int MODE, bool NT1>
__global__ void __launch_bounds__(TB)
k_tile_force(int nbins, int rmax, const int *__restrict__ desc, const int *__restrict__ gidx,
             const double4 *__restrict__ xf, const double4 *__restrict__ vr,
             const int *__restrict__ ty, const double *__restrict__ en,
             const int *__restrict__ off, const long long *__restrict__ boff,
             const unsigned *__restrict__ nbr32, const Coefs *__restrict__ cf,
             double4 *__restrict__ fo, double *__restrict__ de, double gx, double gy,
             double gz) {
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BinDesc &h = *reinterpret_cast<BinDesc *>(smem);
  int *cpre = reinterpret_cast<int *>(smem + align16((int)sizeof(BinDesc)));
  double *acc = reinterpret_cast<double *>(smem + tile_fixed_bytes());  // [5][rmax]
  unsigned char *p = smem + tile_fixed_bytes() + align16(5 * 8 * rmax);
  TaitPair *s_t = reinterpret_cast<TaitPair *>(p);
  HeatPair *s_h = reinterpret_cast<HeatPair *>(p + align16((int)sizeof(TaitPair) * NT2));
  if (!NT1) p += kForceCoefBytes;
  const int b = xcd_block();
  if (b >= nbins) return;
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
      if (TAIT) s_t[t] = cf->tait[t];
      if (HEAT) s_h[t] = cf->heat[t];
    }
  load_desc(desc, b, h);
  if (h.nrows == 0) return;
  const int S = h.pre[MAXR];
  double2 *c0 = reinterpret_cast<double2 *>(p);
  double2 *c1 = c0 + S;
  double2 *c2 = c1 + S;
  double2 *c3 = c2 + S;
  double *se = reinterpret_cast<double *>(c3 + S);
  int *sty = reinterpret_cast<int *>(se + (HEAT ? S : 0));
  tile_chunks(h, off, cpre);
  for (int r = threadIdx.x; r < 5 * h.nrows; r += TB) acc[(r % 5) * rmax + r / 5] = 0.0;
  tile_stage<true, HEAT, !NT1>(h, gidx, xf, vr, en, ty, c0, c1, c2, c3, se, sty);
  __syncthreads();
  const Chunk q = tile_chunk(h, off, cpre);
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  const int si = h.slot0 + q.r;
  const double2 a0 = c0[si], a1 = c1[si], a2 = c2[si], a3 = c3[si];
  const double ei = HEAT ? se[si] : 0.0;
  const int it = NT1 ? 1 : sty[si];
  const unsigned *lst = nbr32 + boff[b] + threadIdx.x;
  const int L2 = (h.L + 1) >> 1;
  unsigned sv[TILE_LMAX / 2];
#pragma unroll
  for (int k2 = 0; k2 < TILE_LMAX / 2; k2++) sv[k2] = k2 < L2 ? lst[(size_t)k2 * TB] : 0u;
  double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
  auto pair = [&](int sj, bool ok) {
    const double2 b0 = c0[sj], b1 = c1[sj], b2 = c2[sj], b3 = c3[sj];
    const double dx = a0.x - b0.x, dy = a0.y - b0.y, dz = a1.x - b1.x;
    const double rsq = dx * dx + dy * dy + dz * dz;
    const int pidx = NT1 ? 3 : it * nt1 + sty[sj];
    const double r = sqrt1(rsq);
    if (TAIT) {
      const TaitPair c = NT1 ? t1 : s_t[pidx];
      double wfd = c.h - r;
      wfd = c.wK * (wfd * wfd);
      wfd = (ok && rsq < c.cutsq) ? wfd : 0.0;   // zeroes every term below
      const double velx = a2.x - b2.x, vely = a2.y - b2.y, velz = a3.x - b3.x;
      const double dvdr = dx * velx + dy * vely + dz * velz;
      if (VISC == SPH_VISC_MONAGHAN) {
        const double qv = (c.viscC * dvdr) * rcp1((rsq + c.eps) * (a3.y + b3.y));
        const double fvisc = dvdr < 0. ? qv : 0.0;
        const double fpair = c.mm * (a1.y + b1.y + fvisc) * wfd;
        fx += dx * fpair;
        fy += dy * fpair;
        fz += dz * fpair;
        dE += -0.5 * fpair * dvdr;
      } else {
        double fvisc = c.viscC * rcp1(a3.y * b3.y);
        fvisc *= (-c.mm) * wfd;
        const double fpair = c.mm * (a1.y + b1.y) * wfd;
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
      deltaE *= (a3.y + b3.y) * rcp1(a3.y * b3.y);
      deltaE *= (ei - se[sj]) * wfd;
      dE += deltaE;
    }
  };
#pragma unroll
  for (int k2 = 0; k2 < TILE_LMAX / 2; k2++) {
    if (k2 >= L2) break;  // workgroup-uniform
    pair((int)(sv[k2] & 0xffffu), 2 * k2 < q.n);
    pair((int)(sv[k2] >> 16), 2 * k2 + 1 < q.n);
  }
  if (q.n > 0) {
    if (TAIT) {
      atomicAdd(&acc[0 * rmax + q.r], fx);
      atomicAdd(&acc[1 * rmax + q.r], fy);
      atomicAdd(&acc[2 * rmax + q.r], fz);
      atomicAdd(&acc[3 * rmax + q.r], drho);
    }
    atomicAdd(&acc[4 * rmax + q.r], dE);
  }
  __syncthreads();
  for (int r = threadIdx.x; r < h.nrows; r += TB) {
    const int i = h.row0 + r;
    if (TAIT) {
      const double m = cf->mass[NT1 ? 1 : sty[h.slot0 + r]];
      fo[i] = make_double4(acc[r] + m * gx, acc[rmax + r] + m * gy, acc[2 * rmax + r] + m * gz,
                           acc[3 * rmax + r]);
    }
    de[i] = acc[4 * rmax + r];
  }
}

}  // namespace sph
