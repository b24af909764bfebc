// sph_bin_kernels.h -- LDS-staged neighbor tiles: the engine's hot path.
//
// After a rebuild, owned atoms and ghost atoms are each sorted by bin (bins >= cutneigh,
// x fastest).  One workgroup serves one bin: it stages the bin's 27 (2-D: 9) neighbor
// bins -- 9 (3) x-rows, each an owned range plus a ghost range, contiguous because of
// the sort -- into LDS once, and every pair of the bin's rows then reads its neighbor
// from LDS instead of gathering it through the vector L1 (whose line throughput bounds
// the plain CSR kernels).  The Verlet list itself stores 16-bit LDS slot numbers
// (2 B/entry instead of 4), laid out per bin "thread-major" (entry e of the bin lives at
// k*BT + t with t = e / L, k = e % L, L = ceil(E/BT)) so that each thread walks a
// contiguous run of entries -- load-balanced across the bin's ragged rows -- while every
// list load of a wave is one coalesced 128-B access.  Row sums are folded into LDS
// accumulators (fp64 LDS atomics) where a thread's run crosses a row boundary.
//
// Everything a workgroup needs before its pair loop (its 18 staged ranges, slot prefix,
// rows, list length) is precomputed once per rebuild into a 192-B bin descriptor, and the
// rows' list offsets into a per-atom array, so a pair pass costs each workgroup one
// descriptor load, one burst of independent staging loads, and the pair loop.
//
// Membership is exactly Neighbor::full_bin's (rsq <= cutneighsq, j != i,
// src/neigh_full.cpp:241-344); the physics is that of sph_kernels.h.
#pragma once
#include <hip/hip_runtime.h>

#include "sph_engine_kernels.h"
#include "sph_kernels.h"

namespace sph {

constexpr int BT = 256;      // threads per bin workgroup
constexpr int MAXR = 18;     // staged ranges: 9 x-rows x {owned, ghost}
constexpr int MAXROWS = 256; // max owned atoms per bin handled by one workgroup

struct BinCtx {
  Bins bn;
  int dim, nbins, nlocal;
  const int *obeg;  // [nbins+1] first sorted owned atom of bin b (lower bound)
  const int *gbeg;  // [nbins+1] first sorted ghost atom (absolute index) of bin b
};

// 192-B per-bin descriptor (48 ints), written at rebuild
struct BinDesc {
  int rs[MAXR];       // first atom of each staged range
  int pre[MAXR + 1];  // slot prefix; pre[MAXR] = S (staged atoms)
  int row0, nrows;    // the bin's own owned atoms = its rows
  int slot0;          // slot of row 0
  int E, L;           // list entries, entries per thread = ceil(E/BT)
  int pad[6];
};
static_assert(sizeof(BinDesc) == 192, "BinDesc is 48 ints");
constexpr int kDescInts = 48;

// Staged range r of bin b.
__device__ __forceinline__ void bin_range(const BinCtx &c, int b, int r, int &start,
                                          int &count) {
  const int nbx = c.bn.nb[0], nby = c.bn.nb[1], nbz = c.bn.nb[2];
  const int cx = b % nbx, cy = (b / nbx) % nby, cz = b / (nbx * nby);
  const int nrow = (c.dim == 3) ? 9 : 3;
  start = 0;
  count = 0;
  const int row = r >> 1;
  if (row >= nrow) return;
  const int dy = row % 3 - 1;
  const int dz = (c.dim == 3) ? row / 3 - 1 : 0;
  const int by = cy + dy, bz = cz + dz;
  if (by < 0 || by >= nby || bz < 0 || bz >= nbz) return;
  const int bx0 = cx > 0 ? cx - 1 : 0;
  const int bx1 = cx < nbx - 1 ? cx + 1 : nbx - 1;
  const int b0 = (bz * nby + by) * nbx + bx0;
  const int b1 = (bz * nby + by) * nbx + bx1 + 1;
  const int *beg = (r & 1) ? c.gbeg : c.obeg;
  start = beg[b0];
  count = beg[b1] - start;
}

// the center x-row's owned range (row dy = dz = 0) holds the bin's own rows
__device__ __forceinline__ int center_range(int dim) { return ((dim == 3) ? 4 : 1) * 2; }

// All LDS of the bin kernels is one dynamic array carved at 16-B aligned offsets
// (cdna_hip_programming.md Guideline 17: no static __shared__ in front of the dynamic base).
__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }
constexpr int kHdrBytes = (int)sizeof(BinDesc);
constexpr int kRowoffBytes = align16((MAXROWS + 4) * 4);
constexpr int kFixedNeigh = kHdrBytes + kRowoffBytes;
constexpr int kFixedRho = kFixedNeigh + MAXROWS * 8;
constexpr int kFixedForce = kFixedNeigh + 5 * MAXROWS * 8;
// coefficient tables (multi-type only) and per-staged-atom bytes, per kernel
constexpr int kNeighCoefBytes = align16(8 * NT2);
constexpr int kRhoCoefBytes = align16((int)sizeof(RhoPair) * NT2);
constexpr int kForceCoefBytes = align16((int)sizeof(TaitPair) * NT2) + align16((int)sizeof(HeatPair) * NT2);
__host__ __device__ constexpr int neigh_atom_bytes() { return 32 + 4; }
__host__ __device__ constexpr int rho_atom_bytes(bool nt1) { return 32 + (nt1 ? 0 : 4); }
__host__ __device__ constexpr int force_atom_bytes(bool heat, bool nt1) {
  return 64 + (heat ? 8 : 0) + (nt1 ? 0 : 4);
}

// descriptor of every bin; device maxima of staged size and rows into mx[0], mx[1]
static __global__ void k_bin_desc(BinCtx c, int *__restrict__ desc, int *__restrict__ mx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= c.nbins) return;
  BinDesc d{};
  d.row0 = c.obeg[b];
  d.nrows = c.obeg[b + 1] - d.row0;
  int S = 0;
  for (int r = 0; r < MAXR; r++) {
    int st = 0, cn = 0;
    if (d.nrows > 0) bin_range(c, b, r, st, cn);
    d.rs[r] = st;
    d.pre[r] = S;
    S += cn;
  }
  d.pre[MAXR] = S;
  const int cr = center_range(c.dim);
  d.slot0 = d.pre[cr] + (d.row0 - d.rs[cr]);
  const int *src = reinterpret_cast<const int *>(&d);
  int4 *dst = reinterpret_cast<int4 *>(desc + (size_t)b * kDescInts);
#pragma unroll
  for (int k = 0; k < kDescInts / 4; k++)
    dst[k] = make_int4(src[4 * k], src[4 * k + 1], src[4 * k + 2], src[4 * k + 3]);
  atomicMax(&mx[0], S);
  atomicMax(&mx[1], d.nrows);
}

// descriptor -> LDS (threads 0..47), then a barrier
__device__ __forceinline__ void load_desc(const int *__restrict__ desc, int b, BinDesc &h) {
  if (threadIdx.x < kDescInts)
    reinterpret_cast<int *>(&h)[threadIdx.x] = desc[(size_t)b * kDescInts + threadIdx.x];
  __syncthreads();
}

// slot -> global atom index
__device__ __forceinline__ int slot_atom(const BinDesc &h, int s) {
  int r = 0;
#pragma unroll
  for (int k = 1; k < MAXR; k++) r += (s >= h.pre[k]) ? 1 : 0;
  return h.rs[r] + (s - h.pre[r]);
}

// Stage the bin's neighborhood records into LDS.  Each thread issues the loads of K slots
// before its first LDS store, so a whole neighborhood (~1000 atoms) is one burst of
// independent loads rather than 18 dependent range loops.
template <bool VEL, bool EN, bool TY>
__device__ __forceinline__ void stage_atoms(const BinDesc &h, const double4 *__restrict__ xf,
                                            const double4 *__restrict__ vr,
                                            const double *__restrict__ en,
                                            const int *__restrict__ ty, double4 *sx, double4 *sv,
                                            double *se, int *sty) {
  const int S = h.pre[MAXR];
  constexpr int K = 4;
  for (int s0 = threadIdx.x; s0 < S; s0 += BT * K) {
    int g[K];
    double4 a[K], v[K];
    double e[K];
    int t[K];
#pragma unroll
    for (int k = 0; k < K; k++) g[k] = slot_atom(h, min(s0 + k * BT, S - 1));
#pragma unroll
    for (int k = 0; k < K; k++) {
      a[k] = xf[g[k]];
      if (VEL) v[k] = vr[g[k]];
      if (EN) e[k] = en[g[k]];
      if (TY) t[k] = ty[g[k]];
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int s = s0 + k * BT;
      if (s < S) {
        sx[s] = a[k];
        if (VEL) sv[s] = v[k];
        if (EN) se[s] = e[k];
        if (TY) sty[s] = t[k];
      }
    }
  }
}

// per-bin lower bounds of sorted keys: beg[b] = first p with key[p] >= b (b in [0,nbins])
static __global__ void k_lower_bound(int nbins, int n, int base, const unsigned *__restrict__ key,
                                     int *__restrict__ beg) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nbins) return;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (key[mid] < (unsigned)b) lo = mid + 1;
    else hi = mid;
  }
  beg[b] = base + lo;
}

// ---- list build: count pass (row counts, row offsets, per-bin E/L) and fill pass --------
template <bool FILL>
__global__ void __launch_bounds__(BT)
k_bin_neigh(int nbins, int *__restrict__ desc, const double4 *__restrict__ xf,
            const int *__restrict__ ty, const Coefs *__restrict__ cf, int *__restrict__ cnt,
            int *__restrict__ roff, int *__restrict__ binE, const long long *__restrict__ boff,
            unsigned short *__restrict__ nbr16) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BinDesc &h = *reinterpret_cast<BinDesc *>(smem);
  int *s_cnt = reinterpret_cast<int *>(smem + kHdrBytes);
  double *s_cns = reinterpret_cast<double *>(smem + kFixedNeigh);
  const int b = xcd_block();
  if (b >= nbins) return;
  const int nt1 = cf->ntypes + 1;
  for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_cns[t] = cf->cutneighsq[t];
  load_desc(desc, b, h);
  const int R = h.nrows;
  if (R == 0) {  // no owned atoms: nothing to list
    if (!FILL && threadIdx.x == 0) binE[b] = 0;
    return;
  }
  const int S = h.pre[MAXR];
  double4 *sx = reinterpret_cast<double4 *>(smem + kFixedNeigh + kNeighCoefBytes);
  int *sty = reinterpret_cast<int *>(sx + S);
  stage_atoms<false, false, true>(h, xf, nullptr, nullptr, ty, sx, nullptr, nullptr, sty);
  __syncthreads();
  constexpr int G = 8;
  const int lane = threadIdx.x & (G - 1);
  const int grp = threadIdx.x / G;
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  const unsigned long long gmask = (1ull << G) - 1ull;
  for (int r = grp; r < R; r += BT / G) {
    const int si = h.slot0 + r;
    const double4 xi = sx[si];
    const double *crow = s_cns + sty[si] * nt1;
    int n = 0;
    int e = FILL ? roff[h.row0 + r] : 0;
    for (int base = 0; base < S; base += G) {
      const int s = base + lane;
      bool hit = false;
      if (s < S && s != si) {
        const double4 xj = sx[s];
        const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
        const double rsq = dx * dx + dy * dy + dz * dz;
        hit = rsq <= crow[sty[s]];
      }
      if (FILL) {
        const unsigned long long m = (__ballot(hit) >> gbase) & gmask;
        if (hit) {
          const int ee = e + __popcll(m & ((1ull << lane) - 1ull));
          nbr16[boff[b] + (long long)(ee % h.L) * BT + ee / h.L] = (unsigned short)s;
        }
        e += __popcll(m);
      } else {
        n += hit ? 1 : 0;
      }
    }
    if (!FILL) {
      n = group_sum_i<G>(n);
      if (lane == 0) s_cnt[r] = n;
    }
  }
  if (!FILL) {
    __syncthreads();
    if (threadIdx.x < 64) {  // one wave: exclusive scan of the row counts -> roff, E, L
      int carry = 0;
      for (int base = 0; base < R; base += 64) {
        const int r = base + threadIdx.x;
        const int c0 = r < R ? s_cnt[r] : 0;
        int v = c0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int u = __shfl_up(v, d, 64);
          if ((int)threadIdx.x >= d) v += u;
        }
        if (r < R) {
          cnt[h.row0 + r] = c0;
          roff[h.row0 + r] = carry + v - c0;
        }
        carry += __shfl(v, 63, 64);
      }
      if (threadIdx.x == 0) {
        binE[b] = carry;
        desc[(size_t)b * kDescInts + offsetof(BinDesc, E) / 4] = carry;
        desc[(size_t)b * kDescInts + offsetof(BinDesc, L) / 4] = (carry + BT - 1) / BT;
      }
    }
  }
}

// bin b's padded list length (multiple of BT): L*BT
static __global__ void k_bin_listlen(int nbins, const int *__restrict__ binE,
                                     long long *__restrict__ blen) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nbins) return;
  blen[b] = (b < nbins) ? (long long)((binE[b] + BT - 1) / BT) * BT : 0;
}

// ---- staged pair passes ------------------------------------------------------------------
// A thread's contiguous run [e0, e1) of its bin's entries and the row holding e0.
struct Run {
  int e0, e1, r;
};

__device__ __forceinline__ Run thread_run(const BinDesc &h, const int *s_rowoff) {
  Run q;
  q.e0 = threadIdx.x * h.L;
  q.e1 = min(q.e0 + h.L, h.E);
  int lo = 0, hi = h.nrows - 1;  // last r with rowoff[r] <= e0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_rowoff[mid] <= q.e0) lo = mid;
    else hi = mid - 1;
  }
  q.r = lo;
  return q;
}

// the rows' list offsets (precomputed at rebuild) plus E at [nrows]
__device__ __forceinline__ void load_rowoffs(const BinDesc &h, const int *__restrict__ roff,
                                             int *s_rowoff) {
  for (int r = threadIdx.x; r < h.nrows; r += blockDim.x) s_rowoff[r] = roff[h.row0 + r];
  if (threadIdx.x == 0) s_rowoff[h.nrows] = h.E;
}

template <int DIM, bool NT1>
__global__ void __launch_bounds__(BT)
k_bin_rhosum(int nbins, const int *__restrict__ desc, double4 *__restrict__ xf,
             const int *__restrict__ ty, double4 *__restrict__ vr, const int *__restrict__ roff,
             const long long *__restrict__ boff, const unsigned short *__restrict__ nbr16,
             const Coefs *__restrict__ cf) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BinDesc &h = *reinterpret_cast<BinDesc *>(smem);
  int *s_rowoff = reinterpret_cast<int *>(smem + kHdrBytes);
  double *s_acc = reinterpret_cast<double *>(smem + kFixedNeigh);
  RhoPair *s_c = reinterpret_cast<RhoPair *>(smem + kFixedRho);
  const int b = xcd_block();
  if (b >= nbins) return;
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_c[t] = cf->rho[t];
  load_desc(desc, b, h);
  if (h.nrows == 0) return;
  const int S = h.pre[MAXR];
  double4 *sx = reinterpret_cast<double4 *>(smem + kFixedRho + (NT1 ? 0 : kRhoCoefBytes));
  int *sty = reinterpret_cast<int *>(sx + S);
  load_rowoffs(h, roff, s_rowoff);
  for (int r = threadIdx.x; r < h.nrows; r += blockDim.x) s_acc[r] = 0.0;
  stage_atoms<false, false, !NT1>(h, xf, nullptr, nullptr, ty, sx, nullptr, nullptr, sty);
  __syncthreads();
  const RhoPair c1 = NT1 ? cf->rho[3] : RhoPair{};
  Run q = thread_run(h, s_rowoff);
  const unsigned short *lst = nbr16 + boff[b] + threadIdx.x;
  if (q.e0 < q.e1) {
    int r = q.r;
    int rend = s_rowoff[r + 1];
    int si = h.slot0 + r;
    double4 xi = sx[si];
    int it = NT1 ? 1 : sty[si];
    double acc = 0.0;
    auto pair = [&](int sj) {
      const double4 xj = sx[sj];
      const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const RhoPair cc = NT1 ? c1 : s_c[it * nt1 + sty[sj]];
      double wf = 1.0 - rsq * cc.ihsq;
      wf = wf * wf;
      wf = wf * wf;
      acc += (rsq < cc.cutsq) ? cc.mK * wf : 0.0;
    };
    const int n = q.e1 - q.e0;
    constexpr int U = 8;
    int nxt[U];
#pragma unroll
    for (int u = 0; u < U; u++) nxt[u] = lst[min(u, n - 1) * BT];
    for (int k = 0; k < n; k += U) {
      int sl[U];
#pragma unroll
      for (int u = 0; u < U; u++) sl[u] = nxt[u];
#pragma unroll
      for (int u = 0; u < U; u++) nxt[u] = lst[min(k + U + u, n - 1) * BT];  // prefetch
      const int e = q.e0 + k;
      if (e + U <= rend && k + U <= n) {  // whole batch inside the current row
#pragma unroll
        for (int u = 0; u < U; u++) pair(sl[u]);
      } else {
        for (int u = 0; u < U && k + u < n; u++) {
          while (e + u >= rend) {  // row boundary: fold the partial sum, next row
            atomicAdd(&s_acc[r], acc);
            acc = 0.0;
            r++;
            rend = s_rowoff[r + 1];
            si = h.slot0 + r;
            xi = sx[si];
            if (!NT1) it = sty[si];
          }
          pair(sl[u]);
        }
      }
    }
    atomicAdd(&s_acc[r], acc);
  }
  __syncthreads();
  for (int r = threadIdx.x; r < h.nrows; r += blockDim.x) {
    const int i = h.row0 + r;
    const int t = NT1 ? 1 : ty[i];
    const double rho = cf->self_rho[t] + s_acc[r];
    vr[i].w = rho;
    xf[i].w = tait_p_over_rho2(rho, cf->rho0[t], cf->B[t]);
  }
}

template <int DIM, int VISC, int MODE, bool NT1>
__global__ void __launch_bounds__(BT)
k_bin_force(int nbins, const int *__restrict__ desc, const double4 *__restrict__ xf,
            const double4 *__restrict__ vr, const int *__restrict__ ty,
            const double *__restrict__ en, const int *__restrict__ roff,
            const long long *__restrict__ boff, const unsigned short *__restrict__ nbr16,
            const Coefs *__restrict__ cf, double4 *__restrict__ fo, double *__restrict__ de,
            double gx, double gy, double gz) {
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BinDesc &h = *reinterpret_cast<BinDesc *>(smem);
  int *s_rowoff = reinterpret_cast<int *>(smem + kHdrBytes);
  double(*s_acc)[MAXROWS] = reinterpret_cast<double(*)[MAXROWS]>(smem + kFixedNeigh);
  TaitPair *s_t = reinterpret_cast<TaitPair *>(smem + kFixedForce);
  HeatPair *s_h = reinterpret_cast<HeatPair *>(smem + kFixedForce + align16((int)sizeof(TaitPair) * NT2));
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
  double4 *sx = reinterpret_cast<double4 *>(smem + kFixedForce + (NT1 ? 0 : kForceCoefBytes));
  double4 *sv = sx + S;
  double *se = reinterpret_cast<double *>(sv + S);
  int *sty = reinterpret_cast<int *>(se + (HEAT ? S : 0));
  load_rowoffs(h, roff, s_rowoff);
  for (int r = threadIdx.x; r < h.nrows; r += blockDim.x) {
    s_acc[0][r] = s_acc[1][r] = s_acc[2][r] = s_acc[3][r] = s_acc[4][r] = 0.0;
  }
  stage_atoms<true, HEAT, !NT1>(h, xf, vr, en, ty, sx, sv, se, sty);
  __syncthreads();
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  Run q = thread_run(h, s_rowoff);
  const unsigned short *lst = nbr16 + boff[b] + threadIdx.x;
  if (q.e0 < q.e1) {
    int r = q.r;
    int rend = s_rowoff[r + 1];
    int si = h.slot0 + r;
    double4 xi = sx[si], vi = sv[si];
    double ei = HEAT ? se[si] : 0.0;
    int it = NT1 ? 1 : sty[si];
    double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
    auto pair = [&](int sj) {
      const double4 xj = sx[sj];
      const double4 vj = sv[sj];
      const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const int pidx = NT1 ? 3 : it * nt1 + sty[sj];
      bool hit_t = false, hit_h = false;
      if (TAIT) hit_t = rsq < (NT1 ? t1.cutsq : s_t[pidx].cutsq);
      if (HEAT) hit_h = rsq < (NT1 ? h1.cutsq : s_h[pidx].cutsq);
      if (!(hit_t || hit_h)) return;
      const double r1 = fast_sqrt(rsq);
      if (TAIT && hit_t) {
        const TaitPair cc = NT1 ? t1 : s_t[pidx];
        double wfd = cc.h - r1;
        wfd = cc.wK * (wfd * wfd);
        const double velx = vi.x - vj.x, vely = vi.y - vj.y, velz = vi.z - vj.z;
        const double dvdr = dx * velx + dy * vely + dz * velz;
        double fpair, deltaE, fvx = 0.0, fvy = 0.0, fvz = 0.0;
        if (VISC == SPH_VISC_MONAGHAN) {
          // mu = h dvdr/(rsq+0.01h^2); fvisc = -visc (c_i+c_j) mu/(rho_i+rho_j), dvdr < 0
          const double qv = (cc.viscC * dvdr) * fast_rcp((rsq + cc.eps) * (vi.w + vj.w));
          const double fvisc = dvdr < 0. ? qv : 0.0;
          fpair = cc.mm * (xi.w + xj.w + fvisc) * wfd;
          deltaE = -0.5 * fpair * dvdr;
        } else {
          double fvisc = cc.viscC * fast_rcp(vi.w * vj.w);
          fvisc *= (-cc.mm) * wfd;
          fpair = cc.mm * (xi.w + xj.w) * wfd;
          deltaE = -0.5 * (fpair * dvdr + fvisc * (velx * velx + vely * vely + velz * velz));
          fvx = velx * fvisc;
          fvy = vely * fvisc;
          fvz = velz * fvisc;
        }
        fx += dx * fpair + fvx;
        fy += dy * fpair + fvy;
        fz += dz * fpair + fvz;
        drho += cc.mj * dvdr * wfd;
        dE += deltaE;
      }
      if (HEAT && hit_h) {
        const HeatPair cc = NT1 ? h1 : s_h[pidx];
        double wfd = cc.h - r1;
        wfd = cc.wK * (wfd * wfd);
        double deltaE = cc.hmD;
        deltaE *= (vi.w + vj.w) * fast_rcp(vi.w * vj.w);
        deltaE *= (ei - se[sj]) * wfd;
        dE += deltaE;
      }
    };
    auto flush = [&]() {
      if (TAIT) {
        atomicAdd(&s_acc[0][r], fx);
        atomicAdd(&s_acc[1][r], fy);
        atomicAdd(&s_acc[2][r], fz);
        atomicAdd(&s_acc[3][r], drho);
      }
      atomicAdd(&s_acc[4][r], dE);
      fx = fy = fz = drho = dE = 0.0;
    };
    const int n = q.e1 - q.e0;
    constexpr int U = 4;
    int nxt[U];
#pragma unroll
    for (int u = 0; u < U; u++) nxt[u] = lst[min(u, n - 1) * BT];
    for (int k = 0; k < n; k += U) {
      int sl[U];
#pragma unroll
      for (int u = 0; u < U; u++) sl[u] = nxt[u];
#pragma unroll
      for (int u = 0; u < U; u++) nxt[u] = lst[min(k + U + u, n - 1) * BT];  // prefetch
      const int e = q.e0 + k;
      if (e + U <= rend && k + U <= n) {  // whole batch inside the current row
#pragma unroll
        for (int u = 0; u < U; u++) pair(sl[u]);
      } else {
        for (int u = 0; u < U && k + u < n; u++) {
          while (e + u >= rend) {  // row boundary: fold partial sums, move to the next row
            flush();
            r++;
            rend = s_rowoff[r + 1];
            si = h.slot0 + r;
            xi = sx[si];
            vi = sv[si];
            if (HEAT) ei = se[si];
            if (!NT1) it = sty[si];
          }
          pair(sl[u]);
        }
      }
    }
    flush();
  }
  __syncthreads();
  for (int r = threadIdx.x; r < h.nrows; r += blockDim.x) {
    const int i = h.row0 + r;
    if (TAIT) {
      const double m = cf->mass[NT1 ? 1 : ty[i]];
      fo[i] = make_double4(s_acc[0][r] + m * gx, s_acc[1][r] + m * gy, s_acc[2][r] + m * gz,
                           s_acc[3][r]);
    }
    de[i] = s_acc[4][r];
  }
}

// reorder the ghost segment by bin: scratch <- ghosts in sorted order
static __global__ void k_permute_ghosts(int ng, int nlocal, const int *__restrict__ perm,
                                        const double4 *__restrict__ xf,
                                        const double4 *__restrict__ vr,
                                        const double *__restrict__ en,
                                        const int *__restrict__ ty,
                                        const int *__restrict__ gowner,
                                        const int *__restrict__ gimg, double4 *__restrict__ xf2,
                                        double4 *__restrict__ vr2, double *__restrict__ en2,
                                        int *__restrict__ ty2, int *__restrict__ gowner2,
                                        int *__restrict__ gimg2) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ng) return;
  const int s = perm[k];  // absolute index of the k-th ghost in bin order
  xf2[k] = xf[s];
  vr2[k] = vr[s];
  en2[k] = en[s];
  ty2[k] = ty[s];
  gowner2[k] = gowner[s - nlocal];
  gimg2[k] = gimg[s - nlocal];
}

}  // namespace sph
