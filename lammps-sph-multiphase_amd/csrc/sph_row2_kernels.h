// sph_row2_kernels.h -- second generation of the engine's CSR-row pair passes.
//
// The row path (engine kernel_path 1): full list, gather only, G lanes per row, U pairs in
// flight per lane, branch-free pair body (a pair outside the cutoff, or a padding slot,
// gets a zero kernel weight, which zeroes every term it feeds).  What bounds these
// passes on gfx950 is the texture addresser (TA): rocprofv3 on C2 1M shows TA_TA_BUSY at
// ~93% of the kernel's cycles, and a body-free variant (EXP=1) runs as long as the full
// kernel.  tools/ta_bench.hip prices the TA: ~2.25 cycles per DISTINCT 128-B line a
// 64-lane load instruction touches (L2-resident; ~5 beyond L2), whatever the bytes per
// lane (4, 8 or 16), and loads dropped by the range check cost the same.  So the design
// maximises the lanes of one instruction that share a line:
//  * the G lanes of a row take consecutive list entries, which are mostly consecutive
//    atoms of one bin (Morton/bin order), so neighbouring lanes hit the same lines;
//  * LP (lane-pair gathers): the two lanes of an adjacent pair fetch each other's
//    32-B records cooperatively -- each 16-B load then touches one record per lane PAIR
//    -- and swap halves with a DPP quad permute (~24 extra 32-bit VALU ops per pair);
//  * IV (index vectors): with a list stored chunk-transposed by the builder (entry
//    c*4G + u*G + l at c*4G + 4l + u, k_neigh3's `perm`), lane l's four entries of a
//    chunk are one 16-B load while the lane -> entry mapping (and so the line sharing
//    of the record gathers) stays strided; a quarter of the index loads.  (Giving a
//    lane four CONSECUTIVE entries instead was slower: adjacent lanes then gather
//    records four entries apart and share fewer lines.)
//  * buffer loads with 32-bit byte offsets: one shift per neighbor instead of a 64-bit
//    address per array, hardware range check instead of clamped indices (an index slot
//    past the row end reads the next row's entry or 0 -- a valid atom -- and is masked
//    like an out-of-cut pair);
//  * the next chunk's indices are loaded before the current chunk's records are used;
//  * reciprocal and square root seeded by v_rcp_f64 / v_rsq_f64 with one Newton
//    correction each (relative error ~1e-15, inside the 1e-10 parity bar).
// Byte offsets are 32-bit: the host uses these kernels only while the list and the atom
// arrays stay below 2 GiB (row2_fits), the first generation otherwise.
//
// EXP (study builds only, SPH_EXP): 1 = gathers with a trivial body (the gather-bound
// time of the pass), 2 = the full body on synthetic neighbors without gathers (the
// VALU-bound time).  Their outputs are meaningless.
#pragma once
#include <hip/hip_runtime.h>

#include "sph_kernels.h"

namespace sph {

// the engine's per-pass arguments (owned rows, layout of sph_kernels.h)
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

typedef __amdgpu_buffer_rsrc_t Rsrc;

// Cache policy of the neighbour-index stream loads: nt (bit 1, non-temporal), so the
// ~620 MB/pass index stream, read once, does not push the gathered records out of L2.
// Measured on C2 1M (kernel_sweep, 50 reps): rhosum 0.313 -> 0.302 ms, taitwater
// 0.560 -> 0.548 ms; sc0|nt (3) 0.305 / 0.553; sc0 on the record gathers instead: 0.305 /
// 0.561; nontemporal stores of f/drho/de: no gain (profiles/r01/kernels/sweep_cachepolicy.log)
#ifndef SPH_IDX_AUX
#define SPH_IDX_AUX 2
#endif

// Typed list entries (k_neigh3 tbits): atom index in bits 0-27, type-1 in bits 28-30.
// Slots past a row's end may hold anything: the decoded type is clamped to ntypes so the
// coefficient lookup of a masked slot stays inside the loaded table.
__device__ __forceinline__ unsigned ent_atom(unsigned e, bool tb) {
  return tb ? (e & (unsigned)SPH_TBIT_MASK) : e;
}
__device__ __forceinline__ int ent_type(unsigned e, int ntypes) {
  return min((int)(e >> SPH_TBIT_SHIFT) + 1, ntypes);
}
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ Rsrc make_rsrc(const void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ __forceinline__ int ld_i32(Rsrc r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ v4u ld_b128(Rsrc r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ double u2d(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}
__device__ __forceinline__ double4 ld_d4(Rsrc r, unsigned off) {
  const v4u a = ld_b128(r, off);
  const v4u b = ld_b128(r, off + 16);
  return make_double4(u2d(a.x, a.y), u2d(a.z, a.w), u2d(b.x, b.y), u2d(b.z, b.w));
}
// x, y, z only (24 B: one b128 + one b64)
__device__ __forceinline__ double3 ld_d3(Rsrc r, unsigned off) {
  const v4u a = ld_b128(r, off);
  const v2u b = __builtin_amdgcn_raw_buffer_load_b64(r, off + 16, 0, 0);
  return make_double3(u2d(a.x, a.y), u2d(a.z, a.w), u2d(b.x, b.y));
}
__device__ __forceinline__ double ld_d1(Rsrc r, unsigned off) {
  const v2u b = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return u2d(b.x, b.y);
}

// value of the adjacent lane (lane ^ 1): DPP quad_perm [1,0,3,2]
__device__ __forceinline__ unsigned swap1(unsigned v) {
  return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ v4u swap1(v4u v) {
  return v4u{swap1(v.x), swap1(v.y), swap1(v.z), swap1(v.w)};
}
__device__ __forceinline__ v4u sel(bool c, v4u a, v4u b) {
  return v4u{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w};
}
// Lane-pair gather of one 32-B record per lane: lanes 2p (even) and 2p+1 (odd) want the
// records of ja (even lane's neighbor) and jb (odd lane's).  Load 1 hits ja on both
// lanes (even: bytes 0-15, odd: 16-31), load 2 hits jb (even: 16-31, odd: 0-15); each
// lane then hands the half it does not need to its partner.  Both lanes of a pair must
// be active (the DPP read of an inactive lane is undefined).
__device__ __forceinline__ double4 lp_d4(Rsrc r, unsigned ja, unsigned jb, bool odd) {
  const v4u t0 = ld_b128(r, ja * 32u + (odd ? 16u : 0u));
  const v4u t1 = ld_b128(r, jb * 32u + (odd ? 0u : 16u));
  const v4u c1 = swap1(sel(odd, t0, t1));
  const v4u c0 = sel(odd, t1, t0);
  return make_double4(u2d(c0.x, c0.y), u2d(c0.z, c0.w), u2d(c1.x, c1.y), u2d(c1.z, c1.w));
}

// 1/b, b a positive normal: v_rcp_f64 seed + one Newton step
__device__ __forceinline__ double rcp1(double b) {
  const double y = __builtin_amdgcn_rcp(b);
  return fma(y, fma(-b, y, 1.0), y);
}
// sqrt(x), x >= 0: v_rsq_f64 seed y, r = x*y, one Newton correction r += (x - r^2) y / 2.
// x + 1e-300 (== x for any x above ~1e-284) makes a coincident pair give r ~ 1e-150
// instead of NaN.
__device__ __forceinline__ double sqrt1(double x) {
  x += 1e-300;
  const double y = __builtin_amdgcn_rsq(x);
  const double r = x * y;
  return fma(fma(-r, r, x), 0.5 * y, r);
}
// the same for an x that already carries the 1e-300 (rsq_t: folded into its first product)
__device__ __forceinline__ double sqrt1n(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double r = x * y;
  return fma(fma(-r, r, x), 0.5 * y, r);
}
// dx^2 + dy^2 + dz^2 + 1e-300 in three FMAs (sqrt1n's argument)
__device__ __forceinline__ double rsq_t(double dx, double dy, double dz) {
  return fma(dx, dx, fma(dy, dy, fma(dz, dz, 1e-300)));
}

// byte size of n records of T for the range check (the host guarantees < 2 GiB)
template <class T>
__device__ __forceinline__ unsigned nbytes(int n) {
  return (unsigned)n * (unsigned)sizeof(T);
}

// A lane's U neighbor indices of the chunk starting at list entry k0 (row entries
// [beg, end)): entries k0 + el + u*G, el = the lane's entry slot (entry_slot) -- with IV
// from a chunk-transposed list, where they sit contiguously at k0 + 4*lane (one 16-B
// load; U = 4; k0 16-B aligned).
template <int G, int U, bool IV>
__device__ __forceinline__ void chunk_idx(Rsrc rn, int k0, int lane, int el, int (&j)[U]) {
  if (IV) {
    static_assert(!IV || U == 4, "index vectors hold 4 entries");
    const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rn, (unsigned)(k0 + 4 * lane) * 4u, 0,
                                                        SPH_IDX_AUX);
    j[0] = (int)v.x;
    j[1] = (int)v.y;
    j[2] = (int)v.z;
    j[3] = (int)v.w;
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) j[u] = ld_i32(rn, (unsigned)(k0 + el + u * G) * 4u);
  }
}
template <int G, int U, bool IV>
__device__ __forceinline__ int chunk_pos(int k0, int el, int u) {
  return k0 + el + u * G;
}

// TIGHT (strided list, LP): also write this step's in-cut neighbors -- rsq inside the
// force styles' cutoff (fcutsq), the only pairs the force pass can use, positions being
// fixed between the two passes -- as a compacted "tight" list: row rr at tnbr + rr*stride,
// tcnt[rr] entries.  The group compacts its hits through LDS and stores them 16 B at a
// time (a quarter of the store instructions of per-lane 4-B stores, which cost the TA as
// much as gathers); the force pass then walks ~25% fewer chunks.
template <int G, int U, bool NT1, bool LP, bool IV, bool TIGHT>
__global__ void __launch_bounds__(256)
k_row2_rhosum(int n, int nall, int ntot, const int *__restrict__ off, int stride,
              const int *__restrict__ rcnt,
              const int *__restrict__ nbr, double4 *__restrict__ xf,
              const int *__restrict__ ty, double4 *__restrict__ vr,
              const Coefs *__restrict__ cf, int *__restrict__ tnbr, int *__restrict__ tcnt,
              int pi, const int *__restrict__ rows, int tbits) {
  static_assert(!TIGHT || LP, "the tight-list compaction needs wave-uniform trip counts");
  __shared__ RhoPair s_c[NT1 ? 1 : NT2];
  __shared__ double s_fc[(NT1 || !TIGHT) ? 1 : NT2];
  // a group's buffer holds up to 3 carried entries + one chunk's G*U hits, rounded up to
  // whole 16-B stores (G*U = 64 at tile 2 would overflow a 64-entry row)
  constexpr int TQ = TIGHT ? (G * U + 3 + 3) / 4 * 4 : 4;
  static_assert(!TIGHT || TQ >= G * U + 3, "tight-list buffer too small");
  __shared__ __attribute__((aligned(16))) int s_tq[TIGHT ? 256 / G : 1][TQ];
  const int nt1 = cf->ntypes + 1;
  if (!NT1) {
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
      s_c[t] = cf->rho[t];
      if (TIGHT) s_fc[t] = cf->fcutsq[t];
    }
    __syncthreads();
  }
  // rows != nullptr: the launch covers the n rows rows[0..n) (an interior / boundary
  // subset, see sph_engine overlap), else rows 0..n-1
  const int idx = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  const int el = entry_slot<G>(lane, pi);
  // LP: lanes of rows past n stay in the loop (masked) so every DPP partner is active
  if (!LP && idx >= n) return;
  const bool live = idx < n;
  const bool odd = (threadIdx.x & 1) != 0;
  const Rsrc rn = make_rsrc(nbr, nbytes<int>(ntot));
  const Rsrc rx = make_rsrc(xf, nbytes<double4>(nall));
  const Rsrc rt = make_rsrc(ty, nbytes<int>(nall));
  const int rr = rows ? rows[live ? idx : n - 1] : (live ? idx : n - 1);
  const int row = rr;
  const bool tb = !NT1 && tbits != 0;
  const double4 xi = xf[rr];
  const int it = NT1 ? 1 : ty[rr];
  const RhoPair c1 = NT1 ? cf->rho[3] : RhoPair{};
  // stride > 0: fixed-stride rows (row rr at rr*stride, rcnt[rr] entries), else CSR
  const int beg = stride > 0 ? rr * stride : off[rr];
  const int end = live ? (stride > 0 ? beg + rcnt[rr] : off[rr + 1]) : beg;
  const double fc1 = (NT1 && TIGHT) ? cf->fcutsq[3] : 0.0;
  const int gq = threadIdx.x / G, gbase = (threadIdx.x & 63) & ~(G - 1);
  const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
  const unsigned long long below = (1ull << lane) - 1ull;
  int *const trow = TIGHT ? tnbr + (size_t)rr * stride : nullptr;
  int tq = 0, tw = 0;  // tight entries buffered in LDS / already stored (group-uniform)
  double acc = 0.0;
  int jn[U];
  chunk_idx<G, U, IV>(rn, beg, lane, el, jn);
  for (int k0 = beg; LP ? __any(chunk_pos<G, U, IV>(k0, el, 0) < end)
                        : chunk_pos<G, U, IV>(k0, el, 0) < end;
       k0 += G * U) {
    double3 xj[U];
    int tj[U], jc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      jc[u] = jn[u];
      const unsigned o = ent_atom((unsigned)jn[u], tb);
      if (LP) {
        const unsigned jo = swap1(o);
        const unsigned ja = odd ? jo : o, jb = odd ? o : jo;
        const double4 x4 = lp_d4(rx, ja, jb, odd);
        xj[u] = make_double3(x4.x, x4.y, x4.z);
      } else {
        xj[u] = ld_d3(rx, o * 32u);
      }
      tj[u] = NT1 ? 1 : (tb ? ent_type((unsigned)jn[u], nt1 - 1) : ld_i32(rt, o * 4u));
    }
    chunk_idx<G, U, IV>(rn, k0 + G * U, lane, el, jn);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const RhoPair c = NT1 ? c1 : s_c[it * nt1 + tj[u]];
      double wf = 1.0 - rsq * c.ihsq;
      wf = wf * wf;
      wf = wf * wf;
      const bool in = chunk_pos<G, U, IV>(k0, el, u) < end;
      acc += (in && rsq < c.cutsq) ? c.mK * wf : 0.0;
      if (TIGHT) {
        const bool hit = in && rsq < (NT1 ? fc1 : s_fc[it * nt1 + tj[u]]);
        const unsigned long long m = (__ballot(hit) >> gbase) & gmask;
        if (hit) s_tq[gq][tq + __popcll(m & below)] = jc[u];
        tq += __popcll(m);
      }
    }
    if (TIGHT) {  // store the complete 16-B groups, keep the remainder (< 4) buffered
      // (a group's lanes are one wave: its LDS accesses complete in program order, and
      // the compiler keeps may-aliasing LDS accesses in order, so no barrier is needed)
      const int nfull = tq & ~3, rem = tq - nfull;
      for (int k = lane; 4 * k < nfull; k += G)
        *reinterpret_cast<int4 *>(trow + tw + 4 * k) = *reinterpret_cast<const int4 *>(&s_tq[gq][4 * k]);
      const int carry = lane < rem ? s_tq[gq][nfull + lane] : 0;
      if (lane < rem) s_tq[gq][lane] = carry;
      tw += nfull;
      tq = rem;
    }
  }
  acc = group_sum<G>(acc);
  if (TIGHT && live && lane == 0) {
    if (tq > 0)
      *reinterpret_cast<int4 *>(trow + tw) = *reinterpret_cast<const int4 *>(&s_tq[gq][0]);
    tcnt[row] = tw + tq;
  }
  if (lane == 0 && live) {
    const double rho = ((cf->rho_keep >> it) & 1) ? vr[row].w : cf->self_rho[it] + acc;
    vr[row].w = rho;
    xf[row].w = tait_p_over_rho2(rho, cf->rho0[it], cf->B[it]);
  }
}

template <int G, int U, int VISC, int MODE, bool NT1, bool LP, bool IV, int EXP>
__global__ void __launch_bounds__(256)
k_row2_force(int n, int nall, int ntot, const int *__restrict__ off, int stride,
             const int *__restrict__ rcnt,
             const int *__restrict__ nbr, const double4 *__restrict__ xf,
             const double4 *__restrict__ vr, const int *__restrict__ ty,
             const double *__restrict__ en, const Coefs *__restrict__ cf,
             double4 *__restrict__ fo, double *__restrict__ de, double gx, double gy,
             double gz, int pi, const int *__restrict__ rows, int tbits) {
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
  const int idx = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  const int el = entry_slot<G>(lane, pi);
  if (!LP && idx >= n) return;
  const bool live = idx < n;
  const bool odd = (threadIdx.x & 1) != 0;
  const Rsrc rn = make_rsrc(nbr, nbytes<int>(ntot));
  const Rsrc rx = make_rsrc(xf, nbytes<double4>(nall));
  const Rsrc rv = make_rsrc(vr, nbytes<double4>(nall));
  const Rsrc rt = make_rsrc(ty, nbytes<int>(nall));
  const Rsrc re = make_rsrc(en, HEAT ? nbytes<double>(nall) : 0u);
  const int rr = rows ? rows[live ? idx : n - 1] : (live ? idx : n - 1);
  const int row = rr;
  const bool tb = !NT1 && tbits != 0;
  const double4 xi = xf[rr];
  const double4 vi = vr[rr];
  const double ei = HEAT ? en[rr] : 0.0;
  const int it = NT1 ? 1 : ty[rr];
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  // stride > 0: fixed-stride rows (row rr at rr*stride, rcnt[rr] entries), else CSR
  const int beg = stride > 0 ? rr * stride : off[rr];
  const int end = live ? (stride > 0 ? beg + rcnt[rr] : off[rr + 1]) : beg;
  double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
  int jn[U];
  chunk_idx<G, U, IV>(rn, beg, lane, el, jn);
  for (int k0 = beg; LP ? __any(chunk_pos<G, U, IV>(k0, el, 0) < end)
                        : chunk_pos<G, U, IV>(k0, el, 0) < end;
       k0 += G * U) {
    double4 xj[U], vj[U];
    double ej[U];
    int tj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const unsigned o = ent_atom((unsigned)jn[u], tb);
      if (EXP == 2) {
        xj[u] = make_double4(xi.x + 0.25 * (double)(o & 7u), xi.y + 0.5,
                             xi.z - 0.125 * (double)(o & 3u), xi.w);
        vj[u] = make_double4(vi.x, vi.y - 0.01 * (double)(o & 1u), vi.z, vi.w);
      } else if (LP) {
        const unsigned jo = swap1(o);
        const unsigned ja = odd ? jo : o, jb = odd ? o : jo;
        xj[u] = lp_d4(rx, ja, jb, odd);
        vj[u] = lp_d4(rv, ja, jb, odd);
      } else {
        xj[u] = ld_d4(rx, o * 32u);
        vj[u] = ld_d4(rv, o * 32u);
      }
      ej[u] = HEAT ? ld_d1(re, o * 8u) : 0.0;
      tj[u] = NT1 ? 1 : (tb ? ent_type((unsigned)jn[u], nt1 - 1) : ld_i32(rt, o * 4u));
    }
    chunk_idx<G, U, IV>(rn, k0 + G * U, lane, el, jn);
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (EXP == 1) {
        fx += xj[u].x + vj[u].x;
        fy += xj[u].y + vj[u].y;
        fz += xj[u].z + vj[u].z;
        drho += xj[u].w + vj[u].w;
        continue;
      }
      const double dx = xi.x - xj[u].x, dy = xi.y - xj[u].y, dz = xi.z - xj[u].z;
      const double rsq = dx * dx + dy * dy + dz * dz;
      const int pidx = NT1 ? 3 : it * nt1 + tj[u];
      const bool ok = chunk_pos<G, U, IV>(k0, el, u) < end;
      const double r = sqrt1(rsq);
      if (TAIT) {
        const TaitPair c = NT1 ? t1 : s_t[pidx];
        // masked slots may hold any record (or zeros past the range check): wfd = 0
        // zeroes every finite term below; the 1/(rho_i rho_j) terms are selected away
        const bool hit = ok && rsq < c.cutsq;
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        wfd = hit ? wfd : 0.0;
        const double velx = vi.x - vj[u].x, vely = vi.y - vj[u].y, velz = vi.z - vj[u].z;
        const double dvdr = dx * velx + dy * vely + dz * velz;
        if (VISC == SPH_VISC_MONAGHAN) {
          const double q = (c.viscC * dvdr) * rcp1((rsq + c.eps) * (vi.w + vj[u].w));
          const double fvisc = dvdr < 0. ? q : 0.0;
          const double fpair = c.mm * (xi.w + xj[u].w + fvisc) * wfd;
          fx += dx * fpair;
          fy += dy * fpair;
          fz += dz * fpair;
          dE += -0.5 * fpair * dvdr;
        } else {
          double fvisc = c.viscC * rcp1(vi.w * vj[u].w);
          fvisc = hit ? fvisc * ((-c.mm) * wfd) : 0.0;
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
        const bool hit = ok && rsq < c.cutsq;
        double wfd = c.h - r;
        wfd = c.wK * (wfd * wfd);
        wfd = hit ? wfd : 0.0;
        double deltaE = c.hmD;
        deltaE *= (vi.w + vj[u].w) * rcp1(vi.w * vj[u].w);
        deltaE = hit ? deltaE * ((ei - ej[u]) * wfd) : 0.0;
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
  if (lane == 0 && live) {
    if (TAIT) {
      const double m = cf->mass[it];
      fo[row] = make_double4(fx + m * gx, fy + m * gy, fz + m * gz, drho);
    }
    de[row] = dE;
  }
}

struct Row2Args {
  RowArgs a;
  int nall, ntot;
  bool lp;   // lane-pair gathers
  bool iv;   // index vectors
  bool pi;   // pair-interleaved entry slots (entry_slot)
  int exp;   // study variants (SPH_EXP), 0 in production
  int stride = 0;                 // > 0: fixed-stride rows with counts rcnt (else a.off CSR)
  const int *rcnt = nullptr;
  int *tnbr = nullptr, *tcnt = nullptr;  // rhosum: write the tight list here (strided, LP)
  const int *rows = nullptr;             // a.n rows listed here instead of rows 0..a.n-1
  bool tbits = false;                    // typed list entries (k_neigh3 tbits)
};

// 32-bit byte offsets of every array the row2 kernels read
inline bool row2_fits(long nall, long ntot) {
  return ntot * 4L < 0x7fffffffL && nall * 32L < 0x7fffffffL;
}

template <int G, int U, bool LP, bool IV, bool TIGHT>
inline void row2_rhosum_kt(bool nt1, hipStream_t s, const Row2Args &b) {
  const RowArgs &a = b.a;
  const int grid = (int)(((long long)a.n * G + 255) / 256);
  if (grid == 0) return;
  if (nt1)
    hipLaunchKernelGGL((k_row2_rhosum<G, U, true, LP, IV, TIGHT>), dim3(grid), dim3(256), 0, s,
                       a.n, b.nall, b.ntot, a.off, b.stride, b.rcnt, a.nbr, a.xf, a.ty, a.vr,
                       a.cf, b.tnbr, b.tcnt, b.pi ? 1 : 0, b.rows, b.tbits ? 1 : 0);
  else
    hipLaunchKernelGGL((k_row2_rhosum<G, U, false, LP, IV, TIGHT>), dim3(grid), dim3(256), 0, s,
                       a.n, b.nall, b.ntot, a.off, b.stride, b.rcnt, a.nbr, a.xf, a.ty, a.vr,
                       a.cf, b.tnbr, b.tcnt, b.pi ? 1 : 0, b.rows, b.tbits ? 1 : 0);
}
template <int G, int U, bool LP, bool IV>
inline void row2_rhosum_k(bool nt1, hipStream_t s, const Row2Args &b) {
  if (LP && b.tnbr) row2_rhosum_kt<G, U, LP, IV, LP>(nt1, s, b);
  else row2_rhosum_kt<G, U, LP, IV, false>(nt1, s, b);
}

template <int G, int U>
inline void row2_rhosum_gu(bool nt1, hipStream_t s, const Row2Args &b) {
  const bool iv = b.iv && U == 4;
  if (b.lp) {
    if (iv) row2_rhosum_k<G, U, true, U == 4>(nt1, s, b);
    else row2_rhosum_k<G, U, true, false>(nt1, s, b);
  } else {
    if (iv) row2_rhosum_k<G, U, false, U == 4>(nt1, s, b);
    else row2_rhosum_k<G, U, false, false>(nt1, s, b);
  }
}

template <int G, int U, int VISC, int MODE, bool NT1, bool LP, bool IV, int EXP>
inline void row2_force_t(hipStream_t s, const Row2Args &b) {
  const RowArgs &a = b.a;
  const int grid = (int)(((long long)a.n * G + 255) / 256);
  if (grid == 0) return;
  hipLaunchKernelGGL((k_row2_force<G, U, VISC, MODE, NT1, LP, IV, EXP>), dim3(grid), dim3(256),
                     0, s, a.n, b.nall, b.ntot, a.off, b.stride, b.rcnt, a.nbr, a.xf, a.vr,
                     a.ty, a.en, a.cf, a.fo, a.de, a.gx, a.gy, a.gz, b.pi ? 1 : 0, b.rows,
                     b.tbits ? 1 : 0);
}

template <int G, int U, bool NT1, bool LP, bool IV>
inline void row2_force_n(int visc, int mode, hipStream_t s, const Row2Args &b) {
  const bool mor = visc == SPH_VISC_MORRIS;
  switch (mode) {
    case M_TAIT:
      if (mor) row2_force_t<G, U, 1, M_TAIT, NT1, LP, IV, 0>(s, b);
#ifdef SPH_STUDY  // (outputs meaningless: study builds only, make STUDY=1)
      else if (NT1 && b.exp == 1) row2_force_t<G, U, 0, M_TAIT, NT1, LP, IV, 1>(s, b);
      else if (NT1 && b.exp == 2) row2_force_t<G, U, 0, M_TAIT, NT1, LP, IV, 2>(s, b);
#endif
      else row2_force_t<G, U, 0, M_TAIT, NT1, LP, IV, 0>(s, b);
      break;
    case M_TAIT | M_HEAT:
      if (mor) row2_force_t<G, U, 1, M_TAIT | M_HEAT, NT1, LP, IV, 0>(s, b);
      else row2_force_t<G, U, 0, M_TAIT | M_HEAT, NT1, LP, IV, 0>(s, b);
      break;
    default: row2_force_t<G, U, 0, M_HEAT, NT1, LP, IV, 0>(s, b); break;
  }
}

template <int G, int U, bool LP, bool IV>
inline void row2_force_l(bool nt1, int visc, int mode, hipStream_t s, const Row2Args &b) {
  if (nt1) row2_force_n<G, U, true, LP, IV>(visc, mode, s, b);
  else row2_force_n<G, U, false, LP, IV>(visc, mode, s, b);
}

template <int G, int U>
inline void row2_force_gu(bool nt1, int visc, int mode, hipStream_t s, const Row2Args &b) {
  const bool iv = b.iv && U == 4;
  if (b.lp) {
    if (iv) row2_force_l<G, U, true, U == 4>(nt1, visc, mode, s, b);
    else row2_force_l<G, U, true, false>(nt1, visc, mode, s, b);
  } else {
    if (iv) row2_force_l<G, U, false, U == 4>(nt1, visc, mode, s, b);
    else row2_force_l<G, U, false, false>(nt1, visc, mode, s, b);
  }
}

// (G lanes per row, U pairs per lane) shapes; SPH_ROW2TILE picks one in study builds
// (tuning); the production build has the measured fastest, 8 x 4
#ifdef SPH_STUDY
#define SPH_ROW2_TILES(X) X(0, 16, 2) X(1, 8, 2) X(2, 16, 4) X(3, 8, 4) X(4, 4, 4)
#else
#define SPH_ROW2_TILES(X) X(3, 8, 4)
#endif

int row2_tile();

// lanes per row of the selected shape when it can walk a chunk-transposed list (U = 4),
// else 0
inline int row2_iv_g() {
  switch (row2_tile()) {
#define SPH_CASE(k, G, U) \
  case k: return U == 4 ? G : 0;
    SPH_ROW2_TILES(SPH_CASE)
#undef SPH_CASE
    default: return 8;
  }
}

inline void row2_rhosum(bool nt1, hipStream_t s, const Row2Args &b) {
  switch (row2_tile()) {
#define SPH_CASE(k, G, U) \
  case k: row2_rhosum_gu<G, U>(nt1, s, b); break;
    SPH_ROW2_TILES(SPH_CASE)
#undef SPH_CASE
    default: row2_rhosum_gu<8, 4>(nt1, s, b); break;
  }
}

inline void row2_force(bool nt1, int visc, int mode, hipStream_t s, const Row2Args &b) {
  switch (row2_tile()) {
#define SPH_CASE(k, G, U) \
  case k: row2_force_gu<G, U>(nt1, visc, mode, s, b); break;
    SPH_ROW2_TILES(SPH_CASE)
#undef SPH_CASE
    default: row2_force_gu<8, 4>(nt1, visc, mode, s, b); break;
  }
}

}  // namespace sph
