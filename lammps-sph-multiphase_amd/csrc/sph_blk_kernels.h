// sph_blk_kernels.h -- block-staged pair passes of the engine (production path).
//
// What bounds a gather-per-pair walk of the full list on gfx950 is the texture addresser
// (TA): every pair fetches its neighbour's 32-B records from L2 and the TA prices each
// wave instruction by the distinct 128-B lines it touches (round-1 row2
// kernels: TA_BUSY 93 %, 338 TA cycles per particle per taitwater pass).  Here the gathers
// move into LDS:
//
//  * a BLOCK is R consecutive owned rows (Morton order, so a compact region of space);
//    its UNION is the sorted set of atoms (owned or ghost) that appear in any of its rows'
//    full-list entries -- at C2 (R = 64, h = 3 dx) about 950 atoms against 64 x 155
//    entries, so each record is loaded ~10x less often than by per-pair gathers;
//  * at every rebuild k_blk_build turns the block's rows into 16-bit SLOTS (positions in
//    the union), each row's slots sorted ascending (atom order: lanes of a row read
//    mostly consecutive LDS records) and stored chunk-transposed like the row2 list, so a
//    lane's four slots of a chunk are one 8-byte load.  The index stream of a pass halves
//    (2 B per entry instead of 4);
//  * each pass stages its block's union records into LDS with coalesced loads (the union
//    is sorted by atom index, so a wave's loads hit consecutive records), then the rows'
//    G lanes walk their slot lists reading neighbour records from LDS (ds_read_b128).
//
// Pair arithmetic is the row2 kernels' (sph_row2_kernels.h: v_rcp/v_rsq seeds with one
// Newton step, masked slots get a zero kernel weight), so results agree with the row
// path to rounding of the summation order.  Reference semantics: rhosum
// pair_sph_rhosum.cpp:116-195 (full list, strict rsq < cutsq), taitwater
// pair_sph_taitwater.cpp:117-191, morris pair_sph_taitwater_morris.cpp:156-191,
// heatconduction pair_sph_heatconduction.cpp:106-129 -- each pair evaluated from both
// sides of the full list (Newton's third law by symmetry, no scatter, no atomics).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <utility>

#include "sph_engine_kernels.h"
#include "sph_row2_kernels.h"
#include "sph_util.h"

namespace sph {

constexpr int BLK_TPR = 16;     // lanes per row of k_blk_neigh

// exclusive prefix sum over the BT threads of a workgroup (BT/64 waves); *total = sum
template <int BT>
__device__ __forceinline__ int blk_scan(int v, int *s_w, int *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < BT / 64; k++) {
    const int t = s_w[k];
    base += (k < w) ? t : 0;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// Slot rows are stored chunk-transposed: a chunk holds U*G consecutive entries (ascending
// slots) of a row; lane l of the row's G lanes holds entries l, l+G, .., l+(U-1)G of it in
// ONE word (U 16-bit slots: an 8-byte load for U = 4) at storage position U*l.  So the G
// lanes of a walk step q take G consecutive entries (consecutive LDS records, and a row
// that ends inside a chunk stops after ceil(rest/G) steps: granularity G, not U*G), and each
// lane still reads its slots of a chunk with one load.  Logical entry e -> storage position:
template <int G, int U>
__host__ __device__ __forceinline__ int blk_tpos(int e) {
  return (e / (U * G)) * (U * G) + (e % G) * U + (e % (U * G)) / G;
}

// v_writelane_b32 through its LLVM intrinsic (no clang builtin here; the compiler then
// knows the instruction and inserts the SGPR-write -> lane-read wait states)
__device__ int sph_writelane_i32(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
// lane LANE of v takes the wave-uniform value `val`
template <int LANE>
__device__ __forceinline__ unsigned writelane(unsigned v, unsigned val) {
  return (unsigned)sph_writelane_i32((int)val, LANE, (int)v);
}

// ---- the union image ---------------------------------------------------------------------
// A block's union sits in LDS as an image of 16-slot chunks.  Slot s = union position + 1;
// slot 0 is a sentinel far from every atom (x = 1e100: every pair test fails, every pair
// term is a finite value times a zero kernel weight), so padded list positions need no
// bounds test.  A chunk holds its 16 slots' arrays back to back -- a0 (x, y) at +0,
// a1 (z, P/rho^2) at +256, a2 (vx, vy) at +512, a3 (vz, rho) at +768, e at +1024 (heat,
// 16-byte stride like the others) -- CH = 1024 (1280 with e) bytes, and a slot-row word
// holds q = (s/16)*(CH/16) + s%16, the
// slot's byte offset / 16: every array of the slot is one immediate offset from q*16, and
// 16 consecutive slots of one array cover the 64 banks once (ds_read_b128: 16 lanes per
// LDS cycle).  The rho pass keeps a compact image of its own (x, y at 16 s; z at 16 S + 8 s
// for S slots) and decodes s from q.
constexpr int BLK_CH = 1024, BLK_CHE = 1280;
// the force pass's VISC for one type with Monaghan viscosity and viscC = 0 (no viscosity
// term; the engine selects it, sph_engine.hip force_pass)
constexpr int BLK_VISC_NONE = 2;
// Newton-3 inside the blocks (k_blk_build N3 + the passes' LDS share accumulators): measured
// slower on gfx950 (force 0.291 -> 0.313 ms, build 1.60 -> 2.18 ms at C2 1M),
// so only study builds carry it (SPH_N3=1)
#ifdef SPH_STUDY
constexpr bool BLK_N3_BUILT = true;
#else
constexpr bool BLK_N3_BUILT = false;
#endif
__host__ __device__ inline int blk_q(int s, int cq) { return (s >> 4) * cq + (s & 15); }
template <int CQ>
__device__ __forceinline__ int blk_s(int q) { return (q / CQ) * 16 + (q % CQ); }
// the rho pass's image: S = u + 1 slots of (x, y), z [, type]
__host__ __device__ inline size_t blk_rho_lds(int u, bool nt1) {
  const size_t S = (size_t)u + 1;
  return S * 24 + (nt1 ? 0 : (S + 15) / 16 * 16);
}
// LDS bytes of an image for u union atoms (+ the sentinel), with the per-slot type bytes
// (indexed by q) after it when there are several types
__host__ __device__ inline size_t blk_lds(int u, int cq, bool nt1) {
  const size_t nch = ((size_t)u + 16) / 16;
  return nch * cq * 16 + (nt1 ? 0 : (nch * cq + 15) / 16 * 16);
}
// stage atom j's record into slot s of the image (cq*16-byte chunks)
template <bool HEAT>
__device__ __forceinline__ void blk_put(unsigned char *img, int s, int cq, const double4 &x,
                                        const double4 &v, double e) {
  unsigned char *const r = img + (size_t)(s >> 4) * cq * 16 + (s & 15) * 16;
  *reinterpret_cast<double2 *>(r) = make_double2(x.x, x.y);
  *reinterpret_cast<double2 *>(r + 256) = make_double2(x.z, x.w);
  *reinterpret_cast<double2 *>(r + 512) = make_double2(v.x, v.y);
  *reinterpret_cast<double2 *>(r + 768) = make_double2(v.z, v.w);
  if (HEAT) *reinterpret_cast<double *>(r + 1024) = e;
}
// the sentinel (slot 0): far away, at rest, P/rho^2 = 0, rho = 1, e = 0
template <bool HEAT>
__device__ __forceinline__ void blk_put_sentinel(unsigned char *img) {
  blk_put<HEAT>(img, 0, 0, make_double4(1e100, 1e100, 1e100, 0.0),
                make_double4(0.0, 0.0, 0.0, 1.0), 0.0);
}

// ---- block neighbour build from the bins ------------------------------------------------
// One 256-thread workgroup per block of R rows builds the block's rows DIRECTLY in slot
// form, without a global-index list: Neighbor::full_bin membership (neigh_full.cpp:241-344:
// every j != i with rsq <= cutneighsq[it][jt]) over the half-size bins of k_neigh3.
//  1. each row trims its 5x5 (dz, dy) bin-rows to the x-range that can hold a point within
//     cutneighmax (k_neigh3's conservative slab test); the block's CANDIDATES are, per
//     bin-row, the union of its rows' x-ranges -- one contiguous range of the bin-sorted
//     copy xb per bin-row, numbered in bin order;
//  2. the candidates are staged in LDS BLK_WIN at a time (coalesced loads from xb); each
//     row's lanes walk only the row's OWN trimmed ranges (sub-ranges of the block's, so the
//     same ~N_f/0.7 tests per row as k_neigh3) and set a hit bit per candidate;
//  3. the union is the candidates some row hit, numbered in candidate order (slot = rank
//     among used candidates); each row's slots come out of its bitmap in ascending order.
// Candidate ORDER differs from full_bin's (bins are scanned per block), which changes only
// the summation order of the pair passes.  Overflows (> BLK_MCAP candidates, or a block
// whose bin box exceeds the bin-row table) raise *ovf; the host then takes the row path.
constexpr int BLK_MCAP = 4096;  // candidates per block (hit bitmaps)
constexpr int BLK_MBIG = 8192;  // ... in the large-image variant (wide blocks, small boxes)
constexpr int BLK_UCAP = BLK_MBIG;  // union stride of ulist
constexpr int BLK_WIN = 512;    // candidates staged in LDS at a time
constexpr int BLK_TBL = 256;    // bin-rows per block

template <int R, int G, int U, bool NT1, int MC>
__global__ void __launch_bounds__(R * BLK_TPR)
k_blk_neigh(int n, QBins q, int dim, const double4 *__restrict__ xf, const int *__restrict__ ty,
            const double4 *__restrict__ xb, const int *__restrict__ tb,
            const int *__restrict__ qbeg, const int *__restrict__ xpos,
            const Coefs *__restrict__ cf, int ucap, int sstride,
            int *__restrict__ ulist, int *__restrict__ ucnt, int *__restrict__ rcnt,
            unsigned short *__restrict__ snbr, int *__restrict__ ovf, int *__restrict__ umax,
            int cq, int bexp) {
  // bexp (study builds only, SPH_BEXP; outputs meaningless): 1 = no candidate loads, 2 = no row
  // tests, 4 = no slot-row stores, 8 = no union stores
  constexpr int TPR = BLK_TPR, BLK_BT = R * TPR;
  constexpr int W = MC / 32;
  constexpr int RB = 2, NB = (2 * RB + 1) * (2 * RB + 1);
  static_assert(BLK_BT <= 1024 && BLK_BT >= BLK_TBL && (TPR & (TPR - 1)) == 0, "block shape");
  __shared__ double2 s_cxy[BLK_WIN];
  __shared__ double s_cz[BLK_WIN];
  __shared__ int s_cid[BLK_WIN];
  __shared__ unsigned char s_ct[NT1 ? 1 : BLK_WIN];
  __shared__ unsigned s_bm[R][W];
  __shared__ unsigned s_used[W];
  __shared__ int s_upre[W + 1];
  __shared__ int s_x0[BLK_TBL], s_x1[BLK_TBL], s_pre[BLK_TBL + 1], s_st[BLK_TBL];
  __shared__ int s_rc[R][NB];       // first candidate of each of the row's bin-row ranges
  __shared__ int s_rl[R][NB];       // its length
  __shared__ int s_lim[6];          // min/max bin y, z of the rows
  __shared__ double s_cns[NT1 ? 1 : NT2];
  __shared__ int s_w[BLK_BT / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int r = tid / TPR, sub = tid % TPR;
  const int row = b * R + r;
  const bool live = row < n;
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = tid; t < nt1 * nt1; t += BLK_BT) s_cns[t] = cf->cutneighsq[t];
  if (tid < 6) s_lim[tid] = (tid & 1) ? -0x7fffffff : 0x7fffffff;
  for (int t = tid; t < BLK_TBL; t += BLK_BT) {
    s_x0[t] = 0x7fffffff;
    s_x1[t] = -1;
  }
  __syncthreads();
  const double4 xi = xf[live ? row : 0];
  const int it = NT1 ? 1 : ty[live ? row : 0];
  const int cx = bin_coord(xi.x, q.lo[0], q.inv[0], q.nb[0]);
  const int cy = bin_coord(xi.y, q.lo[1], q.inv[1], q.nb[1]);
  const int cz = bin_coord(xi.z, q.lo[2], q.inv[2], q.nb[2]);
  (void)cx;
  if (live && sub == 0) {
    atomicMin(&s_lim[0], cy);
    atomicMax(&s_lim[1], cy);
    atomicMin(&s_lim[2], cz);
    atomicMax(&s_lim[3], cz);
  }
  __syncthreads();
  const int y0 = s_lim[0] - RB, z0 = (dim == 3) ? s_lim[2] - RB : cz;
  const int ny = s_lim[1] - s_lim[0] + 2 * RB + 1;
  const int nz = (dim == 3) ? s_lim[3] - s_lim[2] + 2 * RB + 1 : 1;
  if (ny * nz > BLK_TBL) {  // workgroup-uniform
    if (tid == 0) atomicMax(ovf, 1 << 20);
    return;
  }
  // 1) per-row trimmed bin-row x-ranges (kept per row: table entry, bx0, bx1), merged per
  // block bin-row
  const int nbr_rows = (dim == 3) ? NB : (2 * RB + 1);
  int myt[(NB + TPR - 1) / TPR], mx0[(NB + TPR - 1) / TPR], mx1[(NB + TPR - 1) / TPR];
#pragma unroll
  for (int k = 0; k < (NB + TPR - 1) / TPR; k++) {
    const int br = sub + k * TPR;
    myt[k] = -1;
    mx0[k] = 0;
    mx1[k] = -1;
    if (!live || br >= nbr_rows) continue;
    const int bz = (dim == 3) ? cz - RB + br / (2 * RB + 1) : cz;
    const int by = cy - RB + br % (2 * RB + 1);
    if (bz < 0 || bz >= q.nb[2] || by < 0 || by >= q.nb[1]) continue;
    const double gz = (dim == 3) ? slab_gap(xi.z, bz, cz, q.lo[2], q.size[2]) : 0.0;
    const double gy = slab_gap(xi.y, by, cy, q.lo[1], q.size[1]);
    const double d2 = gy * gy + gz * gz;
    if (d2 > q.cutmaxsq) continue;
    const double ext = sqrt(q.cutmaxsq - d2) * (1.0 + 1e-9) + 1e-9 * q.size[0];
    const int bx0 = bin_coord(xi.x - ext, q.lo[0], q.inv[0], q.nb[0]);
    const int bx1 = bin_coord(xi.x + ext, q.lo[0], q.inv[0], q.nb[0]);
    const int t = (bz - z0) * ny + (by - y0);
    myt[k] = t;
    mx0[k] = bx0;
    mx1[k] = bx1;
    atomicMin(&s_x0[t], bx0);
    atomicMax(&s_x1[t], bx1);
  }
  __syncthreads();
  // 2) candidate ranges (one per table entry, in linear bin order) and their prefix
  int len = 0, st = 0;
  if (tid < ny * nz && s_x1[tid] >= s_x0[tid]) {
    const int bz = z0 + tid / ny, by = y0 + tid % ny;
    const int brow = (bz * q.nb[1] + by) * q.nb[0];
    st = qbeg[brow + s_x0[tid]];
    len = qbeg[brow + s_x1[tid] + 1] - st;
  }
  int M = 0;
  const int pre = blk_scan<BLK_BT>(len, s_w, &M);
  if (M > MC) {
    if (tid == 0) atomicMax(ovf, M);
    return;
  }
  if (tid < BLK_TBL) {
    s_pre[tid] = pre;
    s_st[tid] = st;
  }
  if (tid == 0) s_pre[BLK_TBL] = M;
  for (int t = tid; t < R * W; t += BLK_BT) (&s_bm[0][0])[t] = 0u;
  __syncthreads();
  // the row's ranges in candidate numbering: xb positions [qbeg(bx0), qbeg(bx1 + 1)) of
  // bin-row t sit at candidates s_pre[t] + (pos - s_st[t])
#pragma unroll
  for (int k = 0; k < (NB + TPR - 1) / TPR; k++) {
    const int br = sub + k * TPR;
    if (br >= NB) continue;
    int c0 = 0, ln = 0;
    if (myt[k] >= 0) {
      const int t = myt[k];
      const int bz = z0 + t / ny, by = y0 + t % ny;
      const int brow = (bz * q.nb[1] + by) * q.nb[0];
      const int a = qbeg[brow + mx0[k]];
      c0 = s_pre[t] + (a - s_st[t]);
      ln = qbeg[brow + mx1[k] + 1] - a;
    }
    s_rc[r][br] = c0;
    s_rl[r][br] = ln;
  }
  int cntr = 0;  // the row's hits (this lane's share)
  // 3) candidates staged BLK_WIN at a time; the row's lanes walk each of the row's ranges
  // (a contiguous run of candidates, clipped to the window) and set a bit per hit
  const double cns1 = NT1 ? cf->cutneighsq[3] : 0.0;
  const double *const crow = s_cns + (NT1 ? 0 : it * nt1);
  for (int p0 = 0; p0 < M; p0 += BLK_WIN) {
    const int pn = min(M - p0, BLK_WIN);
    __syncthreads();  // (the previous window's tests are done; s_rc/s_rl are visible)
#pragma unroll 2
    for (int pw = tid; pw < pn; pw += BLK_BT) {
      const int p = p0 + pw;
      int lo = 0, hi = BLK_TBL - 1;  // last table entry with s_pre <= p (a non-empty range)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= p) lo = mid;
        else hi = mid - 1;
      }
      const int pos = s_st[lo] + (p - s_pre[lo]);
      if (bexp & 1) continue;
      const double4 c = xb[pos];
      s_cxy[pw] = make_double2(c.x, c.y);
      s_cz[pw] = c.z;
      s_cid[pw] = (int)c.w;
      if (!NT1) s_ct[pw] = (unsigned char)tb[pos];
    }
    __syncthreads();
    if (!live || (bexp & 2)) continue;
    for (int br = 0; br < nbr_rows; br++) {
      const int c0 = s_rc[r][br], c1 = c0 + s_rl[r][br];
      const int lo = max(c0, p0), hi = min(c1, p0 + pn);
      for (int p = lo + sub; p < hi; p += TPR) {
        const int pw = p - p0;
        const double2 cxy = s_cxy[pw];
        const double rsq = rsq_ref(xi.x - cxy.x, xi.y - cxy.y, xi.z - s_cz[pw]);
        if (rsq <= (NT1 ? cns1 : crow[s_ct[pw]]) && s_cid[pw] != row) {
          atomicOr(&s_bm[r][p >> 5], 1u << (p & 31));
          cntr++;
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int d = TPR >> 1; d > 0; d >>= 1) cntr += __shfl_xor(cntr, d, TPR);
  const int Mw = (M + 31) >> 5;
  // 4) used candidates -> slots (rank in candidate order); the union list
  for (int w = tid; w < Mw; w += BLK_BT) s_used[w] = 0u;
  __syncthreads();
  {  // the OR over rows: (word, row group) per thread, then one LDS atomic per pair
    constexpr int RG = 8;  // rows per thread
    for (int t = tid; t < Mw * (R / RG); t += BLK_BT) {
      const int w = t % Mw, r0 = (t / Mw) * RG;
      unsigned o = 0u;
#pragma unroll
      for (int rr = 0; rr < RG; rr++) o |= s_bm[r0 + rr][w];
      if (o) atomicOr(&s_used[w], o);
    }
  }
  __syncthreads();
  int u = 0;
  {
    const int v = tid < Mw ? __popc(s_used[tid]) : 0;
    const int ex = blk_scan<BLK_BT>(v, s_w, &u);
    if (tid < Mw) s_upre[tid] = ex;
  }
  __syncthreads();
  for (int p = tid; p < M; p += BLK_BT) {  // (atom ids of used candidates from xb)
    const unsigned wbits = s_used[p >> 5];
    if (((wbits >> (p & 31)) & 1u) && !(bexp & 8)) {
      int lo = 0, hi = BLK_TBL - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= p) lo = mid;
        else hi = mid - 1;
      }
      ulist[(size_t)b * ucap + s_upre[p >> 5] + __popc(wbits & ((1u << (p & 31)) - 1u))] =
          (int)xb[s_st[lo] + (p - s_pre[lo])].w;
    }
  }
  if (tid == 0) {
    ucnt[b] = u;
    atomicMax(umax, u);
    atomicMax(umax + 1, M);   // (stats: largest candidate set, sums of candidates / unions)
    atomicAdd(umax + 2, M);
    atomicAdd(umax + 3, u);
  }
  if (!live) return;
  // 5) the row's slots in ascending order (its TPR lanes take consecutive word ranges)
  const int wp = (Mw + TPR - 1) / TPR;
  const int w0 = min(sub * wp, Mw), w1 = min(w0 + wp, Mw);
  int pc = 0;
  for (int w = w0; w < w1; w++) pc += __popc(s_bm[r][w]);
  int x = pc;
#pragma unroll
  for (int d = 1; d < TPR; d <<= 1) {
    const int y = __shfl_up(x, d, TPR);
    if (sub >= d) x += y;
  }
  int qq = x - pc;
  unsigned short *const out = snbr + (size_t)row * sstride;
  for (int w = w0; w < w1; w++) {
    unsigned m = s_bm[r][w];
    const unsigned used = s_used[w];
    const int base = s_upre[w];
    while (m) {
      const int bit = __ffs(m) - 1;
      m &= m - 1;
      if (qq < sstride && !(bexp & 4))
        out[blk_tpos<G, U>(qq)] =
            (unsigned short)blk_q(base + 1 + __popc(used & ((1u << bit) - 1u)), cq);
      qq++;
    }
  }
  if (sub == 0) {
    rcnt[row] = cntr;
    if (cntr > sstride) atomicMax(ovf, 1 << 21);
  }
  const int cend = min((cntr + U * G - 1) / (U * G) * (U * G), sstride);
  for (int k = cntr + sub; k < cend; k += TPR) out[blk_tpos<G, U>(k)] = 0;  // the sentinel
}

// ---- block neighbour build v2: every row against the block's candidates, ballots --------
// One workgroup (4 waves) per block of R <= 64 rows.
//  1. The block's bounding box; the bins within cutneighmax of it (per (y, z) bin-row the
//     x-range is cut to the sphere-swept box): one contiguous xb range per bin-row, the RAW
//     candidates, numbered in bin order.
//  2. Prefilter: a raw candidate farther than cutneighmax from the box cannot be anyone's
//     neighbour; the others (~60 % at C2) are compacted, in raw order, into the block's
//     CANDIDATES (their xb positions in LDS).
//  3. A wave takes 64 candidates at a time, one per lane, and runs every row of the block
//     against them: the rows' positions are in LDS (broadcast reads), eight rows per
//     unrolled step; the test is Neighbor::full_bin's (rsq <= cutneighsq, j != i;
//     neigh_full.cpp:305-312) and its ballot is the row's 64-bit hit word for those
//     candidates, kept in lane r's registers -- no atomics, no per-row range bookkeeping.
//     A second ballot (rsq < (cut + inner margin)^2) gives the inner rows (k_blk_inner's)
//     in the same pass.
//  4. The union is the OR of the rows' words (candidate order); slots are ranks among used
//     candidates, as in k_blk_neigh, whose outputs (ulist, ucnt, rcnt, chunk-transposed
//     16-bit slot rows, the same overflow and statistics words) this kernel produces.
// Overflow (> BLK_MCAP raw or BLK_SCAP kept candidates, or a bin box wider than BLK_TBL
// bin-rows) raises *ovf and the host falls back to k_blk_neigh.
constexpr int BLK_SCAP = 2048;  // kept candidates per block (k_blk_build)
// ... in the small variant, chosen when the previous build's largest block fitted it: 40 KiB
// of LDS, four workgroups per CU instead of three (a block past it raises 1 << 24 and the
// host builds again with BLK_SCAP).  C2 1M: largest kept set 1489-1494, mean 1017
constexpr int BLK_SCAP_S = 1536;
// set bits of a wave-uniform 64-bit mask below this lane (v_mbcnt_lo / v_mbcnt_hi)
__device__ __forceinline__ int blk_mbcnt(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// f(std::integral_constant<int, r>) for r = 0 .. N-1, unrolled at compile time
template <int N, class F, int... I>
__device__ __forceinline__ void blk_rows_(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void blk_rows(F &&f) {
  blk_rows_<N>(f, std::make_integer_sequence<int, N>{});
}
// a wave-uniform 64-bit value into scalar registers
__device__ __forceinline__ unsigned long long blk_uniform64(unsigned long long x) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)x);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(x >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
// BEXP (study builds, SPH_BEXP with the build v2): 1 = return after the bin table, 2 = after
// the candidates, 3 = no emit (rows not written), 4 = no tests (every word 0).  Outputs
// meaningless.
// N3 (Newton's third law inside the block): the union puts the block's own rows first
// (slot r + 1 = row r, whether or not a list names it), and a row keeps a neighbour that is
// another row of the block only if that row comes after it -- each such pair is evaluated
// once, by its earlier row, which also accumulates the later row's share (the pair passes'
// LDS accumulators).  rcnt/icnt then hold the rows' stored (N3) counts and fcnt the full
// counts (Neighbor::full_bin's, for the neighbour statistics).
template <int R, int G, int U, bool NT1, bool INNER, bool N3, int BEXP = 0, int SC = BLK_SCAP>
__global__ void __launch_bounds__(256)
k_blk_build(int n, QBins q, int dim, const double4 *__restrict__ xf,
            const int *__restrict__ ty, const double4 *__restrict__ xb,
            const int *__restrict__ tb, const int *__restrict__ qbeg,
            const Coefs *__restrict__ cf, int ucap, int sstride, int *__restrict__ ulist,
            int *__restrict__ ucnt, int *__restrict__ rcnt, unsigned short *__restrict__ snbr,
            int *__restrict__ icnt, unsigned short *__restrict__ snbi,
            int *__restrict__ ovf, int *__restrict__ umax, int cq, int *__restrict__ fcnt,
            unsigned char *__restrict__ bperm, int *__restrict__ uilist,
            int *__restrict__ uicnt, int *__restrict__ kcnt) {
  constexpr int NT = 256, NW = NT / 64, MCH = BLK_MCAP / 64, SCH = SC / 64;
  constexpr int RPW = R / NW, UG = U * G, WS = INNER ? 2 : 1;
  // the INNER UNION (uilist != nullptr): the inner rows index a union of their own -- the
  // atoms some inner row names, ~15 % fewer than the full union at C2 -- so the passes stage
  // a smaller LDS image while the inner rows are live (more workgroups per CU)
  const bool iu = INNER && !N3 && uilist != nullptr;
  static_assert(R <= 64 && R % 32 == 0, "one lane per row, rows in steps of 8 per wave");
  static_assert(UG <= 64, "a row's padding in one store");
  // the rows' hit words per chunk (full, inner); before the tests the same storage holds
  // the raw candidates' bin-row numbers
  __shared__ __attribute__((aligned(16))) unsigned long long s_w[SCH * R * WS];
  static_assert(SCH * R * WS * 8 >= BLK_MCAP, "the bin-row table fits the hit words");
  unsigned char *const s_rowof = reinterpret_cast<unsigned char *>(s_w);
  __shared__ unsigned long long s_used[SCH];
  __shared__ unsigned long long s_usedi[INNER ? SCH : 1];  // iu: the inner union's words
  __shared__ int s_upi[INNER ? SCH + 1 : 1];
  __shared__ unsigned short s_q[SCH][64];
  __shared__ unsigned long long s_keep[MCH];
  __shared__ int s_cpos[SC];
  __shared__ int s_upre[SCH + 1], s_kpre[MCH + 1];
  __shared__ int s_pre[BLK_TBL + 1], s_st[BLK_TBL];
  __shared__ double4 s_row[R];
  __shared__ int s_rty[R];
  __shared__ int s_self[NW][64];
  __shared__ unsigned long long s_rowm[N3 ? SCH : 1];  // N3: kept candidates that are rows
  __shared__ int s_fc[N3 ? R : 1];                      // N3: the rows' full counts
  __shared__ double s_bb[6];
  __shared__ double s_cns[NT1 ? 1 : NT2], s_cin[(NT1 || !INNER) ? 1 : NT2];
  __shared__ int s_sc[NW];
  __shared__ int s_len[R];  // (bperm: the rows' walked lengths)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, 
            wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: scalar)
  const int row0 = b * R;
  const int nrow = min(R, n - row0);
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = tid; t < nt1 * nt1; t += NT) {
      s_cns[t] = cf->cutneighsq[t];
      if (INNER) s_cin[t] = cf->cutinsq[t];
    }
  if (N3 && tid < R) s_fc[tid] = 0;
  // 1) the rows (far away past the last row: never a hit) and their bounding box (wave 0)
  if (wv == 0) {
    double lo[3], hi[3];
    if (lane < R) {
      const double4 x = lane < nrow ? xf[row0 + lane] : make_double4(1e300, 1e300, 1e300, 0.0);
      s_row[lane] = x;
      if (!NT1) s_rty[lane] = lane < nrow ? ty[row0 + lane] : 1;
    }
    if (lane < nrow) {
      const double4 x = xf[row0 + lane];
      lo[0] = hi[0] = x.x;
      lo[1] = hi[1] = x.y;
      lo[2] = hi[2] = x.z;
    } else {
      lo[0] = lo[1] = lo[2] = 1e300;
      hi[0] = hi[1] = hi[2] = -1e300;
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        lo[k] = fmin(lo[k], __shfl_xor(lo[k], d, 64));
        hi[k] = fmax(hi[k], __shfl_xor(hi[k], d, 64));
      }
    if (lane == 0)
      for (int k = 0; k < 3; k++) {
        s_bb[k] = lo[k];
        s_bb[3 + k] = hi[k];
      }
  }
  __syncthreads();
  // the bin-rows of the sphere-swept box and their x-ranges (conservative margins as
  // k_neigh3's slab tests)
  const double cm = sqrt(q.cutmaxsq) * (1.0 + 1e-9);
  const int by0 = bin_coord(s_bb[1] - cm, q.lo[1], q.inv[1], q.nb[1]);
  const int by1 = bin_coord(s_bb[4] + cm, q.lo[1], q.inv[1], q.nb[1]);
  const int bz0 = dim == 3 ? bin_coord(s_bb[2] - cm, q.lo[2], q.inv[2], q.nb[2]) : 0;
  const int bz1 = dim == 3 ? bin_coord(s_bb[5] + cm, q.lo[2], q.inv[2], q.nb[2]) : 0;
  const int ny = by1 - by0 + 1, nz = bz1 - bz0 + 1;
  if (ny * nz > BLK_TBL) {  // workgroup-uniform
    if (tid == 0) atomicMax(ovf, 1 << 20);
    return;
  }
  int len = 0, st = 0;
  if (tid < ny * nz) {
    const int by = by0 + tid % ny, bz = bz0 + tid / ny;
    auto gap = [&](int bb, int k) {  // box interval to bin slab bb along axis k
      const double slo = q.lo[k] + bb * q.size[k], shi = slo + q.size[k];
      const double g = fmax(slo - s_bb[3 + k], s_bb[k] - shi);
      return fmax(g - 1e-6 * q.size[k], 0.0);
    };
    const double gy = gap(by, 1), gz = dim == 3 ? gap(bz, 2) : 0.0;
    const double d2 = gy * gy + gz * gz;
    if (d2 <= q.cutmaxsq) {
      const double ext = sqrt(q.cutmaxsq - d2) * (1.0 + 1e-9) + 1e-9 * q.size[0];
      const int bx0 = bin_coord(s_bb[0] - ext, q.lo[0], q.inv[0], q.nb[0]);
      const int bx1 = bin_coord(s_bb[3] + ext, q.lo[0], q.inv[0], q.nb[0]);
      const int brow = (bz * q.nb[1] + by) * q.nb[0];
      st = qbeg[brow + bx0];
      len = qbeg[brow + bx1 + 1] - st;
    }
  }
  int M = 0;
  const int pre = blk_scan<NT>(len, s_sc, &M);
  if (M > BLK_MCAP) {
    if (tid == 0) atomicMax(ovf, M);
    return;
  }
  const int ntab = ny * nz;
  if (tid < ntab) {
    s_pre[tid] = pre;
    s_st[tid] = st;
    for (int k = 0; k < len; k++) s_rowof[pre + k] = (unsigned char)tid;
  }
  __syncthreads();
  if (BEXP == 1) return;
  const int mch = (M + 63) >> 6;
  // raw candidate p -> its xb position
  auto rpos = [&](int p) {
    const int t = s_rowof[p];
    return s_st[t] + (p - s_pre[t]);
  };
  // 2) prefilter: distance to the box <= cutneighmax (conservative margins); two chunks per
  // step, so that their loads overlap
  const double cmsq = q.cutmaxsq * (1.0 + 1e-9) + 1e-12 * q.size[0] * q.size[0];
  auto near = [&](const double4 &x) {
    const double gx = fmax(fmax(s_bb[0] - x.x, x.x - s_bb[3]), 0.0);
    const double gy = fmax(fmax(s_bb[1] - x.y, x.y - s_bb[4]), 0.0);
    const double gz = fmax(fmax(s_bb[2] - x.z, x.z - s_bb[5]), 0.0);
    return gx * gx + gy * gy + gz * gz <= cmsq;
  };
  for (int c = wv; c < mch; c += 2 * NW) {
    const int p = c * 64 + lane, p2 = p + NW * 64;
    double4 x = make_double4(0.0, 0.0, 0.0, 0.0), x2 = x;
    if (p < M) x = xb[rpos(p)];
    if (p2 < M) x2 = xb[rpos(p2)];
    const unsigned long long k = __ballot(p < M && near(x));
    const unsigned long long k2 = __ballot(p2 < M && near(x2));
    if (lane == 0) {
      s_keep[c] = k;
      if (c + NW < mch) s_keep[c + NW] = k2;
    }
  }
  __syncthreads();
  int K = 0;
  {
    const int v = tid < mch ? __popcll(s_keep[tid]) : 0;
    const int ex = blk_scan<NT>(v, s_sc, &K);
    if (tid < mch) s_kpre[tid] = ex;
  }
  if (K > SC) {  // workgroup-uniform
    if (tid == 0) atomicMax(ovf, SC < BLK_SCAP ? (1 << 24) : (1 << 22));
    return;
  }
  __syncthreads();
  for (int c = wv; c < mch; c += NW) {
    const unsigned long long k = s_keep[c];
    if ((k >> lane) & 1ull)
      s_cpos[s_kpre[c] + __popcll(k & ((1ull << lane) - 1ull))] = rpos(c * 64 + lane);
  }
  __syncthreads();
  if (BEXP == 2) return;
  const int nch = (K + 63) >> 6;
  // 3) tests: chunk c of 64 kept candidates (one per lane) against every row; the next
  // chunk's candidates are loaded while this one is tested
  const double cns1 = NT1 ? cf->cutneighsq[3] : 0.0;
  const double cin1 = (NT1 && INNER) ? cf->cutinsq[3] : 0.0;
  auto cload = [&](int c, double4 &x, int &t) {
    const int p = c * 64 + lane;
    x = make_double4(-1e300, -1e300, -1e300, -1.0);
    t = 1;
    if (p < K) {
      const int pos = s_cpos[p];
      x = xb[pos];
      if (!NT1) t = tb[pos];
    }
  };
  double4 xn;
  int tn = 1;
  int fc = 0;  // N3: lane r's share of row r's full count
  if (wv < nch) cload(wv, xn, tn);
  for (int c = wv; c < nch; c += NW) {
    const int p = c * 64 + lane;
    const bool valid = p < K;
    const double4 xc = xn;
    const int tc = tn;
    if (c + NW < nch) cload(c + NW, xn, tn);
    const int cid = valid ? (int)xc.w : -1;
    if (valid) s_cpos[p] = cid;  // (the xb position is spent: the union takes the atom id)
    // j != i: the lane holding row r's own atom (if this chunk has it), for lane r
    s_self[wv][lane] = -1;
    if (cid >= row0 && cid < row0 + R) s_self[wv][cid - row0] = lane;
    unsigned my_lo = 0u, my_hi = 0u, mi_lo = 0u, mi_hi = 0u;
    // (an opaque 0: the compiler must not hoist the 64 rows' positions out of the chunk
    // loop into registers -- 256+ VGPRs, one wave per SIMD)
    int ro = 0;
    asm volatile("" : "+s"(ro));
    // every row, fully unrolled (lane r keeps row r's 64-bit word)
    if (BEXP != 4) blk_rows<R>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      const double4 xi = s_row[r + ro];
      const double rsq = rsq_ref(xi.x - xc.x, xi.y - xc.y, xi.z - xc.z);
      double cn = cns1, ci = cin1;
      if (!NT1) {
        const int it = s_rty[r];
        cn = s_cns[it * nt1 + tc];
        if (INNER) ci = s_cin[it * nt1 + tc];
      }
      const unsigned long long m = __builtin_amdgcn_ballot_w64(rsq <= cn);
      my_lo = writelane<r>(my_lo, (unsigned)m);
      my_hi = writelane<r>(my_hi, (unsigned)(m >> 32));
      if (INNER) {
        const unsigned long long mi = __builtin_amdgcn_ballot_w64(rsq < ci);
        mi_lo = writelane<r>(mi_lo, (unsigned)mi);
        mi_hi = writelane<r>(mi_hi, (unsigned)(mi >> 32));
      }
    });
    // (rows past the last one sit at 1e300: their words are 0 already)
    const int self = s_self[wv][lane];
    const unsigned long long sbit = (unsigned long long)(self >= 0) << (self & 63);
    unsigned long long keep = ~sbit;
    if (N3) {  // lane r also drops the rows before it: prefix OR of the rows' own bits
      unsigned long long lo = sbit;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned a = (unsigned)__shfl_up((int)(unsigned)lo, d, 64);
        const unsigned h = (unsigned)__shfl_up((int)(unsigned)(lo >> 32), d, 64);
        if (lane >= d) lo |= ((unsigned long long)h << 32) | a;
      }
      keep = ~lo;
    }
    const unsigned long long full = (((unsigned long long)my_hi << 32) | my_lo) & ~sbit;
    const unsigned long long mine = full & keep;
    const unsigned long long minei = (((unsigned long long)mi_hi << 32) | mi_lo) & keep;
    if (N3 && lane < R) fc += __popcll(full);
    if (lane < R) {
      if (INNER)
        reinterpret_cast<ulonglong2 *>(s_w)[c * R + lane] = make_ulonglong2(mine, minei);
      else
        s_w[c * R + lane] = mine;
    }
    unsigned long long u = mine;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) u |= __shfl_xor(u, d, 64);
    if (INNER && iu) {
      unsigned long long ui = minei;
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) ui |= __shfl_xor(ui, d, 64);
      if (lane == 0) s_usedi[c] = ui;
    }
    if (N3) {  // the rows have fixed slots: the union proper is the other used candidates
      const unsigned long long rm = __ballot(cid >= row0 && cid < row0 + nrow);
      u &= ~rm;
      if (lane == 0) s_rowm[c] = rm;
    }
    if (lane == 0) s_used[c] = u;
  }
  if (N3 && lane < R) atomicAdd(&s_fc[lane], fc);
  __syncthreads();
  // 4) the union: used candidates in candidate order (slot = rank + 1); N3: the block's rows
  // first (slot r + 1), then the other used candidates
  int u = 0;
  {
    const int v = tid < nch ? __popcll(s_used[tid]) : 0;
    const int ex = blk_scan<NT>(v, s_sc, &u);
    if (tid < nch) s_upre[tid] = ex;
  }
  const int ubase = N3 ? nrow : 0;
  u += ubase;
  if (N3 && tid < nrow) ulist[(size_t)b * ucap + tid] = row0 + tid;
  int ui_tot = 0;  // iu: the inner union, numbered in candidate order like the full one
  if (iu) {
    const int v = tid < nch ? __popcll(s_usedi[tid]) : 0;
    const int ex = blk_scan<NT>(v, s_sc, &ui_tot);
    if (tid < nch) s_upi[tid] = ex;
  }
  __syncthreads();
  // the union list, and each chunk's slot words: candidate l of chunk c, if used, has slot
  // ubase + s_upre[c] + 1 + (used candidates below it); a row (N3) has slot r + 1
  for (int c = wv; c < nch; c += NW) {
    const unsigned long long used = s_used[c];
    const int below = blk_mbcnt(used);
    int sl = ubase + s_upre[c] + 1 + below;
    if (N3 && ((s_rowm[c] >> lane) & 1ull)) sl = s_cpos[c * 64 + lane] - row0 + 1;
    s_q[c][lane] = (unsigned short)blk_q(sl, cq);
    if ((used >> lane) & 1ull)
      ulist[(size_t)b * ucap + ubase + s_upre[c] + below] = s_cpos[c * 64 + lane];
    if (iu) {
      const unsigned long long usedi = s_usedi[c];
      if ((usedi >> lane) & 1ull)
        uilist[(size_t)b * ucap + s_upi[c] + blk_mbcnt(usedi)] = s_cpos[c * 64 + lane];
    }
  }
  if (tid == 0) {  // (the statistics words: k_blk_stats over these, not one atomic each --
                   // 15k workgroups' atomics on one line serialise)
    ucnt[b] = u;
    kcnt[b] = K;
    if (iu) uicnt[b] = ui_tot;
  }
  __syncthreads();
  // iu: the inner slots' words, over the candidates' atom ids (spent: the lists are written)
  unsigned short(*const s_qi)[64] = reinterpret_cast<unsigned short(*)[64]>(s_cpos);
  static_assert(sizeof(s_cpos) >= sizeof(unsigned short) * SCH * 64, "s_qi fits s_cpos");
  if (iu) {
    for (int c = wv; c < nch; c += NW)
      s_qi[c][lane] = (unsigned short)blk_q(s_upi[c] + 1 + blk_mbcnt(s_usedi[c]), cq);
    __syncthreads();
  }
  if (BEXP == 3) return;
  // 5) the slot rows, full and inner: wave w writes rows w*RPW .. w*RPW + RPW-1 with LPR
  // lanes per row; lane `part` of a row writes the row's chunks part, part + LPR, .. (U*G
  // entries each, transposed as blk_tpos: entry q*G + l of the chunk into lane word l at
  // bit 16q), walking the row's set bits from the chunk's first entry (ascending slots), and
  // stores each chunk whole (the tail chunk zero-padded: the sentinel slot).
  constexpr int LPR = 64 / RPW;
  static_assert(U * 16 <= 64, "a lane word of U 16-bit slots in 64 bits");
  const int r = wv * RPW + lane / LPR, part = lane % LPR;
  const bool live = r < nrow;
  auto word0 = [&](int c, int sel) -> unsigned long long {
    return INNER ? s_w[(c * R + r) * 2 + sel] : s_w[c * R + r];
  };
  // N3: a row's entries that are rows of the block come first (virtual words 0 .. nch-1),
  // then the others (nch .. 2 nch-1), each part in candidate order -- the pair passes meet a
  // row's Newton-3 pairs in its first walk steps only
  const int nv = N3 ? 2 * nch : nch;
  auto word = [&](int v, int sel) -> unsigned long long {
    if (!N3) return word0(v, sel);
    const int c = v < nch ? v : v - nch;
    const unsigned long long m = s_rowm[c];
    return word0(c, sel) & (v < nch ? m : ~m);
  };
  // the slot words of candidate `bit` of (virtual) word v in table qt: s_q, or s_qi for
  // the inner rows over their own union
  auto qof = [&](const unsigned short (*qt)[64], int v, int bit) -> unsigned short {
    return qt[(N3 && v >= nch) ? v - nch : v][bit];
  };
  bool over = false;
  auto emit = [&](int sel, unsigned short *__restrict__ rows, int *__restrict__ cnt_out) {
    int cnt = 0;
    if (live)
      for (int c = 0; c < nch; c++) cnt += __popcll(word0(c, sel));
    const int nchunk = min((cnt + UG - 1) / UG, sstride / UG);
    unsigned short *const out = rows + (size_t)(row0 + r) * sstride;
    const unsigned short(*const qt)[64] = (iu && sel == 1) ? s_qi : s_q;
    int c = 0, acc = 0;  // (virtual) word c holds the entries from acc on
    unsigned long long w = (live && nv > 0) ? word(0, sel) : 0ull;
    for (int ch = part; ch < nchunk; ch += LPR) {
      const int e0 = ch * UG;
      while (acc + __popcll(w) <= e0) {  // (e0 < cnt: the word holding it exists)
        acc += __popcll(w);
        w = word(++c, sel);
      }
      unsigned long long m = w;
      for (int j = e0 - acc; j > 0; j--) m &= m - 1ull;
      int cc = c;
      const int ne = min(cnt - e0, UG);
      unsigned long long buf[G];
#pragma unroll
      for (int l = 0; l < G; l++) buf[l] = 0ull;
#pragma unroll
      for (int q = 0; q < U; q++)
#pragma unroll
        for (int l = 0; l < G; l++)
          if (q * G + l < ne) {
            while (m == 0ull) m = word(++cc, sel);
            const int bit = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            buf[l] |= (unsigned long long)qof(qt, cc, bit) << (16 * q);
          }
      if (U == 4) {
        ulonglong2 *const o = reinterpret_cast<ulonglong2 *>(out + e0);
#pragma unroll
        for (int t = 0; t < G / 2; t++) o[t] = make_ulonglong2(buf[2 * t], buf[2 * t + 1]);
      } else {
#pragma unroll
        for (int l = 0; l < G; l++)
#pragma unroll
          for (int q = 0; q < U; q++) out[e0 + l * U + q] = (unsigned short)(buf[l] >> (16 * q));
      }
    }
    if (live && part == 0) {
      cnt_out[row0 + r] = cnt;
      over |= cnt > sstride;
      if (sel == WS - 1) s_len[r] = cnt;
    }
  };
  if (N3 && live && part == 0) fcnt[row0 + r] = s_fc[r];
  if (bperm && tid < R) s_len[tid] = -1;
  __syncthreads();
  emit(0, snbr, rcnt);
  if (INNER) emit(1, snbi, icnt);
  if (over) atomicMax(ovf, 1 << 21);
  if (bperm) {
    // the pair passes' row order inside the block: longest walked row (inner if built) first,
    // so that a wave's rows -- walked to the longest of them -- have similar lengths
    __syncthreads();
    if (tid < R) {
      const int my = s_len[tid];
      int rank = 0;
      for (int k = 0; k < R; k++) {
        const int o = s_len[k];
        rank += (o > my || (o == my && k < tid)) ? 1 : 0;
      }
      bperm[row0 + rank] = (unsigned char)tid;
    }
  }
}

// the block's lr-th walked row: the build's length order (bperm, k_blk_build) or in place
__device__ __forceinline__ int blk_row(const unsigned char *bperm, int base, int lr) {
  return bperm ? (int)bperm[base + lr] : lr;
}

// A lane's slot words: U = 2 slots in one 4-byte word, U = 4 in one 8-byte pair.
template <int U>
struct SlotWord;
template <>
struct SlotWord<2> {
  typedef unsigned T;
  __device__ static int get(const T &w, int q) { return (int)((w >> (16 * q)) & 0xffffu); }
};
template <>
struct SlotWord<4> {
  typedef v2u T;
  __device__ static int get(const T &w, int q) {
    return (int)(((q < 2 ? w.x : w.y) >> (16 * (q & 1))) & 0xffffu);
  }
};

// A row's c slots for the row's G lanes, chunk-transposed (blk_tpos): walk step (k, q) gives
// lane l the row's entry k*U*G + q*G + l.  load() issues the lane's slot-word loads -- before
// the block's staging, so their latency overlaps it; walk() calls body(slot, in) for the
// lane's slot positions (in = entry < c; padded positions hold the sentinel slot 0) and skips
// a step once every row of the wave has passed its count (steps of G entries, not U*G).
// NCH > 0: all of the row's chunks (at most NCH, the host guarantees c <= NCH*U*G) are held
// in registers; NCH = 0 (long rows): the next chunk is prefetched while the current one is
// evaluated (the slot array is padded by two chunks).
template <int G, int U, int NCH>
struct BlkSlots {
  typedef typename SlotWord<U>::T SW;
  SW w[NCH > 0 ? NCH : 1];
  const unsigned short *sl;
  __device__ __forceinline__ void load(const unsigned short *row, int c, int lane) {
    sl = row;
    if (NCH > 0) {
#pragma unroll
      for (int k = 0; k < NCH; k++)
        w[k] = k * U * G < c ? *reinterpret_cast<const SW *>(sl + k * U * G + U * lane) : SW{};
    } else {
      w[0] = *reinterpret_cast<const SW *>(sl + U * lane);
    }
  }
  template <class Body>
  __device__ __forceinline__ void walk(int c, int lane, Body body) {
    if (NCH > 0) {
#pragma unroll
      for (int k = 0; k < NCH; k++) {
        if (k * U * G >= c) break;
#pragma unroll
        for (int q = 0; q < U; q++)
          if (k * U * G + q * G < c) body(SlotWord<U>::get(w[k], q), k * U * G + q * G + lane < c);
      }
    } else {
      SW wn = w[0];
      for (int k0 = 0; k0 < c; k0 += U * G) {
        const SW cur = wn;
        wn = *reinterpret_cast<const SW *>(sl + k0 + U * G + U * lane);
#pragma unroll
        for (int q = 0; q < U; q++)
          if (k0 + q * G < c) body(SlotWord<U>::get(cur, q), k0 + q * G + lane < c);
      }
    }
  }
};
// walk2: the same slots, but each record is read by load(slot) and used by body(record); with
// SPH_BLK_PIPE a lane's records of a chunk are all read before the first is used (U
// independent pair evaluations in flight, the LDS latency covered by the next pairs' reads)
#ifndef SPH_BLK_PIPE
#define SPH_BLK_PIPE 1
#endif
template <int G, int U, int NCH, class Load, class Body>
__device__ __forceinline__ void blk_walk2(BlkSlots<G, U, NCH> &sw, int c, int lane, Load load,
                                          Body body) {
  if (NCH > 0 && SPH_BLK_PIPE) {
#pragma unroll
    for (int k = 0; k < (NCH > 0 ? NCH : 1); k++) {
      if (k * U * G >= c) break;
      decltype(load(0)) r[U];
#pragma unroll
      for (int q = 0; q < U; q++)
        if (k * U * G + q * G < c) r[q] = load(SlotWord<U>::get(sw.w[k], q));
#pragma unroll
      for (int q = 0; q < U; q++)
        if (k * U * G + q * G < c) body(r[q]);
    }
  } else {
    sw.walk(c, lane, [&](int q, bool) { body(load(q)); });
  }
}
// walk3 (SPH_BLK_WALK = 1, NCH > 0): the same slots as one flat sequence of steps (step s:
// chunk s / U, position s % U), walked to the WAVE's longest row with scalar branches -- a
// shorter row's extra steps read its padding (the sentinel slot, whose terms are exactly 0),
// which costs nothing: a masked lane's issue slot is spent anyway -- and software-pipelined:
// the records of steps s + 1 and s + 2 are read from LDS before step s is evaluated, so each
// record's LDS latency is covered by two pair evaluations of the same wave (the LDS image
// caps the pass at 4 waves per SIMD, which leaves the VGPRs for that).
#ifndef SPH_BLK_WALK
#define SPH_BLK_WALK 1
#endif
#ifndef SPH_BLK_ILP
#define SPH_BLK_ILP 1  // (pair evaluations per scheduling group; 2: 0.288 vs 0.282 ms, 3: 0.375)
#endif
template <class F, int... I>
__device__ __forceinline__ void blk_steps_(F &&f, std::integer_sequence<int, I...>) {
  (void)(f(std::integral_constant<int, I>{}) && ...);
}
// Lane map of the pair passes (SPH_BLK_LMAP, G = 8): a ds_read_b128 serves a wave in four
// 16-lane groups, {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32; each group holds
// two whole rows instead of halves of four, so the 16 records it reads are two runs of 8
// consecutive entries of two rows (consecutive union slots where a row's neighbours run
// along a bin row: distinct banks) -- rows r = 0..3 of a half at lanes {0-3,12-15},
// {20-27}, {4-11}, {16-19,28-31}.  A row's lanes are closed under xor 1, 2 and 12, so its
// sums stay butterflies.
#ifndef SPH_BLK_LMAP
#define SPH_BLK_LMAP 0
#endif
template <int G>
__device__ __forceinline__ int blk_lrow(int tid) {  // the workgroup-local row of thread tid
  if constexpr (G == 8 && SPH_BLK_LMAP) {
    const int p = tid & 31;
    const int r = p < 4 ? 0 : p < 12 ? 2 : p < 16 ? 0 : p < 20 ? 3 : p < 28 ? 1 : 3;
    return ((tid >> 5) << 2) + r;
  } else {
    return tid / G;
  }
}
template <int G>
__device__ __forceinline__ int blk_llane(int tid) {  // its lane in the row (entry order)
  if constexpr (G == 8 && SPH_BLK_LMAP) {
    const int p = tid & 31;
    return p < 4 ? p : p < 12 ? p - 4 : p < 16 ? p - 8 : p < 20 ? p - 16 : p < 28 ? p - 20 : p - 24;
  } else {
    return tid & (G - 1);
  }
}
template <int G>
__device__ __forceinline__ double blk_row_sum(double v) {
  if constexpr (G == 8 && SPH_BLK_LMAP) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    return v + __shfl_xor(v, 12, 64);
  } else {
    return group_sum<G>(v);
  }
}
template <int G>
__device__ __forceinline__ int wave_max_count(int c) {
#pragma unroll
  for (int d = (G == 8 && SPH_BLK_LMAP) ? 1 : G; d < 64; d <<= 1) c = max(c, __shfl_xor(c, d, 64));
  return __builtin_amdgcn_readfirstlane(c);
}
// AHEAD = 0: no records read ahead (each group reads its own, fewer VGPRs -- for a pass
// run at more waves per SIMD, whose other waves cover the LDS latency instead)
template <int AHEAD = 1, int G, int U, int NCH, class Load, class Body>
__device__ __forceinline__ void blk_walk3(BlkSlots<G, U, NCH> &sw, int cmax, Load load,
                                          Body body) {
  static_assert(NCH > 0, "walk3: rows held in registers");
  constexpr int NS = NCH * U;
  if (cmax <= 0) return;
  typedef decltype(load(0)) Rec;
  if constexpr (AHEAD == 0) {
    constexpr int IL = SPH_BLK_ILP, NG = (NS + IL - 1) / IL;
    auto group0 = [&](auto gc) -> bool {
      constexpr int g = decltype(gc)::value;
      if (g * IL * G >= cmax) return false;  // (wave-uniform)
      Rec r[IL];
      blk_steps_([&](auto sc) -> bool {
        constexpr int s = g * IL + decltype(sc)::value;
        if constexpr (s < NS) r[decltype(sc)::value] = load(SlotWord<U>::get(sw.w[s / U], s % U));
        return true;
      }, std::make_integer_sequence<int, IL>{});
      blk_steps_([&](auto sc) -> bool {
        constexpr int s = g * IL + decltype(sc)::value;
        if constexpr (s < NS) body(r[decltype(sc)::value]);
        return true;
      }, std::make_integer_sequence<int, IL>{});
      return true;
    };
    blk_steps_(group0, std::make_integer_sequence<int, NG>{});
    return;
  }
  // ILP steps form a group: the group's pair evaluations share one basic block (the scheduler
  // interleaves their dependency chains); the records of the next group are read before it.
  // A group runs whole once its first step is inside the wave's longest row (its later
  // steps may read only padding: exactly-zero terms).  The reads ahead are unconditional:
  // past a row's count its slot words hold the sentinel slot 0, a valid record.
  constexpr int IL = SPH_BLK_ILP, NG = (NS + IL - 1) / IL;
  Rec r[2 * IL];
  blk_steps_([&](auto sc) -> bool {
    constexpr int s = decltype(sc)::value;
    if constexpr (s < NS) r[s] = load(SlotWord<U>::get(sw.w[s / U], s % U));
    return true;
  }, std::make_integer_sequence<int, IL>{});
  // groups unrolled at compile time (the slot words stay in registers), left at the first
  // group past the wave's longest row
  auto group = [&](auto gc) -> bool {
    constexpr int g = decltype(gc)::value;
    if (g * IL * G >= cmax) return false;  // (wave-uniform)
    blk_steps_([&](auto sc) -> bool {
      constexpr int s = (g + 1) * IL + decltype(sc)::value;
      if constexpr (s < NS) r[s % (2 * IL)] = load(SlotWord<U>::get(sw.w[s / U], s % U));
      return true;
    }, std::make_integer_sequence<int, IL>{});
    // (keeps the reads ahead of the evaluations: the scheduler would sink them to their
    // use, tuning for an occupancy the LDS image does not allow)
    __builtin_amdgcn_sched_barrier(0);
    blk_steps_([&](auto sc) -> bool {
      constexpr int s = g * IL + decltype(sc)::value;
      if constexpr (s < NS) body(r[s % (2 * IL)]);
      return true;
    }, std::make_integer_sequence<int, IL>{});
    return true;
  };
  blk_steps_(group, std::make_integer_sequence<int, NG>{});
}

// a neighbour's record in the force pass's image (blk_put layout)
struct BlkRec {
  double2 a0, a1, a2, a3;
  double e;
  int q;
};

// union positions staged from registers loaded ahead of the slot rows (the rest, for
// unions over BLK_SP*threads atoms, in a plain loop)
constexpr int BLK_SP = 2;

// sph/rhosum over the block union (+ the Tait EOS epilogue: P/rho^2 into xf[i].w, rho into
// vr[i].w), pair_sph_rhosum.cpp:116-195.  The cut test rides on the kernel weight:
// max(1 - rsq/h^2, 0) is zero exactly where rsq >= cutsq = h^2 fails, up to the last bit of
// rsq/h^2 at rsq = h^2 (a weight ~1e-64 then); one type: sum_j w_j, times m_j K at the end.
template <int R, int G, int U, int NCH, bool NT1, int CQ>
__global__ void __launch_bounds__(R * G)
k_blk_rhosum(int n, const int *__restrict__ ulist, const int *__restrict__ ucnt, int ucap,
             const unsigned short *__restrict__ snbr, int sstride,
             const int *__restrict__ rcnt, double4 *__restrict__ xf,
             const int *__restrict__ ty, double4 *__restrict__ vr,
             const Coefs *__restrict__ cf, int um, const unsigned short *__restrict__ snbi,
             const int *__restrict__ icnt, const int *__restrict__ moved, int n3,
             const unsigned char *__restrict__ bperm, const int *__restrict__ uilist,
             const int *__restrict__ uicnt, const int *__restrict__ blist) {
  constexpr int NTH = R * G;
  if (snbi && *moved == 0) {  // (workgroup-uniform) the inner rows are still exact
    snbr = snbi;
    rcnt = icnt;
    ulist = uilist;  // (over their own union)
    ucnt = uicnt;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char blk_smem[];
  __shared__ RhoPair s_c[NT1 ? 1 : NT2];
  __shared__ double s_acc[R];  // n3: the later rows' shares (k_blk_build N3)
  const int nt1 = cf->ntypes + 1;
  // (blist: a subset of the blocks -- the interior or the boundary ones, overlap_on)
  const int b = blist ? blist[xcd_block()] : (int)xcd_block(), tid = threadIdx.x;
  // (bperm: the block's rows in the build's length order, blk_row)
  const int row = b * R + blk_row(bperm, b * R, blk_lrow<G>(tid)), lane = blk_llane<G>(tid);
  const bool live = row < n;
  const int rr = live ? row : n - 1;
  // n3: slots 1 .. nrow are the block's rows (q <= qn3); a row's entries among them are the
  // later rows, whose share (m_i W_ij) goes to their accumulator
  const bool n3on = BLK_N3_BUILT && n3;
  const int qn3 = n3on ? blk_q(min(R, n - b * R), CQ) : -1;
  if (n3on && tid < R) s_acc[tid] = 0.0;
  // loads first: the row's count, the union's atom ids, then the row's slots and the
  // union's positions, so that one latency covers them all
  const int u = ucnt[b];
  const int c = live ? rcnt[rr] : 0;
  const int *const ul = ulist + (size_t)b * ucap;
  int jj[BLK_SP];
#pragma unroll
  for (int k = 0; k < BLK_SP; k++) jj[k] = tid + k * NTH < u ? ul[tid + k * NTH] : -1;
  BlkSlots<G, U, NCH> sw;
  sw.load(snbr + (size_t)rr * sstride, c, lane);
  const double4 xi = xf[rr];
  const int it = NT1 ? 1 : ty[rr];
  double4 gx[BLK_SP];
  int gt[BLK_SP];
#pragma unroll
  for (int k = 0; k < BLK_SP; k++)
    if (jj[k] >= 0) {
      gx[k] = xf[jj[k]];
      if (!NT1) gt[k] = ty[jj[k]];
    }
  double2 *const s_xy = reinterpret_cast<double2 *>(blk_smem);
  double *const s_z = reinterpret_cast<double *>(blk_smem + (size_t)(um + 1) * 16);
  unsigned char *const s_t = blk_smem + (size_t)(um + 1) * 24;
  if (!NT1)
    for (int t = tid; t < nt1 * nt1; t += NTH) s_c[t] = cf->rho[t];
#pragma unroll
  for (int k = 0; k < BLK_SP; k++)
    if (jj[k] >= 0) {
      const int sl = tid + k * NTH + 1;
      s_xy[sl] = make_double2(gx[k].x, gx[k].y);
      s_z[sl] = gx[k].z;
      if (!NT1) s_t[sl] = (unsigned char)gt[k];
    }
  for (int p = tid + BLK_SP * NTH; p < u; p += NTH) {
    const int j = ul[p];
    const double4 x = xf[j];
    s_xy[p + 1] = make_double2(x.x, x.y);
    s_z[p + 1] = x.z;
    if (!NT1) s_t[p + 1] = (unsigned char)ty[j];
  }
  if (tid == 0) {
    s_xy[0] = make_double2(1e100, 1e100);
    s_z[0] = 1e100;
    if (!NT1) s_t[0] = 1;
  }
  __syncthreads();
  const RhoPair c1 = NT1 ? cf->rho[3] : RhoPair{};
  double acc = 0.0;
  struct RhoRec {
    double2 xy;
    double z;
    int q;
  };
  auto load = [&](int q) {
    const int sj = blk_s<CQ>(q);
    return RhoRec{s_xy[sj], s_z[sj], q};
  };
  auto pair = [&](const RhoRec &rc) {
    const int q = rc.q, sj = blk_s<CQ>(q);
    const double2 xy = rc.xy;
    const double dx = xi.x - xy.x, dy = xi.y - xy.y, dz = xi.z - rc.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    const RhoPair cc = NT1 ? c1 : s_c[it * nt1 + s_t[sj]];
    double wf = fmax(fma(-rsq, cc.ihsq, 1.0), 0.0);
    wf = wf * wf;
    wf = wf * wf;
    acc = NT1 ? acc + wf : fma(cc.mK, wf, acc);
    if (q > 0 && q <= qn3)  // a later row of this block: its share (cut and weight symmetric)
      atomicAdd(&s_acc[sj - 1], NT1 ? wf : s_c[s_t[sj] * nt1 + it].mK * wf);
  };
  if constexpr (NCH > 0 && SPH_BLK_WALK == 1) {
    if (!n3on)
      blk_walk3(sw, wave_max_count<G>(c), load, pair);
    else
      sw.walk(c, lane, [&](int q, bool) { pair(load(q)); });
  } else {
    sw.walk(c, lane, [&](int q, bool) { pair(load(q)); });
  }
  acc = blk_row_sum<G>(acc);
  if (n3on) {  // (workgroup-uniform) the earlier rows' shares of this row
    __syncthreads();
    acc += s_acc[blk_lrow<G>(tid)];
  }
  if (lane == 0 && live) {
    const double rho = ((cf->rho_keep >> it) & 1) ? vr[row].w
                                                   : cf->self_rho[it] + (NT1 ? c1.mK * acc : acc);
    vr[row].w = rho;
    xf[row].w = tait_p_over_rho2(rho, cf->rho0[it], cf->B[it]);
  }
}

// INNER rows for the pair passes: the entries of each full row (cutneighsq = (cut + skin)^2)
// whose pair is within cut + m now, m = a sixteenth of the skin, over the block's INNER UNION
// (the atoms some inner row names, renumbered in full-union order).  While no atom has moved
// m/2 since (k_initial_integrate / k_final_initial raise *moved otherwise) every pair inside
// a pair style's cut is among them, so the passes walk ~115 instead of ~155 entries per row
// at C2 with identical terms (a dropped entry's kernel weight is exactly zero) and stage
// ~15 % fewer union records; once an atom has moved further the passes fall back to the full
// rows and union until the next rebuild.  Each row keeps its full-row order (rank by ballot
// within the row's G lanes); tails are padded with the sentinel like the full rows.
// Written by k_blk_build's second ballot at a rebuild; here when the bitmap build took the
// rebuild (k_blk_neigh, no inner ballot), and for a refresh (cond != nullptr; one workgroup
// per several blocks, grid-stride): only if *cond is set -- an atom moved more than half the
// margin since the rows were written -- the rows and inner unions are derived again from the
// full rows at the current positions and x0 (the owned rows' reference positions) takes
// them; *zero (the next step's flag) is cleared either way.  The pair passes then walk inner
// rows again instead of the full rows for the rest of the build.
// Two walks per block: the hits mark a bitmap over the full union's slots; its prefix
// numbers the inner union; the second walk writes the rows in that numbering.
template <int R, int G, int U, int NCH, bool NT1, int CQ>
__global__ void __launch_bounds__(R * G)
k_blk_inner(int n, const int *__restrict__ ulist, const int *__restrict__ ucnt, int ucap,
            const unsigned short *__restrict__ snbr, int sstride, const int *__restrict__ rcnt,
            const double4 *__restrict__ xf, const int *__restrict__ ty,
            const Coefs *__restrict__ cf, unsigned short *__restrict__ snbi,
            int *__restrict__ icnt, int um, const int *__restrict__ cond,
            int *__restrict__ zero, double4 *__restrict__ x0, int *__restrict__ uilist,
            int *__restrict__ uicnt, int *__restrict__ umax) {
  constexpr int NTH = R * G;
  constexpr int NWD = (BLK_UCAP + 1 + 31) / 32;       // bitmap words over slots 0 .. BLK_UCAP
  constexpr int WPT = (NWD + NTH - 1) / NTH;          // consecutive words per thread (scan)
  if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;
  if (cond && *cond == 0) return;  // (workgroup-uniform)
  extern __shared__ __attribute__((aligned(16))) unsigned char blk_smem[];
  __shared__ double s_c[NT1 ? 1 : NT2];
  __shared__ unsigned s_bm[NWD];
  __shared__ int s_pre[NWD];
  __shared__ int s_w[NTH / 64];
  const int tid = threadIdx.x;
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = tid; t < nt1 * nt1; t += NTH) s_c[t] = cf->cutinsq[t];
  const int nb = (n + R - 1) / R;
  for (int b = cond ? (int)blockIdx.x : (int)xcd_block(); b < nb; b += cond ? gridDim.x : nb) {
    const int row = b * R + tid / G, lane = tid & (G - 1);
    const bool live = row < n;
    const int rr = live ? row : n - 1;
    const int u = ucnt[b];
    const int c = live ? rcnt[rr] : 0;
    const int *const ul = ulist + (size_t)b * ucap;
    BlkSlots<G, U, NCH> sw;
    sw.load(snbr + (size_t)rr * sstride, c, lane);
    const double4 xi = xf[rr];
    const int it = NT1 ? 1 : ty[rr];
    double2 *const s_xy = reinterpret_cast<double2 *>(blk_smem);
    double *const s_z = reinterpret_cast<double *>(blk_smem + (size_t)(um + 1) * 16);
    unsigned char *const s_t = blk_smem + (size_t)(um + 1) * 24;
    const int nw = (u + 1 + 31) >> 5;
    __syncthreads();  // (the previous block's image and bitmap are no longer read)
    for (int p = tid; p < u; p += NTH) {
      const int j = ul[p];
      const double4 x = xf[j];
      s_xy[p + 1] = make_double2(x.x, x.y);
      s_z[p + 1] = x.z;
      if (!NT1) s_t[p + 1] = (unsigned char)ty[j];
    }
    for (int w = tid; w < nw; w += NTH) s_bm[w] = 0u;
    if (tid == 0) {
      s_xy[0] = make_double2(1e100, 1e100);
      s_z[0] = 1e100;
      if (!NT1) s_t[0] = 1;
    }
    __syncthreads();
    const double c1 = NT1 ? cf->cutinsq[3] : 0.0;
    auto hit_of = [&](int q, bool in) {
      const int sj = blk_s<CQ>(q);
      const double2 xy = s_xy[sj];
      const double dx = xi.x - xy.x, dy = xi.y - xy.y, dz = xi.z - s_z[sj];
      const double rsq = dx * dx + dy * dy + dz * dz;
      return in && live && rsq < (NT1 ? c1 : s_c[it * nt1 + s_t[sj]]);
    };
    // 1) the inner union: the full-union slots some inner pair names (uilist == nullptr:
    // none, the rows keep the full union's numbering)
    const bool ren = uilist != nullptr;
    if (ren) sw.walk(c, lane, [&](int q, bool in) {
      if (hit_of(q, in)) {
        const int sj = blk_s<CQ>(q);
        atomicOr(&s_bm[sj >> 5], 1u << (sj & 31));
      }
    });
    __syncthreads();
    int tot = 0;
    if (ren) {
      int v = 0;
#pragma unroll
      for (int k = 0; k < WPT; k++) {
        const int w = tid * WPT + k;
        v += w < nw ? __popc(s_bm[w]) : 0;
      }
      int ex = blk_scan<NTH>(v, s_w, &tot);
#pragma unroll
      for (int k = 0; k < WPT; k++) {
        const int w = tid * WPT + k;
        if (w < nw) {
          s_pre[w] = ex;
          ex += __popc(s_bm[w]);
        }
      }
    }
    __syncthreads();
    auto rank = [&](int sj) {  // 0-based position of slot sj in the inner union
      const unsigned w = s_bm[sj >> 5];
      return s_pre[sj >> 5] + __popc(w & ((1u << (sj & 31)) - 1u));
    };
    if (ren)
      for (int p = tid; p < u; p += NTH)
        if ((s_bm[(p + 1) >> 5] >> ((p + 1) & 31)) & 1u)
          uilist[(size_t)b * ucap + rank(p + 1)] = ul[p];
    if (ren && tid == 0) {
      uicnt[b] = tot;
      if (umax) {
        atomicMax(umax, tot);
        atomicAdd(umax + 1, tot);
      }
    }
    // 2) the rows in the inner numbering
    const int grp = (tid & 63) / G;                   // the row's lane group in the wave
    unsigned short *const out = snbi + (size_t)rr * sstride;
    int base = 0;
    sw.walk(c, lane, [&](int q, bool in) {
      const bool hit = hit_of(q, in);
      const unsigned long long m = __ballot(hit);
      const unsigned g = (unsigned)(m >> (grp * G)) & ((1u << G) - 1u);
      if (hit)
        out[blk_tpos<G, U>(base + __popc(g & ((1u << lane) - 1u)))] =
            (unsigned short)(ren ? blk_q(rank(blk_s<CQ>(q)) + 1, CQ) : q);
      base += __popc(g);
    });
    if (live) {
      if (lane == 0) {
        icnt[row] = base;
        if (x0) x0[row] = xi;
      }
      const int cend = min((base + U * G - 1) / (U * G) * (U * G), sstride);
      for (int k = base + lane; k < cend; k += G) out[blk_tpos<G, U>(k)] = 0;  // the sentinel
    }
  }
}

// sph/taitwater[/morris] [+ sph/heatconduction] over the block union (full list, i side
// only), pair_sph_taitwater.cpp:139-191, pair_sph_taitwater_morris.cpp:139-191,
// pair_sph_heatconduction.cpp:103-124.  blist == nullptr: every block whose union fits the
// um-atom LDS image (larger ones return at once); else the blocks listed in blist (the
// second launch, with an image as large as the largest union).
// The styles' cut is their h (cutsq = h^2), so the cut test rides on the weight:
// d = max(h - r, 0) is zero exactly where rsq < cutsq fails (up to the last bit of r at
// r = h, a weight ~1e-32 then).  The pair's uniform factors (-m_i m_j wK, m_j wK, -1/2,
// the heat prefactor) are applied once per row when there is one type, per pair otherwise.
// EXP (study builds, SPH_EXP): 1 = neighbour records synthesised from the slot (no LDS
// reads), 2 = LDS reads with a trivial body, 3 = no staging loads (LDS image left as is).
// Outputs meaningless.
// Occupancy the pair passes really get: the LDS image (~64 KiB at C2) admits two 512-thread
// workgroups per CU, i.e. 4 waves per SIMD -- told to the compiler so that it schedules for
// that (loads further ahead, up to 128 VGPRs) instead of for the 6-8 waves VGPRs alone allow
#ifndef SPH_BLK_WPE
#define SPH_BLK_WPE 0
#endif
#if SPH_BLK_WPE > 0
#define SPH_BLK_OCC __attribute__((amdgpu_waves_per_eu(SPH_BLK_WPE, SPH_BLK_WPE)))
#else
#define SPH_BLK_OCC
#endif

#define SPH_BLK_FORCE_PARAMS                                                              \
  int n, const int *__restrict__ ulist, const int *__restrict__ ucnt, int ucap,                 \
      const unsigned short *__restrict__ snbr, int sstride, const int *__restrict__ rcnt,     \
      const double4 *__restrict__ xf, const double4 *__restrict__ vr,                         \
      const int *__restrict__ ty, const double *__restrict__ en,                              \
      const Coefs *__restrict__ cf, double4 *__restrict__ fo, double *__restrict__ de,        \
      double gx, double gy, double gz, int um, int cq,                                        \
      const unsigned short *__restrict__ snbi, const int *__restrict__ icnt,                  \
      const int *__restrict__ moved, int n3, const unsigned char *__restrict__ bperm,         \
      const int *__restrict__ uilist, const int *__restrict__ uicnt,                          \
      const int *__restrict__ blist
#define SPH_BLK_FORCE_ARGS                                                                \
  n, ulist, ucnt, ucap, snbr, sstride, rcnt, xf, vr, ty, en, cf, fo, de, gx, gy, gz, um, cq, \
      snbi, icnt, moved, n3, bperm, uilist, uicnt, blist
// (the body of the force pass; the kernels below differ only in their occupancy request)
template <int R, int G, int U, int NCH, int VISC, int MODE, bool NT1, int EXP = 0, int AHEAD = 1>
__device__ __forceinline__ void blk_force_body(SPH_BLK_FORCE_PARAMS) {
  if (snbi && *moved == 0) {  // (workgroup-uniform) the inner rows are still exact
    snbr = snbi;
    rcnt = icnt;
    ulist = uilist;  // (over their own union)
    ucnt = uicnt;
  }
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  constexpr int NTH = R * G;
  constexpr int CQ = (HEAT ? BLK_CHE : BLK_CH) / 16;  // (= cq)
  // one type, Monaghan viscosity, no heat term: the records carry rho_j / viscC (the row
  // rho_i / viscC), so fvisc = min(dvdr, 0) / ((rsq + eps)(rho_i + rho_j) / viscC) needs no
  // multiply by viscC per pair.  viscC = 0 never gets here: the host launches VISC =
  // BLK_VISC_NONE then (no viscosity term, as viscC * ... = 0 in the reference)
  constexpr bool FOLDV = TAIT && !HEAT && NT1 && VISC == SPH_VISC_MONAGHAN;
  constexpr int NA = HEAT ? 6 : 5;  // a row's shares: F (3), D, E [, EH]
  extern __shared__ __attribute__((aligned(16))) unsigned char blk_smem[];
  __shared__ TaitPair s_tp[(TAIT && !NT1) ? NT2 : 1];
  __shared__ HeatPair s_hp[(HEAT && !NT1) ? NT2 : 1];
  __shared__ double s_acc[BLK_N3_BUILT ? R * NA : 1];  // n3: the later rows' shares
  const int nt1 = cf->ntypes + 1;
  const int b = blist ? blist[xcd_block()] : (int)xcd_block();  // (blist: a subset of blocks)
  const int tid = threadIdx.x;
  const int u = EXP == 3 ? 0 : ucnt[b];
  // the LDS image holds um union records (a multiple of 16); a larger union is walked in
  // WINDOWS of um records: each window staged in turn, every row walked against it with the
  // entries outside it read as the sentinel (workgroup-uniform; the host sizes um so that
  // few blocks need it, and never with n3)
  const int nwin = u > um ? (u + um - 1) / um : 1;
  const int u0 = min(u, um);
  // n3: slots 1 .. nrow are the block's rows (q <= qn3); a row's entries among them are the
  // later rows, whose shares go to their accumulators (Newton's third law: F and the heat
  // term change sign, D and E do not)
  const bool n3on = BLK_N3_BUILT && n3;
  const int qn3 = n3on ? blk_q(min(R, n - b * R), CQ) : -1;
  if (n3on)
    for (int t = tid; t < R * NA; t += NTH) s_acc[t] = 0.0;
  const int row = b * R + blk_row(bperm, b * R, blk_lrow<G>(tid)), lane = blk_llane<G>(tid);
  const bool live = row < n;
  const int rr = live ? row : n - 1;
  // loads first: the row's count, the union's atom ids, then the row's slots and the
  // union's records, so that one latency covers them all
  const int c = live ? rcnt[rr] : 0;
  const int *const ul = ulist + (size_t)b * ucap;
  int jj[BLK_SP];
#pragma unroll
  for (int k = 0; k < BLK_SP; k++) jj[k] = tid + k * NTH < u0 ? ul[tid + k * NTH] : -1;
  BlkSlots<G, U, NCH> sw;
  sw.load(snbr + (size_t)rr * sstride, c, lane);
  const double4 xi = xf[rr];
  const double vsc = FOLDV ? 1.0 / cf->tait[3].viscC : 1.0;
  double4 vi = vr[rr];
  if (FOLDV) vi.w *= vsc;
  const double ei = HEAT ? en[rr] : 0.0;
  const int it = NT1 ? 1 : ty[rr];
  double4 qx[BLK_SP], qv[BLK_SP];
  double ge[BLK_SP];
  int gt[BLK_SP];
#pragma unroll
  for (int k = 0; k < BLK_SP; k++)
    if (jj[k] >= 0) {
      qx[k] = xf[jj[k]];
      qv[k] = vr[jj[k]];
      if (HEAT) ge[k] = en[jj[k]];
      if (!NT1) gt[k] = ty[jj[k]];
    }
  if (!NT1)
    for (int t = tid; t < nt1 * nt1; t += NTH) {
      if (TAIT) s_tp[t] = cf->tait[t];
      if (HEAT) s_hp[t] = cf->heat[t];
    }
  unsigned char *const s_t = blk_smem + (size_t)((u0 + 16) >> 4) * cq * 16;
#pragma unroll
  for (int k = 0; k < BLK_SP; k++)
    if (jj[k] >= 0) {
      const int sl = tid + k * NTH + 1;
      if (FOLDV) qv[k].w *= vsc;
      blk_put<HEAT>(blk_smem, sl, cq, qx[k], qv[k], HEAT ? ge[k] : 0.0);
      if (!NT1) s_t[blk_q(sl, cq)] = (unsigned char)gt[k];
    }
  // window w's union records [w um, min(u, (w + 1) um)) from p0 on into slots 1, 2, ..
  auto stage = [&](int w, int p0) {
    const int base = w * um, end = min(u, base + um);
    for (int p = base + p0; p < end; p += NTH) {
      const int j = ul[p];
      double4 v = vr[j];
      if (FOLDV) v.w *= vsc;
      blk_put<HEAT>(blk_smem, p - base + 1, cq, xf[j], v, HEAT ? en[j] : 0.0);
      if (!NT1) s_t[blk_q(p - base + 1, cq)] = (unsigned char)ty[j];
    }
  };
  stage(0, tid + BLK_SP * NTH);
  if (tid == 0) {
    blk_put_sentinel<HEAT>(blk_smem);
    if (!NT1) s_t[0] = 1;
  }
  __syncthreads();
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  // F: sum of (d x) sp (- vel sv); E: sum of sp dvdr (- sv vel^2); D: sum of dvdr w; EH:
  // the heat terms.  One type: sp = (P_i/rho_i^2 + P_j/rho_j^2 [+ fvisc]) w, the row's
  // factors applied at the end; several types: sp, sv, D and EH terms carry them per pair.
  double fx = 0.0, fy = 0.0, fz = 0.0, D = 0.0, E = 0.0, EH = 0.0;
  auto load = [&](int q) {
    const unsigned char *const rec = blk_smem + q * 16;
    BlkRec r;
    r.q = q;
    if (EXP == 1) {
      const double o = (double)(q & 7);
      r.a0 = make_double2(xi.x + 0.25 * o, xi.y + 0.5);
      r.a1 = make_double2(xi.z - 0.125 * o, xi.w);
      r.a2 = make_double2(vi.x, vi.y - 0.01 * o);
      r.a3 = make_double2(vi.z, vi.w);
    } else {
      r.a0 = *reinterpret_cast<const double2 *>(rec);
      r.a1 = *reinterpret_cast<const double2 *>(rec + 256);
      r.a2 = *reinterpret_cast<const double2 *>(rec + 512);
      r.a3 = *reinterpret_cast<const double2 *>(rec + 768);
    }
    r.e = HEAT ? *reinterpret_cast<const double *>(rec + 1024) : 0.0;
    return r;
  };
  auto pair = [&](const BlkRec &rc) {
    const int q = rc.q;
    const double2 a0 = rc.a0, a1 = rc.a1, a2 = rc.a2, a3 = rc.a3;
    if (EXP == 2) {
      fx += a0.x + a2.x;
      fy += a0.y + a2.y;
      fz += a1.x + a3.x;
      D += a1.y + a3.y;
      return;
    }
    const double dx = xi.x - a0.x, dy = xi.y - a0.y, dz = xi.z - a1.x;
    const double rsq = rsq_t(dx, dy, dz);  // (+ 1e-300)
    const int pidx = NT1 ? 3 : it * nt1 + s_t[q];
    const double r = sqrt1n(rsq);
    // this pair's terms (i side); a later row of the block takes its share too (n3)
    double tfx = 0.0, tfy = 0.0, tfz = 0.0, tD = 0.0, tDj = 0.0, tE = 0.0, tEH = 0.0;
    if (TAIT) {
      const TaitPair cc = NT1 ? t1 : s_tp[pidx];
      const double d = fmax(cc.h - r, 0.0);
      const double w = NT1 ? d * d : cc.wK * (d * d);
      const double velx = vi.x - a2.x, vely = vi.y - a2.y, velz = vi.z - a3.x;
      const double dvdr = dx * velx + dy * vely + dz * velz;
      if (VISC == SPH_VISC_MONAGHAN) {
        // fvisc = viscC dvdr / ((rsq + eps)(rho_i + rho_j)) for dvdr < 0, else 0
        const double fv = FOLDV ? fmin(dvdr, 0.0) * rcp1((rsq + cc.eps) * (vi.w + a3.y))
                                : (cc.viscC * fmin(dvdr, 0.0)) * rcp1((rsq + cc.eps) * (vi.w + a3.y));
        const double sp = NT1 ? (xi.w + a1.y + fv) * w : cc.mm * ((xi.w + a1.y + fv) * w);
        tfx = dx * sp;
        tfy = dy * sp;
        tfz = dz * sp;
        tE = sp * dvdr;
      } else if (VISC == BLK_VISC_NONE) {  // (one type, Monaghan with viscC = 0)
        const double sp = (xi.w + a1.y) * w;
        tfx = dx * sp;
        tfy = dy * sp;
        tfz = dz * sp;
        tE = sp * dvdr;
      } else {
        const double sp = NT1 ? (xi.w + a1.y) * w : cc.mm * ((xi.w + a1.y) * w);
        const double cv = cc.viscC * rcp1(vi.w * a3.y);
        const double sv = NT1 ? cv * w : cc.mm * (cv * w);
        tfx = dx * sp - velx * sv;
        tfy = dy * sp - vely * sv;
        tfz = dz * sp - velz * sv;
        tE = sp * dvdr - sv * (velx * velx + vely * vely + velz * velz);
      }
      tD = NT1 ? dvdr * w : cc.mj * (dvdr * w);
      tDj = NT1 ? tD : cc.mi * (dvdr * w);  // (the share of row j: m_i instead of m_j)
      fx += tfx;
      fy += tfy;
      fz += tfz;
      E += tE;
      D += tD;
    }
    if (HEAT) {
      const HeatPair cc = NT1 ? h1 : s_hp[pidx];
      const double d = fmax(cc.h - r, 0.0);
      const double w = NT1 ? d * d : cc.wK * (d * d);
      const double ej = rc.e;
      const double t = ((vi.w + a3.y) * rcp1(vi.w * a3.y)) * ((ei - ej) * w);
      tEH = NT1 ? t : cc.hmD * t;
      EH += tEH;
    }
    if (q > 0 && q <= qn3) {
      double *const a = s_acc + (blk_s<CQ>(q) - 1) * NA;
      if (TAIT) {
        atomicAdd(a + 0, -tfx);
        atomicAdd(a + 1, -tfy);
        atomicAdd(a + 2, -tfz);
        atomicAdd(a + 3, tDj);
        atomicAdd(a + 4, tE);
      }
      if (HEAT) atomicAdd(a + 5, -tEH);
    }
  };
  auto walk = [&](auto ld) {
    if constexpr (NCH > 0 && SPH_BLK_WALK == 1) {
      if (!n3on)
        blk_walk3<AHEAD>(sw, wave_max_count<G>(c), ld, pair);
      else
        blk_walk2(sw, c, lane, ld, pair);
    } else {
      blk_walk2(sw, c, lane, ld, pair);
    }
  };
  if (nwin == 1) {
    walk(load);
  } else {
    // window w holds slots (w um, (w + 1) um] at 1 .. um: q (monotone in the slot, um a
    // multiple of 16) shifts by qo = blk_q(w um); the others read the sentinel
    const int qmax = blk_q(um, CQ);
    for (int w = 0; w < nwin; w++) {
      if (w > 0) {
        __syncthreads();  // (the previous window is walked)
        stage(w, tid);
        __syncthreads();
      }
      const int qo = blk_q(w * um, CQ);
      walk([&](int q) {
        const int qq = q - qo;
        return load((unsigned)(qq - 1) < (unsigned)qmax ? qq : 0);
      });
    }
  }
  if (TAIT) {
    fx = blk_row_sum<G>(fx);
    fy = blk_row_sum<G>(fy);
    fz = blk_row_sum<G>(fz);
    D = blk_row_sum<G>(D);
    E = blk_row_sum<G>(E);
  }
  if (HEAT) EH = blk_row_sum<G>(EH);
  if (n3on) {  // (workgroup-uniform) the earlier rows' shares of this row
    __syncthreads();
    const double *const a = s_acc + blk_lrow<G>(tid) * NA;
    if (TAIT) {
      fx += a[0];
      fy += a[1];
      fz += a[2];
      D += a[3];
      E += a[4];
    }
    if (HEAT) EH += a[5];
  }
  if (lane == 0 && live) {
    double dE = 0.0;
    if (TAIT) {
      // one type: F, E scale by m_i m_j wK (mm = -m_i m_j), D by m_j wK
      const double g = NT1 ? t1.mm * t1.wK : 1.0;
      const double gd = NT1 ? t1.mj * t1.wK : 1.0;
      const double m = cf->mass[it];
      fo[row] = make_double4(g * fx + m * gx, g * fy + m * gy, g * fz + m * gz, gd * D);
      dE = -0.5 * (g * E);
    }
    if (HEAT) dE += NT1 ? (h1.hmD * h1.wK) * EH : EH;
    de[row] = dE;
  }
}

template <int R, int G, int U, int NCH, int VISC, int MODE, bool NT1, int EXP = 0>
__global__ void __launch_bounds__(R * G) SPH_BLK_OCC k_blk_force(SPH_BLK_FORCE_PARAMS) {
  blk_force_body<R, G, U, NCH, VISC, MODE, NT1, EXP>(SPH_BLK_FORCE_ARGS);
}
// one type, taitwater alone (C2): asked for 5 waves per SIMD (<= 96 VGPRs, no spill) -- the
// compiler otherwise settles at 98 VGPRs, 4 waves, while the LDS image admits 6
// (0.2550 vs 0.272-0.273 ms per launch on one box, profiles/r05/README.md); the heat and
// multi-type variants keep the default (at 96 VGPRs they would spill)
template <int R, int G, int U, int NCH, int VISC, int MODE, bool NT1, int EXP = 0>
__global__ void __launch_bounds__(R * G) __attribute__((amdgpu_waves_per_eu(5, 5)))
k_blk_force_w5(SPH_BLK_FORCE_PARAMS) {
  blk_force_body<R, G, U, NCH, VISC, MODE, NT1, EXP>(SPH_BLK_FORCE_ARGS);
}
// ... and at 6 waves per SIMD (<= 80 VGPRs: what the 49 KiB image allows, three workgroups
// per CU) with no records read ahead -- the other waves cover the LDS latency: 0.2435 /
// 0.2497 vs 0.2632 / 0.2627 ms per launch (two A/B pairs on one box, profiles/r05/README.md).
// Production for C2; SPH_BLK_W6=0 (study) keeps the 5-wave kernel with the read-ahead.
template <int R, int G, int U, int NCH, int VISC, int MODE, bool NT1, int EXP = 0>
__global__ void __launch_bounds__(R * G) __attribute__((amdgpu_waves_per_eu(6, 6)))
k_blk_force_w6(SPH_BLK_FORCE_PARAMS) {
  blk_force_body<R, G, U, NCH, VISC, MODE, NT1, EXP, 0>(SPH_BLK_FORCE_ARGS);
}
#ifndef SPH_BLK_W6
#define SPH_BLK_W6 1
#endif

// blocks of a build whose union exceeds the force pass's LDS image (um records): the pass
// walks them in windows of um union records (statistics only, sph_engine_stats blk_nbig)
static __global__ void k_blk_count_big(int nb, const int *__restrict__ ucnt, int um,
                                       int *__restrict__ nbig) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nb && ucnt[b] > um) atomicAdd(nbig, 1);
}

// k_blk_build's statistics words from its per-block counts (one workgroup of 1024):
// umax[0] largest union, [1] largest candidate set, [2] sum of candidates, [3] sum of
// unions, [6] largest inner union, [7] sum of inner unions (uicnt == nullptr: none)
static __global__ void __launch_bounds__(1024)
k_blk_stats(int nb, const int *__restrict__ ucnt, const int *__restrict__ kcnt,
            const int *__restrict__ uicnt, int *__restrict__ umax) {
  __shared__ int s_r[6][16];
  int v[6] = {0, 0, 0, 0, 0, 0};  // max u, max K, sum K, sum u, max ui, sum ui
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const int u = ucnt[b], k = kcnt[b], ui = uicnt ? uicnt[b] : 0;
    v[0] = max(v[0], u);
    v[1] = max(v[1], k);
    v[2] += k;
    v[3] += u;
    v[4] = max(v[4], ui);
    v[5] += ui;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1)
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const int o = __shfl_xor(v[q], d, 64);
      v[q] = (q == 0 || q == 1 || q == 4) ? max(v[q], o) : v[q] + o;
    }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int q = 0; q < 6; q++) s_r[q][w] = v[q];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int q = threadIdx.x;
    int r = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++)
      r = (q == 0 || q == 1 || q == 4) ? max(r, s_r[q][k]) : r + s_r[q][k];
    const int slot[6] = {0, 1, 2, 3, 6, 7};
    umax[slot[q]] = r;
  }
}

// ---- host-side launch helpers ----------------------------------------------------------
// Block shapes (rows per block R, lanes per row G, slots per lane and chunk U); SPH_BLK
// picks one (tuning).  R*G threads per pair-pass workgroup.
#ifdef SPH_STUDY
#define SPH_BLK_SHAPES(X) X(0, 64, 8, 4) X(1, 32, 8, 4) X(2, 32, 16, 2) X(3, 64, 16, 4) X(4, 32, 16, 4)
#else
#define SPH_BLK_SHAPES(X) X(0, 64, 8, 4) X(1, 32, 8, 4)
#endif
constexpr int BLK_NCH = 8;  // slot chunks preloaded per row (rows up to BLK_NCH*U*G entries)
// The pair passes walk a row's chunks of U * G entries in steps of G (the transposed layout,
// blk_tpos, ties the walk's U to the build's; round 3's 16-entry chunks with U = 2 were
// slower, profiles/r03/README.md)
template <int U>
struct BlkWalk {
  static constexpr int UW = U;
  static constexpr int NCH = BLK_NCH;
};
struct BlkShape {
  int R, G, U;
};
inline BlkShape blk_shape(int k) {
  switch (k) {
#define SPH_CASE(k, R, G, U) \
  case k: return BlkShape{R, G, U};
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
    default: return BlkShape{32, 16, 2};
  }
}

struct BlkArgs {
  int n = 0;            // owned rows
  int shape = 2;        // index into SPH_BLK_SHAPES
  int ucap = 0;         // union stride of ulist
  int um = 0;           // largest union of the build (the rho / inner passes' images)
  int umf = 0;          // force pass's LDS image (records, a multiple of 16); larger
                        // unions are walked in windows of umf records
  int sstride = 0;      // slot-row stride (entries)
  int exp = 0;          // study variants (SPH_EXP), 0 in production
  int cq = BLK_CH / 16;  // image chunk bytes / 16 (BLK_CHE / 16 with the heat term)
  const int *ulist = nullptr, *ucnt = nullptr, *rcnt = nullptr;
  // the union the inner rows index: their own (iu: k_blk_build / k_blk_inner renumbered
  // them) or the full one
  int *uilist = nullptr, *uicnt = nullptr;
  bool iu = false;
  const unsigned short *snbr = nullptr;
  // inner rows (k_blk_inner) and the device flag that retires them; snbi == nullptr: none
  const unsigned short *snbi = nullptr;
  const int *icnt = nullptr, *moved = nullptr;
  bool n3 = false;      // rows built with Newton-3 inside the blocks (k_blk_build N3)
  const unsigned char *bperm = nullptr;  // the passes' row order per block (k_blk_build)
  // a subset of the blocks (nlist ids; the pair passes only): the interior or the boundary
  // blocks of a brick (k_blk_interior), so the interior ones run while the halos move
  const int *blist = nullptr;
  int nlist = 0;
  bool pre(const BlkShape &sh) const { return sstride <= BLK_NCH * sh.U * sh.G; }
};

// a block is INTERIOR when its union names no ghost (index >= nlocal; the union is in the
// build's candidate order, so every entry is looked at: one wave per block, rebuilds only)
static __global__ void __launch_bounds__(64)
k_blk_interior(int nb, const int *__restrict__ ulist, const int *__restrict__ ucnt, int ucap,
               int nlocal, unsigned char *__restrict__ fin, unsigned char *__restrict__ fbd) {
  const int b = blockIdx.x;
  const int u = ucnt[b];
  const int *const ul = ulist + (size_t)b * ucap;
  bool ghost = false;
  for (int k = threadIdx.x; k < u; k += 64) ghost |= ul[k] >= nlocal;
  const bool any = __any(ghost);
  if (threadIdx.x == 0) {
    fin[b] = any ? 0 : 1;
    fbd[b] = any ? 1 : 0;
  }
}

inline int blk_blocks(int n, int R) { return (n + R - 1) / R; }

template <int R, int G, int U, int MC>
inline void blk_neigh_t(bool nt1, hipStream_t s, int n, const QBins &q, int dim,
                        const double4 *xf, const int *ty, const double4 *xb, const int *tb,
                        const int *qbeg, const int *xpos, const Coefs *cf, int ucap,
                        int sstride, int *ulist, int *ucnt, int *rcnt, unsigned short *snbr,
                        int *ovf, int *umax, int cq, int bexp) {
  if (nt1)
    hipLaunchKernelGGL((k_blk_neigh<R, G, U, true, MC>), dim3(blk_blocks(n, R)),
                       dim3(R * BLK_TPR), 0, s, n, q, dim, xf, ty, xb, tb, qbeg, xpos, cf, ucap,
                       sstride, ulist, ucnt, rcnt, snbr, ovf, umax, cq, bexp);
  else
    hipLaunchKernelGGL((k_blk_neigh<R, G, U, false, MC>), dim3(blk_blocks(n, R)),
                       dim3(R * BLK_TPR), 0, s, n, q, dim, xf, ty, xb, tb, qbeg, xpos, cf, ucap,
                       sstride, ulist, ucnt, rcnt, snbr, ovf, umax, cq, bexp);
}
// big: the large candidate image (BLK_MBIG; 32-row shapes only)
inline void blk_neigh(int shape, bool big, bool nt1, hipStream_t s, int n, const QBins &q,
                      int dim, const double4 *xf, const int *ty, const double4 *xb,
                      const int *tb, const int *qbeg, const int *xpos, const Coefs *cf,
                      int ucap, int sstride, int *ulist, int *ucnt, int *rcnt,
                      unsigned short *snbr, int *ovf, int *umax, int cq, int bexp = 0) {
  switch (shape) {
#define SPH_CASE(k, R, G, U)                                                                \
  case k:                                                                                 \
    if (big && R == 32)                                                                   \
      blk_neigh_t<R, G, U, BLK_MBIG>(nt1, s, n, q, dim, xf, ty, xb, tb, qbeg, xpos, cf,   \
                                     ucap, sstride, ulist, ucnt, rcnt, snbr, ovf, umax, cq, bexp); \
    else                                                                                  \
      blk_neigh_t<R, G, U, BLK_MCAP>(nt1, s, n, q, dim, xf, ty, xb, tb, qbeg, xpos, cf,   \
                                     ucap, sstride, ulist, ucnt, rcnt, snbr, ovf, umax, cq, bexp); \
    break;
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
  }
}

// k_blk_build (the default block build; k_blk_neigh remains the large-image fallback)
template <int R, int G, int U, bool NT1, bool INNER, bool N3>
inline void blk_build_t(hipStream_t s, int n, const QBins &q, int dim, const double4 *xf,
                        const int *ty, const double4 *xb, const int *tb, const int *qbeg,
                        const Coefs *cf, int ucap, int sstride, int *ulist, int *ucnt,
                        int *rcnt, unsigned short *snbr, int *icnt, unsigned short *snbi,
                        int *ovf, int *umax, int cq, int bexp, int *fcnt, unsigned char *bperm,
                        int *uilist, int *uicnt, int *kcnt) {
  // (bexp bit 8: the small candidate image, BLK_SCAP_S)
  const bool small = (bexp & 0x100) != 0;
  bexp &= 0xff;
#ifdef SPH_STUDY
  auto fn = bexp == 1 ? k_blk_build<R, G, U, NT1, INNER, N3, 1>
          : bexp == 2 ? k_blk_build<R, G, U, NT1, INNER, N3, 2>
          : bexp == 3 ? k_blk_build<R, G, U, NT1, INNER, N3, 3>
          : bexp == 4 ? k_blk_build<R, G, U, NT1, INNER, N3, 4>
          : small     ? k_blk_build<R, G, U, NT1, INNER, N3, 0, BLK_SCAP_S>
                      : k_blk_build<R, G, U, NT1, INNER, N3, 0>;
#else
  auto fn = small ? k_blk_build<R, G, U, NT1, INNER, N3, 0, BLK_SCAP_S>
                  : k_blk_build<R, G, U, NT1, INNER, N3, 0>;
#endif
  hipLaunchKernelGGL(fn, dim3(blk_blocks(n, R)), dim3(256), 0, s, n, q, dim, xf, ty, xb, tb,
                     qbeg, cf, ucap, sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, umax, cq,
                     fcnt, bperm, uilist, uicnt, kcnt);
  hipLaunchKernelGGL(k_blk_stats, dim3(1), dim3(1024), 0, s, blk_blocks(n, R), ucnt, kcnt,
                     uicnt, umax);
}
template <int R, int G, int U, bool N3>
inline void blk_build_n(bool nt1, bool inner, hipStream_t s, int n, const QBins &q, int dim,
                        const double4 *xf, const int *ty, const double4 *xb, const int *tb,
                        const int *qbeg, const Coefs *cf, int ucap, int sstride, int *ulist,
                        int *ucnt, int *rcnt, unsigned short *snbr, int *icnt,
                        unsigned short *snbi, int *ovf, int *umax, int cq, int bexp, int *fcnt,
                        unsigned char *bperm, int *uilist, int *uicnt, int *kcnt) {
  if (nt1 && inner)
    blk_build_t<R, G, U, true, true, N3>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap, sstride,
                                         ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, umax, cq, bexp,
                                         fcnt, bperm, uilist, uicnt, kcnt);
  else if (nt1)
    blk_build_t<R, G, U, true, false, N3>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap, sstride,
                                          ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, umax, cq,
                                          bexp, fcnt, bperm, uilist, uicnt, kcnt);
  else if (inner)
    blk_build_t<R, G, U, false, true, N3>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap, sstride,
                                          ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, umax, cq,
                                          bexp, fcnt, bperm, uilist, uicnt, kcnt);
  else
    blk_build_t<R, G, U, false, false, N3>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,
                                           sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf,
                                           umax, cq, bexp, fcnt, bperm, uilist, uicnt, kcnt);
}
// n3: Newton-3 inside the blocks (rows first in the union, the later rows' share; fcnt gets
// the full counts)
inline void blk_build(int shape, bool nt1, bool inner, bool n3, hipStream_t s, int n,
                      const QBins &q, int dim, const double4 *xf, const int *ty,
                      const double4 *xb, const int *tb, const int *qbeg, const Coefs *cf,
                      int ucap, int sstride, int *ulist, int *ucnt, int *rcnt,
                      unsigned short *snbr, int *icnt, unsigned short *snbi, int *ovf, int *umax,
                      int cq, int bexp, int *fcnt, unsigned char *bperm, int *uilist,
                      int *uicnt, int *kcnt) {
#ifdef SPH_STUDY
#define SPH_IF_N3(R, G, U)                                                                  \
  if (n3)                                                                                 \
    blk_build_n<R, G, U, true>(nt1, inner, s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,    \
                               sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, umax, cq, \
                               bexp, fcnt, bperm, uilist, uicnt, kcnt);                           \
  else
#else
#define SPH_IF_N3(R, G, U) (void)n3;
#endif
  switch (shape) {
#define SPH_CASE(k, R, G, U)                                                                \
  case k:                                                                                 \
    SPH_IF_N3(R, G, U)                                                                    \
    blk_build_n<R, G, U, false>(nt1, inner, s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,   \
                                sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, umax, cq, \
                                bexp, fcnt, bperm, uilist, uicnt, kcnt);                          \
    break;
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
#undef SPH_IF_N3
  }
}

template <int R, int G, int U, int NCH, bool NT1>
inline void blk_rhosum_t(hipStream_t s, const BlkArgs &k, double4 *xf, const int *ty,
                         double4 *vr, const Coefs *cf) {
  const size_t lds = blk_rho_lds(k.um, NT1);
  auto fn = k.cq == BLK_CH / 16 ? k_blk_rhosum<R, G, U, NCH, NT1, BLK_CH / 16>
                                : k_blk_rhosum<R, G, U, NCH, NT1, BLK_CHE / 16>;
  SPH_HIP_TRY(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  const int nb = k.blist ? k.nlist : blk_blocks(k.n, R);
  if (nb == 0) return;
  hipLaunchKernelGGL(fn, dim3(nb), dim3(R * G), lds, s, k.n, k.ulist, k.ucnt,
                     k.ucap, k.snbr, k.sstride, k.rcnt, xf, ty, vr, cf, k.um, k.snbi, k.icnt,
                     k.moved, k.n3 ? 1 : 0, k.bperm, k.uilist, k.uicnt, k.blist);
}
template <int R, int G, int U>
inline void blk_rhosum_s(bool nt1, hipStream_t s, const BlkArgs &k, double4 *xf, const int *ty,
                         double4 *vr, const Coefs *cf) {
  const bool pre = k.pre(BlkShape{R, G, U});
  constexpr int UW = BlkWalk<U>::UW, NW = BlkWalk<U>::NCH;
  if (nt1) {
    if (pre) blk_rhosum_t<R, G, UW, NW, true>(s, k, xf, ty, vr, cf);
    else blk_rhosum_t<R, G, U, 0, true>(s, k, xf, ty, vr, cf);
  } else {
    if (pre) blk_rhosum_t<R, G, UW, NW, false>(s, k, xf, ty, vr, cf);
    else blk_rhosum_t<R, G, U, 0, false>(s, k, xf, ty, vr, cf);
  }
}
inline void blk_rhosum(bool nt1, hipStream_t s, const BlkArgs &k, double4 *xf, const int *ty,
                       double4 *vr, const Coefs *cf) {
  if (k.n == 0) return;
  switch (k.shape) {
#define SPH_CASE(q, R, G, U) \
  case q: blk_rhosum_s<R, G, U>(nt1, s, k, xf, ty, vr, cf); break;
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
  }
}

template <int R, int G, int U, int NCH, int VISC, int MODE, bool NT1, int EXP = 0>
inline void blk_force_t(hipStream_t s, const BlkArgs &k, const RowArgs &a) {
  auto fn = [] {
    if constexpr (NT1 && MODE == M_TAIT && EXP == 0 && NCH > 0 && SPH_BLK_WPE == 0 && SPH_BLK_W6)
      return k_blk_force_w6<R, G, U, NCH, VISC, MODE, NT1, EXP>;
    else if constexpr (NT1 && MODE == M_TAIT && EXP == 0 && NCH > 0 && SPH_BLK_WPE == 0)
      return k_blk_force_w5<R, G, U, NCH, VISC, MODE, NT1, EXP>;
    else
      return k_blk_force<R, G, U, NCH, VISC, MODE, NT1, EXP>;
  }();
  // one launch: every block, its union in windows of umf records where it exceeds the image
  size_t lds = blk_lds(k.umf, k.cq, NT1);
#ifdef SPH_STUDY  // (SPH_LDS_PAD: extra LDS per workgroup, an occupancy study)
  if (const char *e = getenv("SPH_LDS_PAD")) lds += (size_t)atoi(e);
#endif
  SPH_HIP_TRY(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  const int nb = k.blist ? k.nlist : blk_blocks(k.n, R);
  if (nb == 0) return;
  hipLaunchKernelGGL(fn, dim3(nb), dim3(R * G), lds, s, k.n, k.ulist, k.ucnt,
                     k.ucap, k.snbr, k.sstride, k.rcnt, a.xf, a.vr, a.ty, a.en, a.cf, a.fo,
                     a.de, a.gx, a.gy, a.gz, k.umf, k.cq, k.snbi, k.icnt, k.moved,
                     k.n3 ? 1 : 0, k.bperm, k.uilist, k.uicnt, k.blist);
}

// the inner rows of a build (k_blk_inner): same launch geometry and LDS image as rhosum
// (refresh: cond != nullptr, see k_blk_inner; a grid of at most 512 workgroups, so that a
// launch whose flag is clear costs a few microseconds)
struct BlkInnerRefresh {
  const int *cond = nullptr;
  int *zero = nullptr;
  double4 *x0 = nullptr;
  int *umax = nullptr;  // (the inner unions' largest and sum, as k_blk_build's umax + 6, 7)
};
template <int R, int G, int U, int NCH, bool NT1>
inline void blk_inner_t(hipStream_t s, const BlkArgs &k, const double4 *xf, const int *ty,
                        const Coefs *cf, unsigned short *snbi, int *icnt,
                        const BlkInnerRefresh &rf) {
  const size_t lds = blk_rho_lds(k.um, NT1);
  auto fn = k.cq == BLK_CH / 16 ? k_blk_inner<R, G, U, NCH, NT1, BLK_CH / 16>
                                : k_blk_inner<R, G, U, NCH, NT1, BLK_CHE / 16>;
  SPH_HIP_TRY(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  const int nb = blk_blocks(k.n, R);
  hipLaunchKernelGGL(fn, dim3(rf.cond ? std::min(nb, 512) : nb), dim3(R * G), lds, s, k.n,
                     k.ulist, k.ucnt, k.ucap, k.snbr, k.sstride, k.rcnt, xf, ty, cf, snbi, icnt,
                     k.um, rf.cond, rf.zero, rf.x0, k.iu ? k.uilist : nullptr,
                     k.iu ? k.uicnt : nullptr, rf.umax);
}
template <int R, int G, int U>
inline void blk_inner_s(bool nt1, hipStream_t s, const BlkArgs &k, const double4 *xf,
                        const int *ty, const Coefs *cf, unsigned short *snbi, int *icnt,
                        const BlkInnerRefresh &rf) {
  const bool pre = k.pre(BlkShape{R, G, U});
  if (nt1) {
    if (pre) blk_inner_t<R, G, U, BLK_NCH, true>(s, k, xf, ty, cf, snbi, icnt, rf);
    else blk_inner_t<R, G, U, 0, true>(s, k, xf, ty, cf, snbi, icnt, rf);
  } else {
    if (pre) blk_inner_t<R, G, U, BLK_NCH, false>(s, k, xf, ty, cf, snbi, icnt, rf);
    else blk_inner_t<R, G, U, 0, false>(s, k, xf, ty, cf, snbi, icnt, rf);
  }
}
inline void blk_inner(bool nt1, hipStream_t s, const BlkArgs &k, const double4 *xf,
                      const int *ty, const Coefs *cf, unsigned short *snbi, int *icnt,
                      const BlkInnerRefresh &rf = BlkInnerRefresh{}) {
  if (k.n == 0) return;
  switch (k.shape) {
#define SPH_CASE(q, R, G, U) \
  case q: blk_inner_s<R, G, U>(nt1, s, k, xf, ty, cf, snbi, icnt, rf); break;
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
  }
}
template <int R, int G, int U, int NCH, bool NT1>
inline void blk_force_n(int visc, int mode, hipStream_t s, const BlkArgs &k, const RowArgs &a) {
  const bool mor = visc == SPH_VISC_MORRIS;
  switch (mode) {
    case M_TAIT:
      if (mor) blk_force_t<R, G, U, NCH, 1, M_TAIT, NT1>(s, k, a);
      else if (NT1 && visc == BLK_VISC_NONE)
        blk_force_t<R, G, U, NCH, BLK_VISC_NONE, M_TAIT, NT1>(s, k, a);
#ifdef SPH_STUDY  // (outputs meaningless: study builds only, make STUDY=1)
      else if (NT1 && k.exp == 1) blk_force_t<R, G, U, NCH, 0, M_TAIT, NT1, 1>(s, k, a);
      else if (NT1 && k.exp == 2) blk_force_t<R, G, U, NCH, 0, M_TAIT, NT1, 2>(s, k, a);
      else if (NT1 && k.exp == 3) blk_force_t<R, G, U, NCH, 0, M_TAIT, NT1, 3>(s, k, a);
#endif
      else blk_force_t<R, G, U, NCH, 0, M_TAIT, NT1>(s, k, a);
      break;
    case M_TAIT | M_HEAT:
      if (mor) blk_force_t<R, G, U, NCH, 1, M_TAIT | M_HEAT, NT1>(s, k, a);
      else blk_force_t<R, G, U, NCH, 0, M_TAIT | M_HEAT, NT1>(s, k, a);
      break;
    default: blk_force_t<R, G, U, NCH, 0, M_HEAT, NT1>(s, k, a); break;
  }
}
template <int R, int G, int U>
inline void blk_force_s(bool nt1, int visc, int mode, hipStream_t s, const BlkArgs &k,
                        const RowArgs &a) {
  const bool pre = k.pre(BlkShape{R, G, U});
  constexpr int UW = BlkWalk<U>::UW, NW = BlkWalk<U>::NCH;
  if (nt1) {
    if (pre) blk_force_n<R, G, UW, NW, true>(visc, mode, s, k, a);
    else blk_force_n<R, G, U, 0, true>(visc, mode, s, k, a);
  } else {
    if (pre) blk_force_n<R, G, UW, NW, false>(visc, mode, s, k, a);
    else blk_force_n<R, G, U, 0, false>(visc, mode, s, k, a);
  }
}
inline void blk_force(bool nt1, int visc, int mode, hipStream_t s, const BlkArgs &k,
                      const RowArgs &a) {
  if (k.n == 0) return;
  switch (k.shape) {
#define SPH_CASE(q, R, G, U) \
  case q: blk_force_s<R, G, U>(nt1, visc, mode, s, k, a); break;
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
  }
}

}  // namespace sph
