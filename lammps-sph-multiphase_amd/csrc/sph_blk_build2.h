// sph_blk_build2.h -- the block neighbour build with GROUP candidate lists (STUDY builds only:
// measured slower than k_blk_build, 1.37 vs 1.11 ms at C2 1M, profiles/r05/README.md; make STUDY=1).
//
// k_blk_build (sph_blk_kernels.h) tests every row of a 64-row block against every candidate
// of the block's sphere-swept box: ~1000 candidates per row for ~155 hits at C2 (12 %).  A
// group of 8 consecutive rows (Hilbert order: a ~2x2x2 piece of the block) sees only the
// candidates within cutneighmax of ITS box, ~350 of them, so here each group first filters
// the block's candidates against its own box (one box test per candidate and group) and then
// tests its 8 rows against its own list only: ~2.7x fewer row tests.  Everything else is
// k_blk_build's: Neighbor::full_bin membership (rsq <= cutneighsq[it][jt], j != i;
// neigh_full.cpp:305-312), the block's union = the candidates some row names, numbered in
// candidate order (slot = rank + 1), the inner rows (rsq < (cut + margin)^2) over their own
// union, 16-bit slot rows in ascending slot order, chunk-transposed (blk_tpos) -- so the
// outputs are identical to k_blk_build's, bit for bit.
//   1. the rows, the block box and the 8-row groups' boxes;
//   2. the block's raw candidates (bins) and its prefilter (distance to the block box), as
//      k_blk_build;
//   3. each group's list: the kept candidates within cutneighmax of the group box (ordered;
//      the lists share a pool of BLK2_GPOOL entries -- more raises *ovf = 1 << 23 and the host
//      takes k_blk_build);
//   4. tests: a wave takes a group and 64 of its candidates at a time (one per lane), its 8
//      rows unrolled, the rows' 64-bit hit words (full, inner) kept in lanes 0-7 by
//      v_writelane; the words' OR marks the union bits (LDS atomics: groups share candidates);
//   5. the unions (full, inner) and their slot words per kept candidate; 6. the rows.
#pragma once
#include "sph_blk_kernels.h"

namespace sph {

#ifndef SPH_B2EXP
#define SPH_B2EXP 0  // (A/B builds: 1 = return after the group lists, 2 = after the tests,
                     //  3 = after the unions; outputs meaningless)
#endif
constexpr int BLK2_GR = 8;        // rows per group
constexpr int BLK2_GPOOL = 4096;  // candidates in all of a block's group lists together
//                                   (~2.8k at C2; a group spanning a jump of the Hilbert
//                                   curve takes a larger share)

template <int R, int G, int U, bool NT1, bool INNER>
__global__ void __launch_bounds__(256)
k_blk_build2(int n, QBins q, int dim, const double4 *__restrict__ xf,
             const int *__restrict__ ty, const double4 *__restrict__ xb,
             const int *__restrict__ tb, const int *__restrict__ qbeg,
             const Coefs *__restrict__ cf, int ucap, int sstride, int *__restrict__ ulist,
             int *__restrict__ ucnt, int *__restrict__ rcnt, unsigned short *__restrict__ snbr,
             int *__restrict__ icnt, unsigned short *__restrict__ snbi,
             int *__restrict__ ovf, int cq, int *__restrict__ uilist, int *__restrict__ uicnt,
             int *__restrict__ kcnt) {
  constexpr int NT = 256, NW = NT / 64, MCH = BLK_MCAP / 64, SCH = BLK_SCAP / 64;
  constexpr int NG = R / BLK2_GR, UG = U * G, WS = INNER ? 2 : 1;
  static_assert(R <= 64 && R % BLK2_GR == 0, "8-row groups of at most 64 rows");
  static_assert(UG <= 64 && U * 16 <= 64, "a row's padding in one store, U slots per word");
  const bool iu = INNER && uilist != nullptr;
  // the groups' hit words [group][chunk][row] (full, inner); before the tests the storage
  // holds the raw candidates' bin-row numbers
  constexpr int NWD = (BLK2_GPOOL / 64 + NG) * BLK2_GR * WS;  // (chunks of all the groups)
  __shared__ __attribute__((aligned(16)))
  unsigned long long s_w[NWD * 8 >= BLK_MCAP ? NWD : BLK_MCAP / 8];
  unsigned char *const s_rowof = reinterpret_cast<unsigned char *>(s_w);
  __shared__ unsigned long long s_used[SCH], s_usedi[INNER ? SCH : 1];
  __shared__ int s_upre[SCH + 1], s_upi[INNER ? SCH + 1 : 1];
  __shared__ unsigned long long s_keep[MCH];
  __shared__ int s_kpre[MCH + 1];
  __shared__ int s_cpos[BLK_SCAP];
  __shared__ unsigned short s_q[BLK_SCAP], s_qi[INNER ? BLK_SCAP : 1];
  __shared__ unsigned long long s_gm[NG][SCH];  // group membership of the kept candidates
  __shared__ unsigned short s_gl[BLK2_GPOOL];  // the group lists, group g's from s_go[g] on
  __shared__ int s_gn[NG], s_go[NG], s_gc[NG];  // counts, list offsets, first word chunks
  __shared__ int s_pre[BLK_TBL + 1], s_st[BLK_TBL];
  __shared__ double4 s_row[R];
  __shared__ int s_rty[R];
  __shared__ double s_bb[6], s_gbb[NG][6];
  __shared__ double s_cns[NT1 ? 1 : NT2], s_cin[(NT1 || !INNER) ? 1 : NT2];
  __shared__ int s_sc[NW];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63,
            wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = b * R;
  const int nrow = min(R, n - row0);
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = tid; t < nt1 * nt1; t += NT) {
      s_cns[t] = cf->cutneighsq[t];
      if (INNER) s_cin[t] = cf->cutinsq[t];
    }
  // 1) the rows (past the last one: far away, never a hit), the block box and group boxes
  if (wv == 0) {
    double lo[3], hi[3];
    const bool in = lane < nrow;
    double4 x = make_double4(1e300, 1e300, 1e300, 0.0);
    if (in) x = xf[row0 + lane];
    if (lane < R) {
      s_row[lane] = x;
      if (!NT1) s_rty[lane] = in ? ty[row0 + lane] : 1;
    }
    lo[0] = in ? x.x : 1e300;
    lo[1] = in ? x.y : 1e300;
    lo[2] = in ? x.z : 1e300;
    hi[0] = in ? x.x : -1e300;
    hi[1] = in ? x.y : -1e300;
    hi[2] = in ? x.z : -1e300;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        lo[k] = fmin(lo[k], __shfl_xor(lo[k], d, 64));
        hi[k] = fmax(hi[k], __shfl_xor(hi[k], d, 64));
      }
      if (d == BLK2_GR / 2 && (lane & (BLK2_GR - 1)) == 0 && lane < R)
        for (int k = 0; k < 3; k++) {  // (the 8-lane group's box, after 3 steps)
          s_gbb[lane / BLK2_GR][k] = lo[k];
          s_gbb[lane / BLK2_GR][3 + k] = hi[k];
        }
    }
    if (lane == 0)
      for (int k = 0; k < 3; k++) {
        s_bb[k] = lo[k];
        s_bb[3 + k] = hi[k];
      }
  }
  __syncthreads();
  // 2) the bin-rows of the block's sphere-swept box, the raw candidates, the prefilter
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
  if (tid < ny * nz) {
    s_pre[tid] = pre;
    s_st[tid] = st;
    for (int k = 0; k < len; k++) s_rowof[pre + k] = (unsigned char)tid;
  }
  __syncthreads();
  const int mch = (M + 63) >> 6;
  auto rpos = [&](int p) {  // raw candidate p -> its xb position
    const int t = s_rowof[p];
    return s_st[t] + (p - s_pre[t]);
  };
  const double cmsq = q.cutmaxsq * (1.0 + 1e-9) + 1e-12 * q.size[0] * q.size[0];
  auto near = [&](const double *bb, const double4 &x) {  // distance to a box <= cutneighmax
    const double gx = fmax(fmax(bb[0] - x.x, x.x - bb[3]), 0.0);
    const double gy = fmax(fmax(bb[1] - x.y, x.y - bb[4]), 0.0);
    const double gz = fmax(fmax(bb[2] - x.z, x.z - bb[5]), 0.0);
    return gx * gx + gy * gy + gz * gz <= cmsq;
  };
  for (int c = wv; c < mch; c += 2 * NW) {
    const int p = c * 64 + lane, p2 = p + NW * 64;
    double4 x = make_double4(0.0, 0.0, 0.0, 0.0), x2 = x;
    if (p < M) x = xb[rpos(p)];
    if (p2 < M) x2 = xb[rpos(p2)];
    const unsigned long long k = __ballot(p < M && near(s_bb, x));
    const unsigned long long k2 = __ballot(p2 < M && near(s_bb, x2));
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
  if (K > BLK_SCAP) {  // workgroup-uniform
    if (tid == 0) atomicMax(ovf, 1 << 22);
    return;
  }
  __syncthreads();
  for (int c = wv; c < mch; c += NW) {
    const unsigned long long k = s_keep[c];
    if ((k >> lane) & 1ull)
      s_cpos[s_kpre[c] + __popcll(k & ((1ull << lane) - 1ull))] = rpos(c * 64 + lane);
  }
  const int nch = (K + 63) >> 6;
  for (int t = tid; t < nch; t += NT) {
    s_used[t] = 0ull;
    if (INNER) s_usedi[t] = 0ull;
  }
  __syncthreads();
  // 3) the groups' lists: kept candidates near each group's box, in candidate order
  for (int c = wv; c < nch; c += NW) {
    const int p = c * 64 + lane;
    double4 x = make_double4(1e300, 1e300, 1e300, 0.0);
    if (p < K) x = xb[s_cpos[p]];
#pragma unroll
    for (int g = 0; g < NG; g++) {
      const unsigned long long m = __ballot(p < K && near(s_gbb[g], x));
      if (lane == 0) s_gm[g][c] = m;
    }
  }
  __syncthreads();
  if (tid < NG) {  // (NG <= 8 threads: each group's count over its words)
    int cnt = 0;
    for (int c = 0; c < nch; c++) cnt += __popcll(s_gm[tid][c]);
    s_gn[tid] = cnt;
  }
  __syncthreads();
  if (tid == 0) {  // the groups' shares of the pools
    int o = 0, w = 0;
    for (int g = 0; g < NG; g++) {
      s_go[g] = o;
      s_gc[g] = w;
      o += s_gn[g];
      w += (s_gn[g] + 63) >> 6;
    }
    s_sc[0] = o;
  }
  __syncthreads();
  if (s_sc[0] > BLK2_GPOOL) {  // (workgroup-uniform) the host takes k_blk_build
    if (tid == 0) atomicMax(ovf, 1 << 23);
    return;
  }
  // compaction: wave wv takes groups wv, wv + NW, ..; its lanes walk the words in order
  for (int g = wv; g < NG; g += NW) {
    int base = s_go[g];
    for (int c = 0; c < nch; c++) {
      const unsigned long long m = s_gm[g][c];  // (uniform)
      if ((m >> lane) & 1ull) s_gl[base + blk_mbcnt(m)] = (unsigned short)(c * 64 + lane);
      base += __popcll(m);
    }
  }
  __syncthreads();
  // (the A/B variants leave a valid, empty block behind: no union, no entries)
  auto blank = [&]() {
    if (tid == 0) {
      ucnt[b] = 0;
      kcnt[b] = 0;
      if (iu) uicnt[b] = 0;
    }
    if (tid < nrow) {
      rcnt[row0 + tid] = 0;
      if (INNER) icnt[row0 + tid] = 0;
    }
  };
  if (SPH_B2EXP == 1) {
    blank();
    return;
  }
  // 4) tests: group g, 64 of its candidates per step against its 8 rows
  const double cns1 = NT1 ? cf->cutneighsq[3] : 0.0;
  const double cin1 = (NT1 && INNER) ? cf->cutinsq[3] : 0.0;
  for (int g = wv; g < NG; g += NW) {
    const int gn = s_gn[g], gch = (gn + 63) >> 6, go = s_go[g], gc = s_gc[g];
    const int r0 = g * BLK2_GR;
    for (int k = 0; k < gch; k++) {
      const int e = k * 64 + lane;
      const bool valid = e < gn;
      const int p = valid ? s_gl[go + e] : 0;
      double4 xc = make_double4(-1e300, -1e300, -1e300, -1.0);
      int tc = 1;
      if (valid) {
        const int pos = s_cpos[p];
        xc = xb[pos];
        if (!NT1) tc = tb[pos];
      }
      const int cid = valid ? (int)xc.w : -1;
      unsigned my_lo = 0u, my_hi = 0u, mi_lo = 0u, mi_hi = 0u;
      int ro = 0;  // (opaque: keeps the rows' positions in LDS, not hoisted into registers)
      asm volatile("" : "+s"(ro));
      blk_rows<BLK2_GR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        const double4 xi = s_row[r0 + r + ro];
        const double rsq = rsq_ref(xi.x - xc.x, xi.y - xc.y, xi.z - xc.z);
        double cn = cns1, ci = cin1;
        if (!NT1) {
          const int it = s_rty[r0 + r];
          cn = s_cns[it * nt1 + tc];
          if (INNER) ci = s_cin[it * nt1 + tc];
        }
        const bool self = cid == row0 + r0 + r;  // (j != i)
        const unsigned long long m = __builtin_amdgcn_ballot_w64(rsq <= cn && !self);
        my_lo = writelane<r>(my_lo, (unsigned)m);
        my_hi = writelane<r>(my_hi, (unsigned)(m >> 32));
        if (INNER) {
          const unsigned long long mi = __builtin_amdgcn_ballot_w64(rsq < ci && !self);
          mi_lo = writelane<r>(mi_lo, (unsigned)mi);
          mi_hi = writelane<r>(mi_hi, (unsigned)(mi >> 32));
        }
      });
      const unsigned long long full = ((unsigned long long)my_hi << 32) | my_lo;
      const unsigned long long inw = ((unsigned long long)mi_hi << 32) | mi_lo;
      if (lane < BLK2_GR) {
        const int w = (gc + k) * BLK2_GR + lane;
        if (INNER)
          reinterpret_cast<ulonglong2 *>(s_w)[w] = make_ulonglong2(full, inw);
        else
          s_w[w] = full;
      }
      // the union bits: candidate p is used if any of the 8 rows names it
      unsigned long long u = full, ui = inw;
#pragma unroll
      for (int d = 1; d < BLK2_GR; d <<= 1) {
        u |= __shfl_xor(u, d, 64);
        if (INNER) ui |= __shfl_xor(ui, d, 64);
      }
      u = blk_uniform64(u);  // (lanes 0-7 held the rows' words; lane 0 has their OR)
      if (INNER) ui = blk_uniform64(ui);
      if (valid && ((u >> lane) & 1ull)) atomicOr(&s_used[p >> 6], 1ull << (p & 63));
      if (INNER && iu && valid && ((ui >> lane) & 1ull))
        atomicOr(&s_usedi[p >> 6], 1ull << (p & 63));
    }
  }
  __syncthreads();
  if (SPH_B2EXP == 2) {
    blank();
    return;
  }
  // 5) the unions (slot = rank among used candidates + 1) and each kept candidate's slot words
  int u = 0, ui_tot = 0;
  {
    const int v = tid < nch ? __popcll(s_used[tid]) : 0;
    const int ex = blk_scan<NT>(v, s_sc, &u);
    if (tid < nch) s_upre[tid] = ex;
  }
  if (iu) {
    const int v = tid < nch ? __popcll(s_usedi[tid]) : 0;
    const int ex = blk_scan<NT>(v, s_sc, &ui_tot);
    if (tid < nch) s_upi[tid] = ex;
  }
  __syncthreads();
  for (int c = wv; c < nch; c += NW) {
    const int p = c * 64 + lane;
    if (p >= K) continue;
    const unsigned long long used = s_used[c];
    const int below = blk_mbcnt(used);
    s_q[p] = (unsigned short)blk_q(s_upre[c] + 1 + below, cq);
    const int aid = (int)xb[s_cpos[p]].w;
    if ((used >> lane) & 1ull) ulist[(size_t)b * ucap + s_upre[c] + below] = aid;
    if (iu) {
      const unsigned long long usedi = s_usedi[c];
      const int bi = blk_mbcnt(usedi);
      s_qi[p] = (unsigned short)blk_q(s_upi[c] + 1 + bi, cq);
      if ((usedi >> lane) & 1ull) uilist[(size_t)b * ucap + s_upi[c] + bi] = aid;
    }
  }
  if (tid == 0) {
    ucnt[b] = u;
    kcnt[b] = K;
    if (iu) uicnt[b] = ui_tot;
  }
  __syncthreads();
  if (SPH_B2EXP == 3) {
    blank();
    return;
  }
  // 6) the slot rows, full and inner: wave w writes rows w*RPW .. with LPR lanes per row,
  // lane `part` the row's output chunks part, part + LPR, .. (U*G entries each, transposed
  // as blk_tpos), walking the row's set bits over its group's words in candidate order
  constexpr int RPW = R / NW, LPR = 64 / RPW;
  const int r = wv * RPW + lane / LPR, part = lane % LPR;
  const bool live = r < nrow;
  const int g = r / BLK2_GR, rg = r % BLK2_GR;
  const int gch = (s_gn[g] + 63) >> 6, go = s_go[g], gc = s_gc[g];
  bool over = false;
  auto emit = [&](int sel, unsigned short *__restrict__ rows, int *__restrict__ cnt_out) {
    auto word = [&](int k) -> unsigned long long {
      const int w = (gc + k) * BLK2_GR + rg;
      return INNER ? s_w[w * 2 + sel] : s_w[w];
    };
    const unsigned short *const qt = (iu && sel == 1) ? s_qi : s_q;
    int cnt = 0;
    if (live)
      for (int k = 0; k < gch; k++) cnt += __popcll(word(k));
    const int nchunk = min((cnt + UG - 1) / UG, sstride / UG);
    unsigned short *const out = rows + (size_t)(row0 + r) * sstride;
    int c = 0, acc = 0;  // word c holds the entries from acc on
    unsigned long long w = (live && gch > 0) ? word(0) : 0ull;
    for (int ch = part; ch < nchunk; ch += LPR) {
      const int e0 = ch * UG;
      while (acc + __popcll(w) <= e0) {  // (e0 < cnt: the word holding it exists)
        acc += __popcll(w);
        w = word(++c);
      }
      unsigned long long m = w;
      for (int j = e0 - acc; j > 0; j--) m &= m - 1ull;
      int cc = c;
      const int ne = min(cnt - e0, UG);
      unsigned long long buf[G];
#pragma unroll
      for (int l = 0; l < G; l++) buf[l] = 0ull;
#pragma unroll
      for (int qq = 0; qq < U; qq++)
#pragma unroll
        for (int l = 0; l < G; l++)
          if (qq * G + l < ne) {
            while (m == 0ull) m = word(++cc);
            const int bit = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            buf[l] |= (unsigned long long)qt[s_gl[go + cc * 64 + bit]] << (16 * qq);
          }
      if (U == 4) {
        ulonglong2 *const o = reinterpret_cast<ulonglong2 *>(out + e0);
#pragma unroll
        for (int t = 0; t < G / 2; t++) o[t] = make_ulonglong2(buf[2 * t], buf[2 * t + 1]);
      } else {
#pragma unroll
        for (int l = 0; l < G; l++)
#pragma unroll
          for (int qq = 0; qq < U; qq++)
            out[e0 + l * U + qq] = (unsigned short)(buf[l] >> (16 * qq));
      }
    }
    if (live && part == 0) {
      cnt_out[row0 + r] = cnt;
      over |= cnt > sstride;
    }
  };
  emit(0, snbr, rcnt);
  if (INNER) emit(1, snbi, icnt);
  if (over) atomicMax(ovf, 1 << 21);
}

template <int R, int G, int U, bool NT1, bool INNER>
inline void blk_build2_t(hipStream_t s, int n, const QBins &q, int dim, const double4 *xf,
                         const int *ty, const double4 *xb, const int *tb, const int *qbeg,
                         const Coefs *cf, int ucap, int sstride, int *ulist, int *ucnt,
                         int *rcnt, unsigned short *snbr, int *icnt, unsigned short *snbi,
                         int *ovf, int *umax, int cq, int *uilist, int *uicnt, int *kcnt) {
  hipLaunchKernelGGL((k_blk_build2<R, G, U, NT1, INNER>), dim3(blk_blocks(n, R)), dim3(256), 0,
                     s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap, sstride, ulist, ucnt, rcnt,
                     snbr, icnt, snbi, ovf, cq, uilist, uicnt, kcnt);
  hipLaunchKernelGGL(k_blk_stats, dim3(1), dim3(1024), 0, s, blk_blocks(n, R), ucnt, kcnt,
                     uilist ? uicnt : nullptr, umax);
}
// the group-list build in the SPH_BLK shape (no Newton-3, no row permutation: k_blk_build
// keeps those study variants)
inline void blk_build2(int shape, bool nt1, bool inner, hipStream_t s, int n, const QBins &q,
                       int dim, const double4 *xf, const int *ty, const double4 *xb,
                       const int *tb, const int *qbeg, const Coefs *cf, int ucap, int sstride,
                       int *ulist, int *ucnt, int *rcnt, unsigned short *snbr, int *icnt,
                       unsigned short *snbi, int *ovf, int *umax, int cq, int *uilist,
                       int *uicnt, int *kcnt) {
  switch (shape) {
#define SPH_CASE(k, R, G, U)                                                                  \
  case k:                                                                                   \
    if (nt1 && inner)                                                                       \
      blk_build2_t<R, G, U, true, true>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,       \
                                        sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf,  \
                                        umax, cq, uilist, uicnt, kcnt);                     \
    else if (nt1)                                                                           \
      blk_build2_t<R, G, U, true, false>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,      \
                                         sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, \
                                         umax, cq, uilist, uicnt, kcnt);                    \
    else if (inner)                                                                         \
      blk_build2_t<R, G, U, false, true>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,      \
                                         sstride, ulist, ucnt, rcnt, snbr, icnt, snbi, ovf, \
                                         umax, cq, uilist, uicnt, kcnt);                    \
    else                                                                                    \
      blk_build2_t<R, G, U, false, false>(s, n, q, dim, xf, ty, xb, tb, qbeg, cf, ucap,     \
                                          sstride, ulist, ucnt, rcnt, snbr, icnt, snbi,     \
                                          ovf, umax, cq, uilist, uicnt, kcnt);              \
    break;
    SPH_BLK_SHAPES(SPH_CASE)
#undef SPH_CASE
  }
}

}  // namespace sph
