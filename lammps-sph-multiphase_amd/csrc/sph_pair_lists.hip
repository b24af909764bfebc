// sph_pair_lists.hip -- neighbor lists built on the device for the pair-style layer
// (include/sph_hip.h sph_hip_build_list; SURVEY.md 8(b) "device-list path (preferred)", the
// GPU package's GPU_NEIGH precedent, src/GPU/pair_lj_cut_gpu.cpp:97-104).
//
// From the atoms the context has staged (owned + ghosts, as LAMMPS holds them after
// comm->borders), a FULL list with Neighbor::full_bin's membership (neigh_full.cpp:241-344:
// every j != i with rsq <= cutneighsq[itype][jtype], owned rows, ilist = identity) and, for
// SPH_LIST_HALF, Neighbor::half_from_full_newton's half of it (neigh_derive.cpp:83-150) --
// the lists LAMMPS would have built for the style, so every pair style runs on them exactly
// as on an uploaded NeighList, without the host list copy and its PCIe upload per rebuild.
// Binning and the row builder are the engine's (half-size bins, k_neigh3: count pass, scan,
// fill pass); rows come out in bin order rather than LAMMPS' stencil order, which changes
// only the summation order of the pair sums.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "sph_ctx.h"
#include "sph_dispatch.h"
#include "sph_engine_kernels.h"
#include "sph_util.h"

namespace {
using namespace sph;

constexpr int LB_BLOCKS = 256;  // partial bounding boxes

// per-block bounding boxes of the staged atoms (min x, y, z, max x, y, z), finished on the host
static __global__ void k_bbox_part(int n, const double4 *__restrict__ xf, double *__restrict__ part) {
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double4 x = xf[i];
    lo[0] = fmin(lo[0], x.x);
    lo[1] = fmin(lo[1], x.y);
    lo[2] = fmin(lo[2], x.z);
    hi[0] = fmax(hi[0], x.x);
    hi[1] = fmax(hi[1], x.y);
    hi[2] = fmax(hi[2], x.z);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1)
#pragma unroll
    for (int k = 0; k < 3; k++) {
      lo[k] = fmin(lo[k], __shfl_xor(lo[k], d, 64));
      hi[k] = fmax(hi[k], __shfl_xor(hi[k], d, 64));
    }
  __shared__ double s[4][6];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 3; k++) {
      s[w][k] = lo[k];
      s[w][3 + k] = hi[k];
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    double v = s[0][k];
    for (int q = 1; q < 4; q++) v = k < 3 ? fmin(v, s[q][k]) : fmax(v, s[q][k]);
    part[6 * blockIdx.x + k] = v;
  }
}

// Neighbor::half_from_full_newton (neigh_derive.cpp:83-150) over a full list, G lanes per
// row: the row is read G entries at a time (coalesced), the kept entries keep their order
// (ballot prefix within the lane group).  COUNT: hcnt[i] = kept; FILL: into hnbr from hoff[i]
template <int G, bool FILL>
__global__ __launch_bounds__(256) void k_half_rows(int nlocal, const int *__restrict__ off,
                                                   const int *__restrict__ nbr,
                                                   const double4 *__restrict__ xf,
                                                   int *__restrict__ hcnt,
                                                   const int *__restrict__ hoff,
                                                   int *__restrict__ hnbr) {
  static_assert(64 % G == 0, "lane groups tile the wave");
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t / G, lane = threadIdx.x % G;
  const int gshift = (threadIdx.x & 63) & ~(G - 1);
  const bool live = i < nlocal;
  const int b = live ? off[i] : 0, e = live ? off[i + 1] : 0;
  const double4 xi = live ? xf[i] : make_double4(0, 0, 0, 0);
  int pos = FILL && live ? hoff[i] : 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  // every lane of the wave runs the longest row's trip count (the ballot is wave-wide)
  int len = e - b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) len = max(len, __shfl_xor(len, d, 64));
  for (int k0 = 0; k0 < len; k0 += G) {
    const int k = b + k0 + lane;
    bool keep = false;
    int j = 0;
    if (k < e) {
      j = nbr[k];
      keep = half_keep(i, j, nlocal, xi, xf[j]);
    }
    const unsigned long long m = (__ballot(keep) >> gshift) & ((G == 64) ? ~0ull : ((1ull << G) - 1));
    if (FILL && keep) hnbr[pos + __popcll(m & below)] = j;
    pos += __popcll(m);
  }
  if (!FILL && live && lane == 0) hcnt[i] = pos;
}

static __global__ void k_iota(int n, int *__restrict__ a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = i;
}

// exclusive scan of cnt[0..n) into off[0..n] (off[n] = total), read back; returns total
long long scan_counts(sph_hip_ctx *c, const int *cnt, int n, DBuf<int> &off) {
  off.reserve(n + 1);
  hipLaunchKernelGGL(k_copy_counts, dim3((n + 1 + 255) / 256), dim3(256), 0, c->stream, n, cnt,
                     off.p);
  size_t tb = 0;
  SPH_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, off.p, off.p, n + 1, c->stream));
  c->tmp.reserve(tb);
  SPH_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, tb, off.p, off.p, n + 1, c->stream));
  int tot = 0;
  SPH_HIP_TRY(hipMemcpyAsync(&tot, off.p + n, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  return tot;
}
// identity ilist, and the row offsets on the host too (the reverse half list and fix
// phase_change read them)
void finish_list(sph_hip_ctx *c, int nlocal) {
  hipLaunchKernelGGL(k_iota, dim3((nlocal + 255) / 256), dim3(256), 0, c->stream, nlocal,
                     c->ilist.p);
  SPH_HIP_TRY(hipMemcpyAsync(c->hoff.data(), c->off.p, (nlocal + 1) * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  SPH_HIP_TRY(hipGetLastError());
}

// the active list := Neighbor::half_from_full_newton of the full list (foff, fnbr)
void derive_half(sph_hip_ctx *c, int nlocal, const int *foff, const int *fnbr) {
  constexpr int G = 16;
  const dim3 grid(grid_for_rows(nlocal, G)), block(256);
  c->lcnt.reserve(nlocal + 1);
  hipLaunchKernelGGL((k_half_rows<G, false>), grid, block, 0, c->stream, nlocal, foff, fnbr,
                     (const double4 *)c->xf.p, c->lcnt.p, (const int *)nullptr, (int *)nullptr);
  const long long tot = scan_counts(c, c->lcnt.p, nlocal, c->off);
  c->nbr.reserve(tot > 0 ? tot : 1);
  if (tot)
    hipLaunchKernelGGL((k_half_rows<G, true>), grid, block, 0, c->stream, nlocal, foff, fnbr,
                       (const double4 *)c->xf.p, (int *)nullptr, (const int *)c->off.p, c->nbr.p);
  finish_list(c, nlocal);
}
}  // namespace

extern "C" {

int sph_hip_build_list(sph_hip_ctx *c, int kind, int64_t key, const double *cutneighsq) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && cutneighsq, SPH_HIP_EINVAL, "sph_hip_build_list: NULL argument");
  SPH_REQUIRE(kind == SPH_LIST_FULL || kind == SPH_LIST_HALF, SPH_HIP_EINVAL, "bad list kind");
  SPH_REQUIRE(c->have_atoms, SPH_HIP_EINVAL, "sph_hip_build_list: no atoms staged");
  SPH_HIP_TRY(hipSetDevice(c->device));
  c->select_list(kind);
  const int nlocal = c->nlocal, nall = c->nlocal + c->nghost;
  // a build of this key is already the staged list of this kind (hybrid/overlay sub-styles
  // of one kind share it; the fix's full list is a copy of the pair's)
  const int nt = c->ntypes, n1 = nt + 1;
  SPH_REQUIRE(n1 * n1 <= NT2, SPH_HIP_EINVAL, "sph_hip_build_list: %d types", nt);
  const std::vector<double> cns(cutneighsq, cutneighsq + n1 * n1);
  if (key >= 0 && c->list_key == key && c->inum == nlocal && c->list_devbuilt &&
      c->list_cns == cns)
    return SPH_HIP_OK;
  c->list_key = -1;
  c->list_devbuilt = false;
  // a half list of the key whose full list is parked (built a moment ago for rhosum /
  // colorgradient, as LAMMPS derives both from one build): derived from it, no new binning
  StagedList &pf = c->parked[SPH_LIST_FULL];
  const bool from_parked = kind == SPH_LIST_HALF && key >= 0 && pf.kind == SPH_LIST_FULL &&
                           pf.key == key && pf.devbuilt && pf.inum == nlocal && pf.cns == cns &&
                           nlocal > 0;
  // Neighbor::cutneighsq of the run (neighbor.cpp:261-268), into the coefficient block
  double cmaxsq = 0.0;
  for (int i = 0; i <= nt; i++)
    for (int j = 0; j <= nt; j++) {
      const double v = cutneighsq[i * n1 + j];
      c->hc.cutneighsq[i * n1 + j] = v;
      if (i >= 1 && j >= 1) {
        SPH_REQUIRE(v >= 0.0 && std::isfinite(v), SPH_HIP_EINVAL,
                    "sph_hip_build_list: cutneighsq[%d][%d] = %g", i, j, v);
        cmaxsq = std::max(cmaxsq, v);
      }
    }
  c->coef_dirty = true;
  c->upload_coefs();
  c->ilist.reserve(nlocal > 0 ? nlocal : 1);
  c->off.reserve(nlocal + 1);
  c->hoff.assign(nlocal + 1, 0);
  c->hilist.resize(nlocal);
  for (int i = 0; i < nlocal; i++) c->hilist[i] = i;
  if (from_parked) {
    derive_half(c, nlocal, pf.off.p, pf.nbr.p);
    c->list_kind = kind;
    c->inum = nlocal;
    c->rev_ok = false;
    c->list_key = key;
    c->list_devbuilt = true;
    c->list_cns = cns;
    return SPH_HIP_OK;
  }
  if (nlocal == 0 || nall == 0) {
    SPH_HIP_TRY(hipMemsetAsync(c->off.p, 0, sizeof(int), c->stream));
    SPH_HIP_TRY(hipStreamSynchronize(c->stream));
    c->list_kind = kind;
    c->inum = 0;
    c->rev_ok = false;
    c->list_key = key;
    c->list_devbuilt = true;
    c->list_cns = cns;
    return SPH_HIP_OK;
  }
  const double cm = std::sqrt(cmaxsq);
  SPH_REQUIRE(cm > 0.0, SPH_HIP_EINVAL, "sph_hip_build_list: zero neighbor cutoff");
  // half-size bins (the row builder reaches two bins, i.e. cutneighmax, each way) over the
  // staged atoms' bounding box
  c->lbox.reserve(6 * LB_BLOCKS);
  hipLaunchKernelGGL(k_bbox_part, dim3(LB_BLOCKS), dim3(256), 0, c->stream, nall, c->xf.p,
                     c->lbox.p);
  std::vector<double> hb(6 * LB_BLOCKS);
  SPH_HIP_TRY(hipMemcpyAsync(hb.data(), c->lbox.p, hb.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int b = 0; b < LB_BLOCKS; b++)
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], hb[6 * b + k]);
      hi[k] = std::max(hi[k], hb[6 * b + 3 + k]);
    }
  QBins q{};
  Bins bn{};
  double lk[3], ek[3];
  int nbk[3];
  for (int k = 0; k < 3; k++) {
    const bool act = k < c->dim;
    const double pad = 1e-6 * std::max(1.0, hi[k] - lo[k]);
    lk[k] = lo[k] - pad;
    ek[k] = (hi[k] - lo[k]) + 2 * pad;
    nbk[k] = act ? std::max(1, std::min((int)(ek[k] / (0.5 * cm)), 8192)) : 1;
  }
  // a box that would need more than 2^26 bins (a wide, sparse rank or a stray far-away
  // ghost): coarser bins along the longest axes -- any bin of at least cutneighmax/2 keeps
  // k_neigh3's two-bin reach, so membership is unchanged, only the candidates per bin grow
  auto bins_of = [&]() { return (long long)nbk[0] * nbk[1] * nbk[2]; };
  while (bins_of() >= (1ll << 26)) {
    const int k = (nbk[0] >= nbk[1] && nbk[0] >= nbk[2]) ? 0 : (nbk[1] >= nbk[2] ? 1 : 2);
    nbk[k] = (nbk[k] + 1) / 2;
  }
  const long long nq = bins_of();
  for (int k = 0; k < 3; k++) {
    const bool act = k < c->dim;
    q.lo[k] = bn.lo[k] = lk[k];
    q.nb[k] = bn.nb[k] = nbk[k];
    q.inv[k] = bn.inv[k] = act ? nbk[k] / ek[k] : 0.0;
    q.size[k] = act ? ek[k] / nbk[k] : 1.0;
  }
  q.cutmaxsq = cmaxsq;
  const int nqbins = (int)nq;
  // bin-ordered copy of every staged atom (xb, tb, qbeg)
  c->bkey.reserve(nall);
  c->bkey2.reserve(nall);
  c->bidx.reserve(nall);
  c->bidx2.reserve(nall);
  c->qbeg.reserve(nqbins + 1);
  c->xb.reserve(nall);
  c->tb.reserve(nall);
  hipLaunchKernelGGL(k_bin_keys, dim3((nall + 255) / 256), dim3(256), 0, c->stream, nall, 0, bn,
                     c->xf.p, c->bkey.p, c->bidx.p, 0, 3);
  int endbit = 1;
  while ((1u << endbit) < (unsigned)nqbins && endbit < 32) endbit++;
  size_t tb = 0;
  SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, c->bkey.p, c->bkey2.p, c->bidx.p,
                                                 c->bidx2.p, nall, 0, endbit, c->stream));
  c->tmp.reserve(tb);
  SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(c->tmp.p, tb, c->bkey.p, c->bkey2.p, c->bidx.p,
                                                 c->bidx2.p, nall, 0, endbit, c->stream));
  hipLaunchKernelGGL(k_lower_bound, dim3((nqbins + 1 + 255) / 256), dim3(256), 0, c->stream,
                     nqbins, nall, 0, c->bkey2.p, c->qbeg.p);
  hipLaunchKernelGGL(k_bin_copy, dim3((nall + 255) / 256), dim3(256), 0, c->stream, nall,
                     c->bidx2.p, c->xf.p, c->ty.p, c->xb.p, c->tb.p, (int *)nullptr, 0);
  // the full list: count pass, scan, fill pass (k_neigh3: Neighbor::full_bin membership)
  constexpr int G = 8;
  c->lcnt.reserve(nlocal + 1);
  c->lbad.reserve(1);
  const dim3 grid(grid_for_rows(nlocal, G)), block(256);
  const bool nt1 = nt == 1;
  DBuf<int> &foff = c->loff, &fnbr = c->lnbr;
#define SPH_N3L(F, T, OFF, NBR)                                                                  \
  hipLaunchKernelGGL((k_neigh3<G, 4, F, T>), grid, block, 0, c->stream, nlocal, q, c->dim,        \
                     (const double4 *)c->xf.p, (const int *)c->ty.p, (const double4 *)c->xb.p,    \
                     (const int *)c->tb.p, (const int *)c->qbeg.p, (const Coefs *)c->dc,         \
                     (F ? (int *)nullptr : c->lcnt.p), OFF, NBR, 0, c->lbad.p, 0, 0, 0)
  if (nt1) SPH_N3L(false, true, (const int *)nullptr, (int *)nullptr);
  else SPH_N3L(false, false, (const int *)nullptr, (int *)nullptr);
  const long long ftot = scan_counts(c, c->lcnt.p, nlocal, foff);
  SPH_REQUIRE(ftot >= 0 && ftot < 0x7fffffffll, SPH_HIP_EOVERFLOW,
              "sph_hip_build_list: %lld list entries", ftot);
  fnbr.reserve(ftot > 0 ? ftot : 1);
  if (ftot) {
    if (nt1) SPH_N3L(true, true, (const int *)foff.p, fnbr.p);
    else SPH_N3L(true, false, (const int *)foff.p, fnbr.p);
  }
#undef SPH_N3L
  if (kind == SPH_LIST_FULL) {
    std::swap(c->off, foff);
    std::swap(c->nbr, fnbr);
    finish_list(c, nlocal);
  } else {
    derive_half(c, nlocal, foff.p, fnbr.p);
  }
  c->list_kind = kind;
  c->inum = nlocal;
  c->rev_ok = false;
  c->list_key = key;
  c->list_devbuilt = true;
  c->list_cns = cns;
  SPH_API_END
}

int sph_hip_list_numneigh(sph_hip_ctx *c, int *numneigh) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && numneigh, SPH_HIP_EINVAL, "sph_hip_list_numneigh: NULL argument");
  SPH_REQUIRE(c->list_kind >= 0 && (int)c->hoff.size() >= c->inum + 1, SPH_HIP_EINVAL,
              "sph_hip_list_numneigh: no neighbor list staged");
  for (int r = 0; r < c->inum; r++) numneigh[r] = c->hoff[r + 1] - c->hoff[r];
  SPH_API_END
}

}  // extern "C"
