// sph_pc.h -- fix phase_change (FixPhaseChange::pre_exchange, fix_phase_change.cpp:167-352),
// shared by the pair-style layer (sph_phasechange.hip) and the device-resident engine.
//
// Split by what the work is:
//  * device, parallel over atoms: the candidate test (type == to_type, T = e/cv >= Tc),
//    and for every candidate one walk of its full-list row giving isfromphasearound()
//    (:538-563) and the quintic weights of the from_type donors with their weighted
//    velocity sums (:233-289) -- everything that does not depend on the random stream;
//  * host, sequential over the (few) candidates: the Park-Miller draws (RanPark::uniform,
//    random_park.cpp:42-49), the insertion positions (create_newpos / create_newpos_simple,
//    :466-520) and the sub-domain test (insert_one_atom, :425-456), which must consume the
//    stream exactly in the reference's order;
//  * device again: the mass taken from the donors (dmass[j] += to_mass w_j / W) for the
//    candidates that did change phase: one record per donation, sorted by (donor,
//    candidate) and summed per donor in candidate order -- the reference's summation
//    order, deterministic (k_pc_dmass_emit / k_pc_dmass_sum; pc_dmass_ordered).
//
// The reference's memory behaviour is reproduced: it creates the k-th new atom of a call at
// index nlocal + k (AtomVecMesoMultiPhase::create_atom, atom_vec_meso_multiphase.cpp:968-997),
// i.e. over the ghost in LAMMPS slot k, before that candidate's donor loops.  So a candidate
// met after K insertions no longer sees the ghosts of slots < K (isfromphasearound) or <= K
// (its weights): they now hold to_type atoms; and create_atom zeroes that slot's drho (= the
// fix's dmass, :193), so every donation to a ghost of slot < nins is lost (the reference then
// does not conserve mass).  Each kernel takes the slot rank of a ghost through PcRank; the
// candidate pass reports each candidate's smallest from_type ghost rank, and the replay
// recomputes, on the device, the (rare) candidates whose row meets an overwritten slot.
// (to_type == from_type would turn those slots into donors at the new atoms' positions: not
// supported, an error.)  Tests: tests/test_phasechange_golden.py pins the restatement
// (oracle orc_pre_exchange_ref) to the reference's own FixPhaseChange.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <functional>
#include <stdexcept>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "../../include/sph_hip.h"
#include "sph_mp_kernels.h"
#include "sph_util.h"

namespace sph {

struct PcDev {
  int dim, from_type, to_type;
  double Tc, to_mass, cutoff;
};

constexpr int PC_NORANK = 0x7fffffff;

// LAMMPS slot rank of atom j among the ghosts (owned atoms: none)
struct PcRank {
  int nlocal;
  int mode;           // 0: atoms staged in LAMMPS order (rank = j - nlocal)
                      // 1: screen -- every ghost ranks 0
                      // 2: table grank[j - nlocal]
  const int *grank;
  __device__ __forceinline__ int operator()(int j) const {
    if (j < nlocal) return PC_NORANK;
    if (mode == 0) return j - nlocal;
    if (mode == 1) return 0;
    return grank[j - nlocal];
  }
};

// candidate flags over rows (ilist: row -> atom, nullptr = identity)
static __global__ void k_pc_flags(int inum, const int *__restrict__ ilist,
                                  const int *__restrict__ ty, const double *__restrict__ en,
                                  const double *__restrict__ cv, PcDev p,
                                  int *__restrict__ flag) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= inum) return;
  const int i = ilist ? ilist[r] : r;
  const double Ti = en[i] / cv[i];  // sph_energy2t
  flag[r] = (!(Ti < p.Tc) && ty[i] == p.to_type) ? 1 : 0;
}

__device__ __forceinline__ double pc_w(int dim, double r) {
  return quintic_w(dim, r);  // sph_kernel_quintic{2,3}d(sqrt(rsq)*cutoff), :247-251 (A.6-3)
}

// one record per candidate: {around, W, Sv[3], Svest[3]} over the candidate's list row,
// without the from_type ghosts of slot rank < dead_a (around) / < dead_w (weights); minr
// (nullable) gets the smallest slot rank of the row's from_type atoms.  vel holds v with
// vstride doubles per atom (3: packed xyz, 4: double4)
template <int G>
__global__ void __launch_bounds__(256)
k_pc_candidates(int ncand, const int *__restrict__ cand, const int *__restrict__ ilist,
                const int *__restrict__ off, const int *__restrict__ nbr,
                const double4 *__restrict__ xf, const double4 *__restrict__ vr,
                const double *__restrict__ vel, int vstride, const int *__restrict__ ty,
                const double *__restrict__ rm, PcDev p, double *__restrict__ rec,
                int lstride, const int *__restrict__ lcnt, PcRank rk, int dead_a, int dead_w,
                int *__restrict__ minr) {
  const int k = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (k >= ncand) return;
  const int row = cand[k];
  const int i = ilist ? ilist[row] : row;
  const double4 xi = xf[i];
  const double cut2 = p.cutoff * p.cutoff;
  int around = 0, mr = PC_NORANK;
  double W = 0.0, sv0 = 0.0, sv1 = 0.0, sv2 = 0.0, se0 = 0.0, se1 = 0.0, se2 = 0.0;
  const MpRow rw(off, lcnt, lstride, row);
  for (long long q = rw.beg + lane; q < rw.end; q += G) {
    const int j = nbr[q] & MP_NMASK;
    if (ty[j] != p.from_type) continue;
    const int r = rk(j);
    mr = min(mr, r);
    const double4 xj = xf[j];
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = rsq_ref(dx, dy, dz);
    // (a decision: the reference's rounding)
    if (r >= dead_a && rsq_ref(dx, dy, dz) <= cut2) around = 1;
    if (r >= dead_w && rm[j] > 0.5 * p.to_mass) {
      const double w = pc_w(p.dim, sqrt(rsq) * p.cutoff);
      const double4 vj = vr[j];
      const double *const v = vel + (size_t)vstride * j;
      W += w;
      sv0 += w * v[0];
      sv1 += w * v[1];
      sv2 += w * v[2];
      se0 += w * vj.x;
      se1 += w * vj.y;
      se2 += w * vj.z;
    }
  }
  around = group_sum_i<G>(around);
  mr = group_min_i<G>(mr);
  W = group_sum<G>(W);
  sv0 = group_sum<G>(sv0);
  sv1 = group_sum<G>(sv1);
  sv2 = group_sum<G>(sv2);
  se0 = group_sum<G>(se0);
  se1 = group_sum<G>(se1);
  se2 = group_sum<G>(se2);
  if (lane == 0) {
    double *o = rec + 8 * (size_t)k;
    o[0] = around > 0 ? 1.0 : 0.0;
    o[1] = W;
    o[2] = sv0;
    o[3] = sv1;
    o[4] = sv2;
    o[5] = se0;
    o[6] = se1;
    o[7] = se2;
    if (minr) minr[k] = mr;
  }
}

// dmass[j] += to_mass * w_j / W over the donors of every inserted candidate; the k-th
// inserted candidate's donors exclude the ghosts of slot rank <= k (overwritten before its
// donor loops), and donations to ghosts of slot rank < nins are dropped (create_atom zeroes
// their drho later in the call).  The reference sums dmass[j] over the inserted
// candidates in candidate order (fix_phase_change.cpp:289-299; a donor appears once per
// row).  Every donation becomes a record (key = j << 32 | k, value), the records are sorted
// by key, and each donor's run is summed in order from zero -- the reference's own
// summation order, so dmass is bit-identical to it and to every other run.  `key` and `val`
// hold `cap` records (an upper bound on the donations, e.g. nins x the longest row); unused
// keys stay ~0 and sort last.
template <int G>
__global__ void __launch_bounds__(256)
k_pc_dmass_emit(int nins, const int *__restrict__ rows, const double *__restrict__ Wtot,
                const int *__restrict__ ilist, const int *__restrict__ off,
                const int *__restrict__ nbr, const double4 *__restrict__ xf,
                const int *__restrict__ ty, const double *__restrict__ rm, PcDev p,
                int lstride, const int *__restrict__ lcnt, PcRank rk,
                unsigned long long *__restrict__ key, double *__restrict__ val,
                int *__restrict__ cnt, long long cap) {
  const int k = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (k >= nins) return;
  const int row = rows[k];
  const int i = ilist ? ilist[row] : row;
  const double4 xi = xf[i];
  const double W = Wtot[k];
  const MpRow rw(off, lcnt, lstride, row);
  for (long long q = rw.beg + lane; q < rw.end; q += G) {
    const int j = nbr[q] & MP_NMASK;
    if (ty[j] != p.from_type || !(rm[j] > 0.5 * p.to_mass)) continue;
    const int r = rk(j);
    if (r < nins) continue;  // overwritten before this donor loop (r <= k) or later (r < nins)
    const double4 xj = xf[j];
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = rsq_ref(dx, dy, dz);
    const int slot = atomicAdd(cnt, 1);
    if (slot >= cap) continue;  // (the host checks the count against cap after the launch)
    key[slot] = ((unsigned long long)(unsigned)j << 32) | (unsigned)k;
    val[slot] = p.to_mass * pc_w(p.dim, sqrt(rsq) * p.cutoff) / W;
  }
}
// after the sort: the first record of each donor's run sums the run in candidate order
static __global__ void k_pc_dmass_sum(long long cap, const unsigned long long *__restrict__ key,
                                      const double *__restrict__ val,
                                      double *__restrict__ dmass) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= cap) return;
  const unsigned long long kq = key[q];
  if (kq == ~0ull) return;
  const unsigned j = (unsigned)(kq >> 32);
  if (q > 0 && (unsigned)(key[q - 1] >> 32) == j) return;
  double s = 0.0;
  for (long long t = q; t < cap && key[t] != ~0ull && (unsigned)(key[t] >> 32) == j; t++)
    s += val[t];
  dmass[j] = s;
}

// one swap of a brick's ghosts: key = LAMMPS index of the atom each ghost was copied from
// (owned: lidx; ghost of an earlier swap: nlocal + its slot), val = position in the swap
static __global__ void k_pc_swapkeys(int ns, int first, const int *__restrict__ gsrc,
                                     int nlocal, const int *__restrict__ lidx,
                                     const int *__restrict__ grank, int *__restrict__ key,
                                     int *__restrict__ val) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ns) return;
  const int src = gsrc[first + k];
  key[k] = src < nlocal ? lidx[src] : nlocal + grank[src - nlocal];
  val[k] = k;
}

// after the sort by key: the swap's p-th ghost in LAMMPS order sits in slot first + p
static __global__ void k_pc_swaprank(int ns, int first, const int *__restrict__ val_sorted,
                                     int *__restrict__ grank) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ns) return;
  grank[first + val_sorted[p]] = first + p;
}

// bricks: the key each sent atom carries to the receiving rank -- its place in the order
// CommBrick::borders scanned this rank's atoms (owned in local order, then ghosts in
// LAMMPS slot order); local indices stay below 2^30
static __global__ void k_pc_sendkeys(int n, const int *__restrict__ list, int nlocal,
                                     const int *__restrict__ lidx,
                                     const int *__restrict__ grank, int *__restrict__ key) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];
  key[k] = i < nlocal ? lidx[i] : (1 << 30) + grank[i - nlocal];
}
// ---- LAMMPS' local atom order (lidx: each owned row's index in the reference's arrays) -----
static __global__ void k_lidx_iota(int n, int base, int *__restrict__ lidx) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) lidx[k] = base + k;
}
// out[k] = lidx[list[k]], a value >= nfin renumbered through tab (CommBrick::exchange's hole
// fill: the tail atoms that moved into departed atoms' slots)
static __global__ void k_lidx_take(int n, const int *__restrict__ list,
                                   const int *__restrict__ lidx, int nfin,
                                   const int *__restrict__ tab, int *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int v = lidx[list ? list[k] : k];
  out[k] = (tab && v >= nfin) ? tab[v - nfin] : v;
}
// Atom::sort's bins (atom.cpp:1590-1600): key = bin << 32 | current index, so the sort is
// stable within a bin as the reference's linked lists are
struct SortBins {
  double lo[3], inv[3];
  int nb[3];
};
static __global__ void k_lidx_sortkeys(int n, SortBins b, const double4 *__restrict__ xf,
                                       const int *__restrict__ lidx,
                                       unsigned long long *__restrict__ key,
                                       int *__restrict__ row) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double4 x = xf[i];
  const double c[3] = {x.x, x.y, x.z};
  int ib[3];
  for (int d = 0; d < 3; d++) {
    const double t = (c[d] - b.lo[d]) * b.inv[d];  // static_cast<int>, then MAX 0 / MIN nb-1
    ib[d] = t < 1.0 ? 0 : (t >= (double)b.nb[d] ? b.nb[d] - 1 : (int)t);
  }
  const unsigned long long bin =
      ((unsigned long long)ib[2] * b.nb[1] + ib[1]) * b.nb[0] + ib[0];
  key[i] = (bin << 32) | (unsigned)lidx[i];
  row[i] = i;
}
static __global__ void k_lidx_tagkeys(int n, const int *__restrict__ tag,
                                      unsigned long long *__restrict__ key,
                                      int *__restrict__ row) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = (unsigned)tag[i];
  row[i] = i;
}
static __global__ void k_lidx_rank(int n, const int *__restrict__ row_sorted,
                                   int *__restrict__ lidx) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) lidx[row_sorted[p]] = p;
}

// received keys of one swap -> (key, position) pairs for the sort
static __global__ void k_pc_keys_in(int n, const int *__restrict__ in, int *__restrict__ key,
                                    int *__restrict__ val) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  key[k] = in[k];
  val[k] = k;
}

// The donors' dmass of the nins inserted candidates (rows[k], total weights Wtot[k], in
// candidate order) into dmass (zeroed by the caller), deterministically.  cap: an upper
// bound on the donations (nins x the longest row).  Scratch grows in the given buffers.
template <int G>
inline void pc_dmass_ordered(hipStream_t s, int nins, const int *rows, const double *Wtot,
                             const int *ilist, const int *off, const int *nbr,
                             const double4 *xf, const int *ty, const double *rm, PcDev p,
                             int lstride, const int *lcnt, PcRank rk, long long cap,
                             DBuf<unsigned long long> &k0, DBuf<unsigned long long> &k1,
                             DBuf<double> &v0, DBuf<double> &v1, DBuf<int> &cnt,
                             DBuf<unsigned char> &tmp, double *dmass) {
  if (nins <= 0 || cap <= 0) return;
  SPH_REQUIRE(cap < (1ll << 31), SPH_HIP_EOVERFLOW, "fix phase_change: %lld donations", cap);
  k0.reserve(cap);
  k1.reserve(cap);
  v0.reserve(cap);
  v1.reserve(cap);
  cnt.reserve(1);
  SPH_HIP_TRY(hipMemsetAsync(k0.p, 0xff, cap * sizeof(unsigned long long), s));
  SPH_HIP_TRY(hipMemsetAsync(cnt.p, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_pc_dmass_emit<G>, dim3((unsigned)(((long long)nins * G + 255) / 256)),
                     dim3(256), 0, s, nins, rows, Wtot, ilist, off, nbr, xf, ty, rm, p, lstride,
                     lcnt, rk, k0.p, v0.p, cnt.p, cap);
  // cap is an upper bound by construction; a stale bound must fail loudly, not drop a
  // donor's share (dmass is the reference's to the bit)
  int emitted = 0;
  SPH_HIP_TRY(hipMemcpyAsync(&emitted, cnt.p, sizeof(int), hipMemcpyDeviceToHost, s));
  SPH_HIP_TRY(hipStreamSynchronize(s));
  SPH_REQUIRE(emitted >= 0 && emitted <= cap, SPH_HIP_EOVERFLOW,
              "fix phase_change: %d donations exceed the bound %lld", emitted, cap);
  size_t tb = 0;
  SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0.p, k1.p, v0.p, v1.p, (int)cap,
                                                 0, 64, s));
  tmp.reserve(tb);
  SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k0.p, k1.p, v0.p, v1.p, (int)cap, 0,
                                                 64, s));
  hipLaunchKernelGGL(k_pc_dmass_sum, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, cap,
                     k1.p, v1.p, dmass);
  SPH_HIP_TRY(hipGetLastError());
}

// ---- host side: the random stream, in the reference's order ----------------------------
inline double park_uniform(int &seed) {  // RanPark::uniform, random_park.cpp:42-49
  const int IA = 16807, IM = 2147483647, IQ = 127773, IR = 2836;
  const double AM = 1.0 / IM;
  const int k = seed / IQ;
  seed = IA * (seed - k * IQ) - IR * k;
  if (seed < 0) seed += IM;
  return AM * seed;
}

inline bool pc_owns(const sph_phasechange_params &p, int dim, const double *c) {  // :441-452
  if (c[0] >= p.sublo[0] && c[0] < p.subhi[0] && c[1] >= p.sublo[1] && c[1] < p.subhi[1] &&
      c[2] >= p.sublo[2] && c[2] < p.subhi[2])
    return true;
  if (dim == 3 && c[2] >= p.boxhi[2] && p.top[2] && c[0] >= p.sublo[0] && c[0] < p.subhi[0] &&
      c[1] >= p.sublo[1] && c[1] < p.subhi[1])
    return true;
  if (dim == 2 && c[1] >= p.boxhi[1] && p.top[1] && c[0] >= p.sublo[0] && c[0] < p.subhi[0])
    return true;
  return false;
}

inline void pc_newpos_simple(int &seed, const double *x, double delta, double *c) {  // :466-470
  c[0] = x[0] + (park_uniform(seed) - 0.5) * delta;
  c[1] = x[1] + (park_uniform(seed) - 0.5) * delta;
  c[2] = x[2] + (park_uniform(seed) - 0.5) * delta;
}

inline void pc_newpos(int dim, int &seed, const double *x, const double *cg, double delta,
                      double *c) {  // :472-520, with the reference's b1abs test on b2 (:494)
  const double CG_SMALL = 1.0e-20;
  double eij[3];
  if (dim == 3) {
    double b1[3] = {-cg[1], cg[0], 0.0};
    const double b1abs = std::sqrt(b1[0] * b1[0] + b1[1] * b1[1] + b1[2] * b1[2]);
    if (b1abs > CG_SMALL)
      for (double &b : b1) b = b / b1abs;
    const double den = std::pow(cg[1], 2) + std::pow(cg[0], 2);
    double b2[3] = {-cg[0] * cg[1] * cg[2] / den, -cg[2] * std::pow(cg[1], 2) / den, cg[1]};
    const double b2abs = std::sqrt(b2[0] * b2[0] + b2[1] * b2[1] + b2[2] * b2[2]);
    if (b1abs > CG_SMALL)
      for (double &b : b2) b = b / b2abs;
    const double a = park_uniform(seed) - 0.5;
    const double b = park_uniform(seed) - 0.5;
    for (int d = 0; d < 3; d++) eij[d] = a * b1[d] + b * b2[d];
  } else {
    double a = park_uniform(seed);
    a = (a > 0.5) ? 1.0 : -1.0;
    eij[0] = -a * cg[1];
    eij[1] = a * cg[0];
    eij[2] = 0.0;
  }
  const double eabs = std::sqrt(eij[0] * eij[0] + eij[1] * eij[1] + eij[2] * eij[2]);
  for (int d = 0; d < 3; d++) c[d] = x[d] + eij[d] * delta / eabs;
}

// What the stream needs of one candidate (in the order the reference meets them)
struct PcCand {
  double x[3], cg[3], e, cv, rho;
  double rec[8];  // k_pc_candidates: around, W, Sv[3], Svest[3]
  int minr;       // smallest slot rank of a from_type ghost in its row (PC_NORANK: none)
};

// recompute(k, dead_a, dead_w, rec): candidate k's record without the ghosts of slot rank
// < dead_a (around) / < dead_w (weights); device work, called only for rows that meet a
// slot a created atom has overwritten
using PcRecompute = std::function<void(size_t, int, int, double *)>;

// The candidate loop of pre_exchange (:198-321).  For each candidate that changes phase:
// its index in `c` (ins_k), its donors' total weight (ins_W), its new energy
// e_i = (e_i - Hwv)/2, and the new atom's 13-double record {x[3], v[3], vest[3], e, rmass,
// rho, cv} (ins_rec).
inline void pc_replay(const sph_phasechange_params &p, int dim, int &seed,
                      const std::vector<PcCand> &c, std::vector<int> &ins_k,
                      std::vector<double> &ins_W, std::vector<double> &ins_rec,
                      const PcRecompute &recompute) {
  ins_k.clear();
  ins_W.clear();
  ins_rec.clear();
  int K = 0;  // atoms created so far: they sit in ghost slots 0..K-1
  for (size_t k = 0; k < c.size(); k++) {
    PcCand a = c[k];
    if (a.minr <= K) {  // the row meets slot K (this candidate's own new atom) or an earlier one
      if (p.from_type == p.to_type)
        throw std::runtime_error(
            "fix phase_change with to_type == from_type: a created atom would become a donor "
            "in a later candidate's list (not supported)");
      recompute(k, K, K + 1, a.rec);
    }
    const double Ti = a.e / a.cv;
    const bool around = a.rec[0] != 0.0;
    bool change;
    if (p.energy_chance) {
      const double threshold = (a.e - p.Tc * a.cv) / p.Hwv * p.dt * p.rate;
      change = (park_uniform(seed) < threshold) && around;
    } else {
      change = (park_uniform(seed) < p.change_chance) && (Ti > p.Tt) && around;
    }
    if (!change) continue;
    double coord[3];
    bool ok = false;
    double delta = p.dr;
    int na = 0;
    do {
      pc_newpos(dim, seed, a.x, a.cg, delta, coord);
      ok = pc_owns(p, dim, coord);
      delta = 0.75 * delta;
      na++;
    } while (!ok && na < p.maxattempt);
    if (!ok) {
      delta = p.dr;
      na = 0;
      do {
        pc_newpos_simple(seed, a.x, delta, coord);
        ok = pc_owns(p, dim, coord);
        delta = 0.75 * delta;
        na++;
      } while (!ok && na < p.maxattempt);
    }
    if (!ok) continue;
    const double W = a.rec[1];
    const double energy_aux = 0.5 * (a.e - p.Hwv);  // :317-320
    double o[13];
    o[0] = coord[0];
    o[1] = coord[1];
    o[2] = coord[2];
    for (int d = 0; d < 3; d++) {
      o[3 + d] = (a.rec[2 + d] * p.to_mass / W) / p.to_mass;  // dmom / to_mass (:300-302)
      o[6 + d] = (a.rec[5 + d] * p.to_mass / W) / p.to_mass;  // dmomest / to_mass
    }
    o[9] = energy_aux;
    o[10] = p.to_mass;
    o[11] = a.rho;
    o[12] = a.cv;
    ins_k.push_back((int)k);
    ins_W.push_back(W);
    ins_rec.insert(ins_rec.end(), o, o + 13);
    K++;
  }
}

}  // namespace sph
