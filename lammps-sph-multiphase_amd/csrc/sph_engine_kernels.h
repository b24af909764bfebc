// sph_engine_kernels.h -- streaming kernels of the device-resident step: FixMeso
// integrate, Domain::pbc, CommBrick borders/forward comm on one process, binning, the
// spatial sort, and the binned full-list build (Neighbor::full_bin membership:
// rsq <= cutneighsq, j != i).  Layout as in sph_kernels.h (xf, vr, ty, en).
#pragma once
#include <hip/hip_runtime.h>

#include "sph_kernels.h"
#include "sph_mp2_kernels.h"

namespace sph {

struct StepConst {
  double dtv, dtf;
  double mass[MAXT + 1];
  int stationary_mask;
  // the block path's inner rows (k_blk_inner): positions when they were written, and the
  // flag raised once an atom has moved more than half their margin since (x0 == nullptr:
  // no inner rows)
  const double4 *x0;
  double lim2;
  int *moved;
};

__device__ __forceinline__ void inner_check(const StepConst &sc, int i, const double4 &x) {
  if (!sc.x0) return;
  const double4 a = sc.x0[i];
  const double dx = x.x - a.x, dy = x.y - a.y, dz = x.z - a.z;
  if (dx * dx + dy * dy + dz * dz > sc.lim2) atomicOr(sc.moved, 1);
}

// bricks: the ghosts' positions arrive from other ranks, so their displacement since the
// inner rows were written is checked after each forward comm (one brick: a ghost moves with
// the owned atom it images, which the integrate kernels check)
static __global__ void k_inner_ghosts(int ng, int nlocal, StepConst sc,
                                      const double4 *__restrict__ xf) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  inner_check(sc, nlocal + g, xf[nlocal + g]);
}

// build_direct: (origin rank, ghost) keys for the stable grouping sort; an origin rank out
// of range sorts last as rank P (the group bounds come from k_lower_bound on the sorted keys)
static __global__ void k_dr_keys(int ng, int P, const int *__restrict__ gorank,
                                 unsigned *__restrict__ key, int *__restrict__ val) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  const int r = gorank[g];
  key[g] = (r >= 0 && r < P) ? (unsigned)r : (unsigned)P;
  val[g] = g;
}
// ... and the grouped ghosts' owned indices on their origin ranks and their slots
static __global__ void k_dr_group(int ng, const int *__restrict__ sg,
                                  const int *__restrict__ goidx, int *__restrict__ byq,
                                  int *__restrict__ byg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ng) return;
  const int g = sg[k];
  byq[k] = goidx[g];
  byg[k] = g;
}

// the ghosts' reference positions of the inner rows, taken again when *cond is raised
// (sph_engine refresh_inner, bricks)
static __global__ void k_x0_cond(int ng, const int *__restrict__ cond,
                                 const double4 *__restrict__ xg, double4 *__restrict__ x0g) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng || *cond == 0) return;
  x0g[g] = xg[g];
}

// FixMeso::initial_integrate (fix_meso.cpp:91-140) / FixMesoStationary (:71-90)
static __global__ void k_initial_integrate(int n, StepConst sc, double4 *__restrict__ xf,
                                           double4 *__restrict__ vr, double *__restrict__ en,
                                           const int *__restrict__ ty,
                                           double4 *__restrict__ vel,
                                           const double4 *__restrict__ fo,
                                           const double *__restrict__ de,
                                           const double *__restrict__ rm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ty[i];
  double4 vv = vr[i];       // vest, rho
  const double4 f = fo[i];  // fx, fy, fz, drho
  en[i] += sc.dtf * de[i];
  vv.w += sc.dtf * f.w;
  if (!((sc.stationary_mask >> t) & 1)) {
    double4 x = xf[i];
    double4 v = vel[i];
    const double dtfm = sc.dtf / (rm ? rm[i] : sc.mass[t]);  // rmass if per-atom
    vv.x = v.x + 2.0 * dtfm * f.x;
    vv.y = v.y + 2.0 * dtfm * f.y;
    vv.z = v.z + 2.0 * dtfm * f.z;
    v.x += dtfm * f.x;
    v.y += dtfm * f.y;
    v.z += dtfm * f.z;
    x.x += sc.dtv * v.x;
    x.y += sc.dtv * v.y;
    x.z += sc.dtv * v.z;
    vel[i] = v;
    xf[i] = x;
    inner_check(sc, i, x);
  }
  vr[i] = vv;
}

// FixMeso::final_integrate (fix_meso.cpp:144-180) / FixMesoStationary (:94-112)
static __global__ void k_final_integrate(int n, StepConst sc, double4 *__restrict__ vr,
                                         double *__restrict__ en, const int *__restrict__ ty,
                                         double4 *__restrict__ vel,
                                         const double4 *__restrict__ fo,
                                         const double *__restrict__ de,
                                         const double *__restrict__ rm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ty[i];
  const double4 f = fo[i];
  if (!((sc.stationary_mask >> t) & 1)) {
    double4 v = vel[i];
    const double dtfm = sc.dtf / (rm ? rm[i] : sc.mass[t]);  // rmass if per-atom
    v.x += dtfm * f.x;
    v.y += dtfm * f.y;
    v.z += dtfm * f.z;
    vel[i] = v;
  }
  en[i] += sc.dtf * de[i];
  vr[i].w += sc.dtf * f.w;
}

// FixMeso::final_integrate of one step fused with initial_integrate of the next: nothing
// between them touches these atoms (Verlet::run: output, then the next step's
// initial_integrate, verlet.cpp:295-307, 230), so one streaming pass does both with the
// two kernels' operations in their order (bit-identical results, half the traffic).
static __global__ void k_final_initial(int n, StepConst sc, double4 *__restrict__ xf,
                                       double4 *__restrict__ vr, double *__restrict__ en,
                                       const int *__restrict__ ty, double4 *__restrict__ vel,
                                       const double4 *__restrict__ fo,
                                       const double *__restrict__ de,
                                       const double *__restrict__ rm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ty[i];
  double4 vv = vr[i];
  const double4 f = fo[i];
  const double dei = de[i];
  double e = en[i];
  e += sc.dtf * dei;        // final
  vv.w += sc.dtf * f.w;
  e += sc.dtf * dei;        // initial
  vv.w += sc.dtf * f.w;
  if (!((sc.stationary_mask >> t) & 1)) {
    double4 x = xf[i];
    double4 v = vel[i];
    const double dtfm = sc.dtf / (rm ? rm[i] : sc.mass[t]);  // rmass if per-atom
    v.x += dtfm * f.x;      // final
    v.y += dtfm * f.y;
    v.z += dtfm * f.z;
    vv.x = v.x + 2.0 * dtfm * f.x;   // initial
    vv.y = v.y + 2.0 * dtfm * f.y;
    vv.z = v.z + 2.0 * dtfm * f.z;
    v.x += dtfm * f.x;
    v.y += dtfm * f.y;
    v.z += dtfm * f.z;
    x.x += sc.dtv * v.x;
    x.y += sc.dtv * v.y;
    x.z += sc.dtv * v.z;
    vel[i] = v;
    xf[i] = x;
    inner_check(sc, i, x);
  }
  en[i] = e;
  vr[i] = vv;
}

// FixMeso::setup_pre_force: vest = v (fix_meso.cpp:68-85)
static __global__ void k_vest_from_v(int n, int stationary_mask, const int *__restrict__ ty,
                                     const double4 *__restrict__ vel,
                                     double4 *__restrict__ vr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // meso/stationary has no setup_pre_force: its vest stays as it was
  if ((stationary_mask >> ty[i]) & 1) return;
  const double4 v = vel[i];
  double4 r = vr[i];
  r.x = v.x;
  r.y = v.y;
  r.z = v.z;
  vr[i] = r;
}

struct Box {
  double lo[3], hi[3], prd[3];
  int periodic[3];
};

// image flags, packed as LAMMPS' imageint (lmptype.h SMALLBIG: 10 bits per dimension,
// IMGMAX = 512 = zero image), carried in the owned atoms' vel[i].w (an exact integer)
constexpr int IMG_MASK = 1023, IMG_MAX = 512, IMG_BITS = 10;
constexpr int IMG_ZERO = (IMG_MAX << (2 * IMG_BITS)) | (IMG_MAX << IMG_BITS) | IMG_MAX;

// Domain::pbc (domain.cpp:478-560), orthogonal box: wrap into the box, counting the image
static __global__ void k_pbc(int n, Box b, double4 *__restrict__ xf, double4 *__restrict__ vel) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double4 x = xf[i];
  double c[3] = {x.x, x.y, x.z};
  int img = (int)vel[i].w;
  const int img0 = img;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (!b.periodic[k]) continue;
    const int sh = k * IMG_BITS;
    if (c[k] < b.lo[k]) {
      c[k] += b.prd[k];
      const int idim = (((img >> sh) & IMG_MASK) - 1) & IMG_MASK;
      img = (img & ~(IMG_MASK << sh)) | (idim << sh);
    }
    if (c[k] >= b.hi[k]) {
      c[k] -= b.prd[k];
      c[k] = fmax(c[k], b.lo[k]);
      const int idim = (((img >> sh) & IMG_MASK) + 1) & IMG_MASK;
      img = (img & ~(IMG_MASK << sh)) | (idim << sh);
    }
  }
  x.x = c[0];
  x.y = c[1];
  x.z = c[2];
  xf[i] = x;
  if (img != img0) vel[i].w = (double)img;
}

// ---- borders (one process: the left/right neighbor is this rank itself) -------------
static __global__ void k_slab_flags(int n, int dim, double lo, double hi,
                                    const double4 *__restrict__ xf,
                                    unsigned char *__restrict__ flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double4 x = xf[i];
  const double c = dim == 0 ? x.x : (dim == 1 ? x.y : x.z);
  flag[i] = (c >= lo && c <= hi) ? 1 : 0;
}

// k_slab_flags over [0, *n) of a launch sized for an upper bound (the count on the device)
static __global__ void k_slab_flags_dev(int nmax, const int *__restrict__ n, int dim, double lo,
                                        double hi, const double4 *__restrict__ xf,
                                        unsigned char *__restrict__ flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nmax) return;
  unsigned char f = 0;
  if (i < *n) {
    const double4 x = xf[i];
    const double c = dim == 0 ? x.x : (dim == 1 ? x.y : x.z);
    f = (c >= lo && c <= hi) ? 1 : 0;
  }
  flag[i] = f;
}

// image packed as 3 x 8-bit signed fields
__host__ __device__ __forceinline__ int img_get(int img, int k) {
  return (int)(signed char)((img >> (8 * k)) & 0xff);
}
__host__ __device__ __forceinline__ int img_add(int img, int k, int d) {
  const int v = img_get(img, k) + d;
  return (img & ~(0xff << (8 * k))) | ((v & 0xff) << (8 * k));
}
// a ghost's position from its owner's: + image * prd in each shifted dimension (k_forward's
// arithmetic, shared with the block passes that read a ghost through its owner, BlkGhosts)
__device__ __forceinline__ double4 img_shift(double4 x, int img, const double *prd) {
  const int ix = img_get(img, 0), iy = img_get(img, 1), iz = img_get(img, 2);
  if (ix) x.x = x.x + ix * prd[0];
  if (iy) x.y = x.y + iy * prd[1];
  if (iz) x.z = x.z + iz * prd[2];
  return x;
}

// append the selected atoms as ghosts shifted by `shift` along `dim`
// (comm_brick.cpp:820-860 -> atom_vec_meso.cpp:422-480 pack/unpack_border)
static __global__ void k_append_ghosts(int nsel, const int *__restrict__ sel, int nlocal,
                                       int nall, int dim, int pbc, double shift,
                                       double4 *__restrict__ xf, double4 *__restrict__ vr,
                                       double *__restrict__ en, int *__restrict__ ty,
                                       int *__restrict__ gowner, int *__restrict__ gimg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nsel) return;
  const int s = sel[k];
  const int g = nall + k;
  double4 x = xf[s];
  if (dim == 0) x.x = x.x + shift;
  else if (dim == 1) x.y = x.y + shift;
  else x.z = x.z + shift;
  xf[g] = x;
  vr[g] = vr[s];
  en[g] = en[s];
  ty[g] = ty[s];
  int own, img;
  if (s < nlocal) {
    own = s;
    img = 0;
  } else {
    own = gowner[s - nlocal];
    img = gimg[s - nlocal];
  }
  gowner[g - nlocal] = own;
  gimg[g - nlocal] = img_add(img, dim, pbc);
}

// k_append_ghosts with the swap's counts on the device (no host round trip per swap):
// *nsel atoms sel[] appended at nall = nalls[0]; nalls[1] <- the new nall.  A swap that would
// pass `cap` atoms appends what fits and raises *ovf (the host redoes the borders with more
// room).  Also the swap's sendlist (gsrc, if given) and the multiphase fields (vel, rm, cv,
// cg, if given; atom_vec_meso_multiphase.cpp pack/unpack_border).
static __global__ void k_append_ghosts_dev(
    int gmax, const int *__restrict__ nsel, const int *__restrict__ sel, int nlocal,
    int *__restrict__ nalls, int cap, int dim, int pbc, double shift, double4 *__restrict__ xf,
    double4 *__restrict__ vr, double *__restrict__ en, int *__restrict__ ty,
    int *__restrict__ gowner, int *__restrict__ gimg, int *__restrict__ gsrc,
    double4 *__restrict__ vel, double *__restrict__ rm, double *__restrict__ cv,
    double4 *__restrict__ cg, int *__restrict__ ovf) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int ns = *nsel, nall = nalls[0];
  if (k == 0) {
    nalls[1] = min(nall + ns, cap);
    if (nall + ns > cap) *ovf = 1;
  }
  if (k >= gmax || k >= ns || nall + k >= cap) return;
  const int s = sel[k];
  const int g = nall + k;
  double4 x = xf[s];
  if (dim == 0) x.x = x.x + shift;
  else if (dim == 1) x.y = x.y + shift;
  else x.z = x.z + shift;
  xf[g] = x;
  vr[g] = vr[s];
  en[g] = en[s];
  ty[g] = ty[s];
  int own, img;
  if (s < nlocal) {
    own = s;
    img = 0;
  } else {
    own = gowner[s - nlocal];
    img = gimg[s - nlocal];
  }
  gowner[g - nlocal] = own;
  gimg[g - nlocal] = img_add(img, dim, pbc);
  if (gsrc) gsrc[g - nlocal] = s;
  if (vel) {
    const double4 v = vel[s], c = cg[s];
    vel[g] = make_double4(v.x, v.y, v.z, vel[g].w);
    rm[g] = rm[s];
    cv[g] = cv[s];
    cg[g] = make_double4(c.x, c.y, c.z, 0.0);
  }
}

// ---- one brick's borders, one dimension in three launches ---------------------------------
// CommBrick::borders (comm_brick.cpp:733-800) for the two swaps of a periodic dimension:
// both scan atoms [0, n) (owned + earlier dimensions' ghosts, n = *nalls), the lower swap
// (x_d in [lo0, hi0], shifted +prd) appends its ghosts first, the upper one (x_d in [lo1,
// hi1], -prd) after them, each in scan order.  k_brd_count: per block of BRD_CH atoms the
// two swaps' counts; k_brd_scan (one block): their exclusive prefixes and the new atom
// counts nalls[1] = n + T0, nalls[2] = n + T0 + T1; k_brd_scatter: the ghosts, in scan
// order (a block-wide prefix per swap), as k_append_ghosts_dev writes them.
constexpr int BRD_T = 256, BRD_IT = 4, BRD_CH = BRD_T * BRD_IT, BRD_W = BRD_T / 64;
__device__ __forceinline__ double brd_coord(const double4 &x, int d) {
  return d == 0 ? x.x : (d == 1 ? x.y : x.z);
}
// A block's BRD_CH atoms in BRD_IT rounds of BRD_T consecutive ones (round k: atom
// blockIdx.x * BRD_CH + k * BRD_T + threadIdx.x -- coalesced loads), and each selected
// atom's rank among the block's selected atoms in scan order (round by round, lanes in
// order): per round and wave a ballot, the waves' counts in LDS, one prefix per thread.
struct BrdSel {
  bool f0[BRD_IT], f1[BRD_IT];
  int r0[BRD_IT], r1[BRD_IT];  // ranks within the block (valid where selected)
  int t0, t1;                  // the block's totals
};
__device__ __forceinline__ void brd_select(BrdSel &s, int n, int d, double lo0, double hi0,
                                           double lo1, double hi1,
                                           const double4 *__restrict__ xf) {
  __shared__ int sw0[BRD_IT][BRD_W], sw1[BRD_IT][BRD_W];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int lp0[BRD_IT], lp1[BRD_IT];
#pragma unroll
  for (int k = 0; k < BRD_IT; k++) {
    const int i = blockIdx.x * BRD_CH + k * BRD_T + threadIdx.x;
    bool a = false, b = false;
    if (i < n) {
      const double c = brd_coord(xf[i], d);
      a = c >= lo0 && c <= hi0;
      b = c >= lo1 && c <= hi1;
    }
    s.f0[k] = a;
    s.f1[k] = b;
    const unsigned long long m0 = __ballot(a), m1 = __ballot(b);
    lp0[k] = __popcll(m0 & lt);
    lp1[k] = __popcll(m1 & lt);
    if (lane == 0) {
      sw0[k][w] = __popcll(m0);
      sw1[k][w] = __popcll(m1);
    }
  }
  __syncthreads();
  int acc0 = 0, acc1 = 0;
#pragma unroll
  for (int k = 0; k < BRD_IT; k++)
#pragma unroll
    for (int v = 0; v < BRD_W; v++) {
      if (v == w) {
        s.r0[k] = acc0 + lp0[k];
        s.r1[k] = acc1 + lp1[k];
      }
      acc0 += sw0[k][v];
      acc1 += sw1[k][v];
    }
  s.t0 = acc0;
  s.t1 = acc1;
}
static __global__ void __launch_bounds__(BRD_T)
k_brd_count(const int *__restrict__ nalls, int d, double lo0, double hi0, double lo1, double hi1,
            const double4 *__restrict__ xf, int *__restrict__ bc, int nh = 0) {
  const int n = nalls ? nalls[0] : nh;  // (bricks: the host's count)
  BrdSel s;
  brd_select(s, n, d, lo0, hi0, lo1, hi1, xf);
  if (threadIdx.x == 0) {
    bc[2 * blockIdx.x] = s.t0;
    bc[2 * blockIdx.x + 1] = s.t1;
  }
}
// exclusive prefix of nb (count0, count1) pairs, in place; one block of 1024 threads
static __global__ void __launch_bounds__(1024)
k_brd_scan(int nb, int *__restrict__ bc, int *__restrict__ nalls, int cap, int *__restrict__ ovf,
           int *__restrict__ nsel = nullptr) {
  __shared__ int s0[1024], s1[1024];
  __shared__ int run0, run1;
  if (threadIdx.x == 0) run0 = run1 = 0;
  __syncthreads();
  for (int b0 = 0; b0 < nb; b0 += 1024) {
    const int b = b0 + threadIdx.x;
    const int v0 = b < nb ? bc[2 * b] : 0, v1 = b < nb ? bc[2 * b + 1] : 0;
    s0[threadIdx.x] = v0;
    s1[threadIdx.x] = v1;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele
      const int a0 = threadIdx.x >= o ? s0[threadIdx.x - o] : 0;
      const int a1 = threadIdx.x >= o ? s1[threadIdx.x - o] : 0;
      __syncthreads();
      s0[threadIdx.x] += a0;
      s1[threadIdx.x] += a1;
      __syncthreads();
    }
    if (b < nb) {
      bc[2 * b] = run0 + s0[threadIdx.x] - v0;
      bc[2 * b + 1] = run1 + s1[threadIdx.x] - v1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      run0 += s0[1023];
      run1 += s1[1023];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && nsel) {  // (bricks: the two send counts)
    nsel[0] = run0;
    nsel[1] = run1;
  } else if (threadIdx.x == 0) {
    const long long n = nalls[0], t0 = n + run0, t1 = t0 + run1;
    nalls[1] = (int)min(t0, (long long)cap);
    nalls[2] = (int)min(t1, (long long)cap);
    if (t1 > cap) *ovf = 1;
  }
}
__device__ __forceinline__ void brd_put(int s, int g, int nlocal, int d, int pbc, double shift,
                                        double4 *__restrict__ xf, double4 *__restrict__ vr,
                                        double *__restrict__ en, int *__restrict__ ty,
                                        int *__restrict__ gowner, int *__restrict__ gimg,
                                        int *__restrict__ gsrc, double4 *__restrict__ vel,
                                        double *__restrict__ rm, double *__restrict__ cv,
                                        double4 *__restrict__ cg) {
  double4 x = xf[s];
  if (d == 0) x.x = x.x + shift;
  else if (d == 1) x.y = x.y + shift;
  else x.z = x.z + shift;
  xf[g] = x;
  vr[g] = vr[s];
  en[g] = en[s];
  ty[g] = ty[s];
  int own, img;
  if (s < nlocal) {
    own = s;
    img = 0;
  } else {
    own = gowner[s - nlocal];
    img = gimg[s - nlocal];
  }
  gowner[g - nlocal] = own;
  gimg[g - nlocal] = img_add(img, d, pbc);
  if (gsrc) gsrc[g - nlocal] = s;
  if (vel) {
    const double4 v = vel[s], c = cg[s];
    vel[g] = make_double4(v.x, v.y, v.z, vel[g].w);
    rm[g] = rm[s];
    cv[g] = cv[s];
    cg[g] = make_double4(c.x, c.y, c.z, 0.0);
  }
}
static __global__ void __launch_bounds__(BRD_T)
k_brd_scatter(const int *__restrict__ nalls, const int *__restrict__ bc, int cap, int nlocal,
              int d, double lo0, double hi0, double lo1, double hi1, double prd,
              double4 *__restrict__ xf, double4 *__restrict__ vr, double *__restrict__ en,
              int *__restrict__ ty, int *__restrict__ gowner, int *__restrict__ gimg,
              int *__restrict__ gsrc, double4 *__restrict__ vel, double *__restrict__ rm,
              double *__restrict__ cv, double4 *__restrict__ cg) {
  const int n = nalls[0], t0 = nalls[1];  // (t0 = n + the lower swap's count, capped)
  BrdSel s;
  brd_select(s, n, d, lo0, hi0, lo1, hi1, xf);
  const int b0 = n + bc[2 * blockIdx.x], b1 = t0 + bc[2 * blockIdx.x + 1];
  // (the ghosts are written after every read of this launch's sources: a ghost slot g >= n
  // is never a source, i < n -- brd_select's barrier orders this block's reads before its
  // writes, and other blocks read only atoms below n)
#pragma unroll
  for (int k = 0; k < BRD_IT; k++) {
    const int i = blockIdx.x * BRD_CH + k * BRD_T + threadIdx.x;
    if (s.f0[k]) {
      const int p0 = b0 + s.r0[k];
      if (p0 < cap && p0 < t0)
        brd_put(i, p0, nlocal, d, 1, prd, xf, vr, en, ty, gowner, gimg, gsrc, vel, rm, cv, cg);
    }
    if (s.f1[k]) {
      const int p1 = b1 + s.r1[k];
      if (p1 < cap) brd_put(i, p1, nlocal, d, -1, -prd, xf, vr, en, ty, gowner, gimg, gsrc, vel,
                            rm, cv, cg);
    }
  }
}

// bricks (CommBrick::borders' sendlists, comm_brick.cpp:733-800): the two swaps' send lists
// of a dimension, indices in scan order -- k_brd_count / k_brd_scan (nsel) then this
static __global__ void __launch_bounds__(BRD_T)
k_brd_lists(int n, const int *__restrict__ bc, int d, double lo0, double hi0, double lo1,
            double hi1, const double4 *__restrict__ xf, int *__restrict__ list0,
            int *__restrict__ list1) {
  BrdSel s;
  brd_select(s, n, d, lo0, hi0, lo1, hi1, xf);
  const int b0 = bc[2 * blockIdx.x], b1 = bc[2 * blockIdx.x + 1];
#pragma unroll
  for (int k = 0; k < BRD_IT; k++) {
    const int i = blockIdx.x * BRD_CH + k * BRD_T + threadIdx.x;
    if (s.f0[k]) list0[b0 + s.r0[k]] = i;
    if (s.f1[k]) list1[b1 + s.r1[k]] = i;
  }
}

// forward_comm (atom_vec_meso.cpp:246-288): ghost <- owner (+image*prd on x), vest, rho, e
// (and p/rho^2, carried in xf.w).  One add per coordinate: each hop adds exactly one
// periodic shift to its own coordinate.
static __global__ void k_forward(int nghost, int nlocal, Box b, const int *__restrict__ gowner,
                                 const int *__restrict__ gimg, double4 *__restrict__ xf,
                                 double4 *__restrict__ vr, double *__restrict__ en) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nghost) return;
  const int o = gowner[g], img = gimg[g];
  xf[nlocal + g] = img_shift(xf[o], img, b.prd);
  vr[nlocal + g] = vr[o];
  en[nlocal + g] = en[o];
}

// forward_comm_pair after rhosum (pair_sph_rhosum.cpp:203, 290-313): rho (+ p/rho^2)
static __global__ void k_forward_rho(int nghost, int nlocal, const int *__restrict__ gowner,
                                     double4 *__restrict__ xf, double4 *__restrict__ vr) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nghost) return;
  const int o = gowner[g];
  vr[nlocal + g].w = vr[o].w;
  xf[nlocal + g].w = xf[o].w;
}

// ---- binning ----------------------------------------------------------------------------
struct Bins {
  double lo[3];
  double inv[3];
  int nb[3];
};

__device__ __forceinline__ int bin_coord(double x, double lo, double inv, int nb) {
  int c = (int)floor((x - lo) * inv);
  return c < 0 ? 0 : (c >= nb ? nb - 1 : c);
}

// spread the low 10 bits of v to every third bit (Morton interleave)
__device__ __forceinline__ unsigned spread3(unsigned v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// Hilbert index of cell (x, y[, z]), b bits per axis (Skilling, "Programming the Hilbert
// curve", AIP Conf. Proc. 707, 2004: axes -> transpose, then bit interleave).  Consecutive
// indices are face-adjacent cells, so a run of consecutive atoms in this order is a
// connected, compact region (Morton order jumps at every level boundary).
__device__ __forceinline__ unsigned spread2(unsigned v) {
  v &= 0xffffu;
  v = (v | (v << 8)) & 0x00ff00ffu;
  v = (v | (v << 4)) & 0x0f0f0f0fu;
  v = (v | (v << 2)) & 0x33333333u;
  v = (v | (v << 1)) & 0x55555555u;
  return v;
}
__device__ __forceinline__ unsigned hilbert_key(int dim, unsigned x, unsigned y, unsigned z,
                                                int b) {
  unsigned X[3] = {x, y, z};
  const int n = dim;
  const unsigned M = 1u << (b - 1);
  for (unsigned Q = M; Q > 1; Q >>= 1) {
    const unsigned P = Q - 1;
    for (int i = 0; i < n; i++) {
      if (X[i] & Q) {
        X[0] ^= P;
      } else {
        const unsigned t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  for (int i = 1; i < n; i++) X[i] ^= X[i - 1];
  unsigned t = 0;
  for (unsigned Q = M; Q > 1; Q >>= 1)
    if (X[n - 1] & Q) t ^= Q - 1;
  for (int i = 0; i < n; i++) X[i] ^= t;
  return n == 3 ? (spread3(X[0]) << 2) | (spread3(X[1]) << 1) | spread3(X[2])
                : (spread2(X[0]) << 1) | spread2(X[1]);
}

// Sort keys: linear bin index (x fastest; the staged path needs each x-row of bins
// contiguous), or the bins' Morton code (morton != 0; the CSR path's row order: a run
// of consecutive rows then covers a compact block of space, so the neighbor records a
// wave of rows gathers stay within one XCD's L2).
// morton: 0 = linear bins, 1 = Morton code, > 1 = Hilbert index with (morton - 1) bits
// per axis of dimension `hdim`
static __global__ void k_bin_keys(int n, int first, Bins bn, const double4 *__restrict__ xf,
                                  unsigned *__restrict__ key, int *__restrict__ idx,
                                  int morton = 0, int hdim = 3) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double4 x = xf[first + k];
  const int cx = bin_coord(x.x, bn.lo[0], bn.inv[0], bn.nb[0]);
  const int cy = bin_coord(x.y, bn.lo[1], bn.inv[1], bn.nb[1]);
  const int cz = bin_coord(x.z, bn.lo[2], bn.inv[2], bn.nb[2]);
  if (morton > 1)
    key[k] = hilbert_key(hdim, (unsigned)cx, (unsigned)cy, (unsigned)cz, morton - 1);
  else
    key[k] = morton ? (spread3(cx) | (spread3(cy) << 1) | (spread3(cz) << 2))
                    : (unsigned)((cz * bn.nb[1] + cy) * bn.nb[0] + cx);
  idx[k] = first + k;
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

// permutation gather for the spatial sort of owned atoms (atom->sort analogue)
static __global__ void k_permute(int n, const int *__restrict__ perm,
                                 const double4 *__restrict__ xf, const double4 *__restrict__ vr,
                                 const double *__restrict__ en, const int *__restrict__ ty,
                                 const double4 *__restrict__ vel, const int *__restrict__ tag,
                                 double4 *__restrict__ xf2, double4 *__restrict__ vr2,
                                 double *__restrict__ en2, int *__restrict__ ty2,
                                 double4 *__restrict__ vel2, int *__restrict__ tag2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = perm[i];
  xf2[i] = xf[s];
  vr2[i] = vr[s];
  en2[i] = en[s];
  ty2[i] = ty[s];
  vel2[i] = vel[s];
  tag2[i] = tag[s];
}

// ---- CSR full-list build over a binned copy ----------------------------------------
// Bins here are >= cutneighmax / 2 (reach S = 2 bins).  Every atom, owned or ghost, is
// copied in bin order into xb (x, y, z, atom index as a double) so that a stencil row is
// one contiguous, coalesced range; per (dy, dz) row of bins the x-range is trimmed to the
// bins that can hold a point within cutneighmax of x_i, and rows whose y/z slab distance
// already exceeds it are skipped.  The trimming is conservative (slab distances shrunk
// by a margin) -- membership itself is decided only by rsq <= cutneighsq[it][jt] in
// fp64, exactly as Neighbor::full_bin (neigh_full.cpp:241-344).
struct QBins {
  double lo[3], inv[3], size[3];
  int nb[3];
  double cutmaxsq;
};

// (xpos, if given: the inverse, atom -> position in xb)
// (tpack: .w = j | (type - 1) << 28 -- the multiphase engine's list entry itself, so its
// builds need no type gather; nall < MP_MAXALL there)
static __global__ void k_bin_copy(int n, const int *__restrict__ perm,
                                  const double4 *__restrict__ xf, const int *__restrict__ ty,
                                  double4 *__restrict__ xb, int *__restrict__ tb,
                                  int *__restrict__ xpos = nullptr, int tpack = 0) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int j = perm[p];
  const double4 x = xf[j];
  xb[p] = make_double4(x.x, x.y, x.z, (double)(tpack ? j | ((ty[j] - 1) << 28) : j));
  tb[p] = ty[j];
  if (xpos) xpos[j] = p;
}

// distance from coordinate v to bin b's slab along one axis (0 inside), shrunk by a margin
__device__ __forceinline__ double slab_gap(double v, int b, int c, double lo, double size) {
  if (b == c) return 0.0;
  const double edge = (b < c) ? lo + (b + 1) * size : lo + b * size;
  const double g = (b < c) ? v - edge : edge - v;
  return fmax(g - 1e-6 * size, 0.0);
}

// ---- full-list build v3: flattened candidate ranges ---------------------------------------
// Half-size bins (reach 2) with per-row trimming: a row's <= 25 (dz, dy) bin-rows are cut
// to the x-range that can hold a point within cutneighmax.  The row's G lanes first resolve
// all bin-row ranges at once (independent loads, into LDS), then walk the concatenated
// candidates as ONE flat range in chunks of G*U -- each chunk one round of independent
// record loads.  Hits are compacted in candidate order.  Modes: count | CSR fill | strided
// fill (fixed-stride rows, the row's count in cnt, a row longer than stride raises *ovf);
// perm_g > 0 stores a strided row chunk-transposed (tpos, stride a multiple of 4*perm_g).
// the half list's owner of pair (i, j) (half_from_full_newton, neigh_derive.cpp:83-150):
// an owned j if i < j, a ghost j if it lies above i in z, then y, then x
__device__ __forceinline__ bool half_keep(int i, int j, int nlocal, const double4 &xi,
                                          const double4 &xj) {
  if (j < nlocal) return i < j;
  if (xj.z < xi.z) return false;
  if (xj.z == xi.z) {
    if (xj.y < xi.y) return false;
    if (xj.y == xi.y && xj.x < xi.x) return false;
  }
  return true;
}

// RHO (fill passes of the multiphase engine, the list built in the step whose forces follow,
// skin 0 as bubble.lmp): rhosum/multiphase (pair_sph_rhosum_multiphase.cpp:118-167) summed
// over the row's hits as they are found -- the pair set and positions k_mp2_rhosum would walk
// right after -- into rho (owned rows; rm = rmass); the separate rhosum pass is then skipped
template <int G, int U, bool FILL, bool NT1, bool RHO = false, bool TP = false>
__global__ void __launch_bounds__(256)
k_neigh3(int nlocal, QBins q, int dim, const double4 *__restrict__ xf,
         const int *__restrict__ ty, const double4 *__restrict__ xb,
         const int *__restrict__ tb, const int *__restrict__ beg,
         const Coefs *__restrict__ cf, int *__restrict__ cnt, const int *__restrict__ off,
         int *__restrict__ nbr, int stride, int *__restrict__ ovf, int perm_g, int perm_pi,
         int tbits, const MpCoefs *__restrict__ mc = nullptr,
         const double *__restrict__ rm = nullptr, double *__restrict__ rho = nullptr) {
  constexpr int R = 2, NB = (2 * R + 1) * (2 * R + 1), GR = 256 / G, KB = (NB + G - 1) / G;
  static_assert(!RHO || FILL, "the rhosum terms ride on the fill passes");
  __shared__ double s_cns[NT2];
  __shared__ double s_rcs[RHO ? NT2 : 1], s_rih[RHO ? NT2 : 1], s_rwn[RHO ? NT2 : 1];
  __shared__ double s_hr[RHO ? GR : 1][RHO ? G * U : 1];  // a chunk's hits: rsq
  __shared__ int s_hp[RHO ? GR : 1][RHO ? G * U : 1];     //   and pair type
  __shared__ int s_rs[GR][NB];       // first candidate (position in xb) of each bin-row
  __shared__ int s_pre[GR][NB + 1];  // candidates before each bin-row (flat numbering)
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_cns[t] = cf->cutneighsq[t];
  if (RHO)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
      s_rcs[t] = mc->rcutsq[t];
      s_rih[t] = mc->rcut_inv[t];
      s_rwn[t] = mp2_wnorm(dim, mc->rcut_inv[t]);
    }
  const int i = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1), grp = threadIdx.x / G;
  const bool live = i < nlocal;
  const double4 xi = xf[live ? i : 0];
  const int cx = bin_coord(xi.x, q.lo[0], q.inv[0], q.nb[0]);
  const int cy = bin_coord(xi.y, q.lo[1], q.inv[1], q.nb[1]);
  const int cz = bin_coord(xi.z, q.lo[2], q.inv[2], q.nb[2]);
  const int nbr_rows = (dim == 3) ? NB : (2 * R + 1);
  // 1) this lane's bin-rows br = lane + k*G, in (bz, by) loop order
#pragma unroll
  for (int k = 0; k < KB; k++) {
    const int br = lane + k * G;
    if (br >= NB) break;
    int start = 0, len = 0;
    if (live && br < nbr_rows) {
      const int bz = (dim == 3) ? cz - R + br / (2 * R + 1) : cz;
      const int by = cy - R + br % (2 * R + 1);
      if (bz >= 0 && bz < q.nb[2] && by >= 0 && by < q.nb[1]) {
        const double gz = (dim == 3) ? slab_gap(xi.z, bz, cz, q.lo[2], q.size[2]) : 0.0;
        const double gy = slab_gap(xi.y, by, cy, q.lo[1], q.size[1]);
        const double d2 = gy * gy + gz * gz;
        if (d2 <= q.cutmaxsq) {
          const double ext = sqrt(q.cutmaxsq - d2) * (1.0 + 1e-9) + 1e-9 * q.size[0];
          const int bx0 = bin_coord(xi.x - ext, q.lo[0], q.inv[0], q.nb[0]);
          const int bx1 = bin_coord(xi.x + ext, q.lo[0], q.inv[0], q.nb[0]);
          const int brow = (bz * q.nb[1] + by) * q.nb[0];
          start = beg[brow + bx0];
          len = beg[brow + bx1 + 1] - start;
        }
      }
    }
    s_rs[grp][br] = start;
    s_pre[grp][br + 1] = len;
  }
  __syncthreads();
  if (lane == 0) {  // serial prefix over the row's <= 25 bin-rows
    int acc = 0;
    s_pre[grp][0] = 0;
    for (int br = 0; br < NB; br++) {
      acc += s_pre[grp][br + 1];
      s_pre[grp][br + 1] = acc;
    }
  }
  __syncthreads();
  if (!live) return;
  const int T = s_pre[grp][NB];
  const double *crow = s_cns + (NT1 ? 0 : ty[i] * nt1);
  const double cns1 = NT1 ? cf->cutneighsq[3] : 0.0;
  // (TP: xb.w packs the type, k_bin_copy tpack)
  const double di = TP ? (double)(i | ((NT1 ? 0 : ty[i] - 1) << 28)) : (double)i;
  const int rrow = RHO ? (NT1 ? 1 : ty[i]) * nt1 : 0;
  double racc = 0.0;
  int n = 0;
  int *const row = FILL ? nbr + (stride > 0 ? (size_t)i * stride : (size_t)off[i]) : nullptr;
  const int cap = stride > 0 ? stride : 0x7fffffff;
  int pos = 0;
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
  int ptr = 0;  // bin-row holding this lane's next candidate (monotone)
  for (int p0 = 0; p0 < T; p0 += G * U) {  // group-uniform trip count
    const int pos0 = pos;
    double4 xj[U];
    int tj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int pp = min(p0 + lane + u * G, T - 1);
      while (pp >= s_pre[grp][ptr + 1]) ptr++;
      const int p = s_rs[grp][ptr] + (pp - s_pre[grp][ptr]);
      xj[u] = xb[p];
      tj[u] = NT1 ? 1 : TP ? ((int)xj[u].w >> 28) + 1 : tb[p];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double rsq = rsq_ref(xi.x - xj[u].x, xi.y - xj[u].y, xi.z - xj[u].z);
      const bool hit = (p0 + lane + u * G < T) && (xj[u].w != di) &&
                       rsq <= (NT1 ? cns1 : crow[tj[u]]);
      if (FILL) {
        const unsigned long long m = (__ballot(hit) >> gbase) & gmask;
        const int qq = pos + __popcll(m & ((1ull << lane) - 1ull));
        if (RHO && hit) {  // the chunk's hits, compacted, for the rhosum terms below
          s_hr[grp][qq - pos0] = rsq;
          s_hp[grp][qq - pos0] = rrow + tj[u];
        }
        // tbits 1 (strided rows, several types): the neighbour's type rides in the entry's
        // bits 28-30 (SPH_TBIT_SHIFT), so the pair passes need no type gather; tbits 2 (the
        // multiphase engine's rows): bit 31 = the pair is i's in the half list
        // (k_mp_gather), frozen at this build as the reference's half list is, and the
        // type - 1 in bits 28-30 (MP_NMASK)
        if (hit && qq < cap) {
          const int j = (int)xj[u].w & (TP ? MP_NMASK : 0x7fffffff);
          int ent = j;
          if (tbits == 1) ent |= (tj[u] - 1) << SPH_TBIT_SHIFT;
          if (tbits == 2) {  // (+ the type, MpArgs::typed)
            ent |= (tj[u] - 1) << 28;
            if (half_keep(i, j, nlocal, xi, xj[u])) ent |= (int)0x80000000u;
          }
          row[perm_g > 0 ? tpos(qq, perm_g, perm_pi) : qq] = ent;
        }
        pos += __popcll(m);
      } else {
        n += hit ? 1 : 0;
      }
    }
    if (RHO) {  // (k_mp2_rhosum's term) over the chunk's hits only: G lanes, <= G*U hits
      __builtin_amdgcn_wave_barrier();
      for (int k = lane; k < pos - pos0; k += G) {
        const double rsq = s_hr[grp][k];
        const int pt = s_hp[grp][k];
        const double w = qr_wpoly(3.0 * (cr_sqrt(rsq + 1e-300) * s_rih[pt])) * s_rwn[pt];
        racc += rsq < s_rcs[pt] ? w : 0.0;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (!FILL) {
    n = group_sum_i<G>(n);
    if (lane == 0) cnt[i] = n;
  } else if (stride > 0 && lane == 0) {
    cnt[i] = pos;
    if (pos > stride) atomicOr(ovf, 1);
  }
  if (RHO) {
    racc = group_sum<G>(racc);
    if (lane == 0) {
      const int pt = rrow + (NT1 ? 1 : ty[i]);
      rho[i] = (qr_wpoly(0.0) * s_rwn[pt] + racc) * rm[i];
    }
  }
}

static __global__ void k_copy_counts(int n, const int *__restrict__ cnt, int *__restrict__ off) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) off[i] = cnt[i];
  if (i == n) off[i] = 0;
}

// fixed-stride rows (row i at i*stride, cnt[i] entries) -> CSR rows at off[i]; 32 lanes a
// row (128-B runs per access)
static __global__ void k_compact_rows(int n, int stride, const int *__restrict__ cnt,
                                      const int *__restrict__ off, const int *__restrict__ src,
                                      int *__restrict__ dst) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(t >> 5), lane = (int)(t & 31);
  if (i >= n) return;
  const int c = cnt[i], o = off[i];
  const int *const r = src + (size_t)i * stride;
  for (int k = lane; k < c; k += 32) dst[o + k] = __builtin_nontemporal_load(r + k);
}

// ---- setup-step forces with the reference's half-list ownership --------------------------
// On the first run after atoms are created, ghosts carry the vest they had at borders()
// (zero for new atoms) while owned atoms already have vest = v (Verlet::setup calls
// borders before FixMeso::setup_pre_force).  The reference then evaluates each
// owned-ghost pair once, from the side that owns it in the half list
// (neigh_derive.cpp:124-131), and reverse-communicates the ghost's share.  The engine
// reproduces that exactly for the setup step: derive the half list from the full one,
// walk it with Newton-3 scatter, then fold ghost sums into their owners.

template <bool FILL>
static __global__ void k_half_from_full(int nlocal, const int *__restrict__ off,
                                        const int *__restrict__ nbr,
                                        const double4 *__restrict__ xf, int *__restrict__ hcnt,
                                        const int *__restrict__ hoff, int *__restrict__ hnbr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nlocal) return;
  const double4 xi = xf[i];
  int n = 0;
  int pos = FILL ? hoff[i] : 0;
  for (int k = off[i]; k < off[i + 1]; k++) {
    const int j = nbr[k];
    if (half_keep(i, j, nlocal, xi, xf[j])) {
      if (FILL) hnbr[pos++] = j;
      n++;
    }
  }
  if (!FILL) hcnt[i] = n;
}

// comm->reverse_comm (atom_vec_meso.cpp:387-418): owner += ghost (f, drho, de)
static __global__ void k_reverse(int nghost, int nlocal, const int *__restrict__ gowner,
                                 double4 *__restrict__ fo, double *__restrict__ de) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nghost) return;
  const int o = gowner[g];
  const double4 f = fo[nlocal + g];
  atomicAdd(&fo[o].x, f.x);
  atomicAdd(&fo[o].y, f.y);
  atomicAdd(&fo[o].z, f.z);
  atomicAdd(&fo[o].w, f.w);
  atomicAdd(&de[o], de[nlocal + g]);
}

// fix gravity post_force body force (fix_gravity.cpp post_force): f += m g for the owned
// atoms of the fix's group (gmask: bit t = type t in the group; 0 = all)
static __global__ void k_add_gravity(int n, StepConst sc, double gx, double gy, double gz,
                                     int gmask, const int *__restrict__ ty,
                                     double4 *__restrict__ fo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ty[i];
  if (gmask != 0 && !((gmask >> t) & 1)) return;
  const double m = sc.mass[t];
  fo[i].x += m * gx;
  fo[i].y += m * gy;
  fo[i].z += m * gz;
}

// Rows whose list holds a ghost (index >= nlocal): bd[i] = 1, in[i] = !bd[i].  One
// 64-lane wave per 8 rows (8 lanes per row walk its entries); strided rows stored
// chunk-transposed (perm_g > 0) are read through tpos.  Interior rows (no ghost) can run
// their pair passes while a halo exchange is in flight.
static __global__ void __launch_bounds__(256)
k_row_ghost_flags(int n, int nlocal, const int *__restrict__ off, int stride,
                  const int *__restrict__ rcnt, const int *__restrict__ nbr, int perm_g,
                  int perm_pi, int tbits, unsigned char *__restrict__ in,
                  unsigned char *__restrict__ bd) {
  constexpr int G = 8;
  const int i = (int)((blockIdx.x * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  const bool live = i < n;
  int beg = 0, cnt = 0;
  if (live) {
    beg = stride > 0 ? i * stride : off[i];
    cnt = stride > 0 ? rcnt[i] : off[i + 1] - beg;
  }
  bool ghost = false;
  for (int e = lane; e < cnt; e += G) {
    const int q = (stride > 0 && perm_g > 0) ? tpos(e, perm_g, perm_pi) : e;
    const int j = nbr[beg + q];
    ghost |= (tbits ? (j & SPH_TBIT_MASK) : j) >= nlocal;
  }
  const unsigned long long m = __ballot(ghost);
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  const bool any = ((m >> gbase) & 0xffull) != 0;
  if (live && lane == 0) {
    bd[i] = any ? 1 : 0;
    in[i] = any ? 0 : 1;
  }
}

}  // namespace sph
