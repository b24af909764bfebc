// sph_cluster_kernels.h -- cluster-pair passes of the engine (kernel_path 3).
//
// Why: the row passes (sph_row2_kernels.h) are bound by the texture addresser (TA), whose
// cost is ~2.25 cycles per distinct 128-B line a 64-lane load touches.  A row pass gives
// each row its own lanes, so one load instruction touches the records of 8 different
// rows' neighbours (~14 lines).  Here the lanes of a wave work on ONE cluster of CI
// consecutive (Morton-ordered, so spatially compact) owned atoms and share their
// neighbours: lane = slot * CI + il pairs cluster atom il with the slot-th neighbour of
// the current batch of J = 64 / CI, so the CI lanes of a slot load the same record and a
// load instruction touches J records of consecutive list entries (mostly consecutive
// atoms: 3-5 lines instead of ~14).
//
// Each pair is evaluated ONCE (Newton's third law, as the reference's half list):
//  * the list of cluster c holds every atom within cutneigh of at least one of its atoms
//    that is a ghost, or owned and in a cluster >= c (inside cluster c only the pairs
//    il < jl are taken);
//  * contributions to j are summed over the slot's CI lanes with DPP and added with fp64
//    hardware atomics (one atomic lane per output component); contributions to i are
//    kept per lane, summed over the slots at the end and added the same way;
//  * a ghost j gets nothing: the brick that owns it evaluates the mirrored pair with this
//    atom's image as its ghost (so no reverse communication).
// So the pass evaluates the ~N_half pairs instead of the full list's 2 N_half, at the
// price of a looser list (union of CI spheres) and of the j-side sums.  Summation order
// differs from the reference (and between runs: atomics); the parity bar is relative
// 1e-10, not bit equality.
#pragma once
#include <hip/hip_runtime.h>

#include "sph_engine_kernels.h"
#include "sph_row2_kernels.h"

namespace sph {

// value of lane (ctrl-permuted) for a double, classic DPP on both halves
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
  return u2d((unsigned)lo, (unsigned)hi);
}
// sum over the CI consecutive lanes of a slot (CI = 4 or 8); every lane gets the same sum
template <int CI>
__device__ __forceinline__ double slot_sum(double v) {
  static_assert(CI == 4 || CI == 8, "cluster size");
  v += dpp_d<0xB1>(v);                // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);                // quad_perm [2,3,0,1]
  if (CI == 8) v += dpp_d<0x141>(v);  // row_half_mirror: quad 0 <-> quad 1 of the 8
  return v;
}
// sum over the slots of one cluster atom (lanes il, il + CI, ..., il + 64 - CI)
template <int CI>
__device__ __forceinline__ double atom_sum(double v) {
#pragma unroll
  for (int m = CI; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ---- cluster list build ------------------------------------------------------------------
// One wave per cluster.  Candidates are the binned atoms of the bin-rows (runs of bins along
// x, contiguous in xb) within cutneighmax of the cluster's bounding box, resolved 64 rows
// at a time; a candidate is kept if rsq <= cutneighsq[it][jt] for at least one cluster
// atom (the reference's criterion, npair_full_bin_atomonly.cpp) and it passes the
// ownership rule above.  Kept entries are compacted in candidate order (bin order:
// consecutive entries are mostly consecutive atoms).  nbr == nullptr: count only.
// Rows are fixed-stride (cluster c at c*stride); a row longer than stride keeps its first
// stride entries and raises *ovf.
template <int CI, bool HALF, bool NT1>
__global__ void __launch_bounds__(256)
k_cl_neigh(int nlocal, QBins q, int dim, const double4 *__restrict__ xf,
           const int *__restrict__ ty, const double4 *__restrict__ xb,
           const int *__restrict__ tb, const int *__restrict__ beg,
           const Coefs *__restrict__ cf, int *__restrict__ cnt, int *__restrict__ nbr,
           int stride, int *__restrict__ ovf) {
  __shared__ double s_cns[NT2];
  __shared__ int s_rs[4][64];
  __shared__ int s_pre[4][65];
  const int nt1 = cf->ntypes + 1;
  if (!NT1)
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_cns[t] = cf->cutneighsq[t];
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = wave_uniform((int)((xcd_block() * blockDim.x + threadIdx.x) >> 6));
  const int i0 = c * CI;
  if (i0 >= nlocal) return;  // wave-uniform
  const int nci = min(CI, nlocal - i0);
  double3 xi[CI];
  int ti[CI];
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
#pragma unroll
  for (int k = 0; k < CI; k++) {
    const double4 p = xf[i0 + (k < nci ? k : 0)];
    xi[k] = make_double3(p.x, p.y, p.z);
    ti[k] = NT1 ? 1 : ty[i0 + (k < nci ? k : 0)];
    lo[0] = fmin(lo[0], p.x); hi[0] = fmax(hi[0], p.x);
    lo[1] = fmin(lo[1], p.y); hi[1] = fmax(hi[1], p.y);
    lo[2] = fmin(lo[2], p.z); hi[2] = fmax(hi[2], p.z);
  }
  const double cut = sqrt(q.cutmaxsq) * (1.0 + 1e-9);
  const int by0 = bin_coord(lo[1] - cut, q.lo[1], q.inv[1], q.nb[1]);
  const int by1 = bin_coord(hi[1] + cut, q.lo[1], q.inv[1], q.nb[1]);
  const int bz0 = dim == 3 ? bin_coord(lo[2] - cut, q.lo[2], q.inv[2], q.nb[2]) : 0;
  const int bz1 = dim == 3 ? bin_coord(hi[2] + cut, q.lo[2], q.inv[2], q.nb[2]) : 0;
  const int nyr = by1 - by0 + 1, nrows = nyr * (bz1 - bz0 + 1);
  const double cns1 = NT1 ? cf->cutneighsq[3] : 0.0;
  int *const row = nbr ? nbr + (size_t)c * stride : nullptr;
  const unsigned long long below = (1ull << lane) - 1ull;
  int pos = 0;
  for (int r0 = 0; r0 < nrows; r0 += 64) {
    // 1) the length of bin-row r0 + lane, trimmed to the bbox's reach in x
    int start = 0, len = 0;
    const int r = r0 + lane;
    if (r < nrows) {
      const int by = by0 + r % nyr, bz = bz0 + r / nyr;
      const double yl = q.lo[1] + by * q.size[1], yh = yl + q.size[1];
      double gy = fmax(fmax(yl - hi[1], lo[1] - yh), 0.0);
      double gz = 0.0;
      if (dim == 3) {
        const double zl = q.lo[2] + bz * q.size[2], zh = zl + q.size[2];
        gz = fmax(fmax(zl - hi[2], lo[2] - zh), 0.0);
      }
      gy = fmax(gy - 1e-6 * q.size[1], 0.0);
      gz = fmax(gz - 1e-6 * q.size[2], 0.0);
      const double d2 = gy * gy + gz * gz;
      if (d2 <= q.cutmaxsq) {
        const double ext = sqrt(q.cutmaxsq - d2) * (1.0 + 1e-9) + 1e-9 * q.size[0];
        const int bx0 = bin_coord(lo[0] - ext, q.lo[0], q.inv[0], q.nb[0]);
        const int bx1 = bin_coord(hi[0] + ext, q.lo[0], q.inv[0], q.nb[0]);
        const int brow = (bz * q.nb[1] + by) * q.nb[0];
        start = beg[brow + bx0];
        len = beg[brow + bx1 + 1] - start;
      }
    }
    // 2) inclusive scan of the lengths across the wave
    int inc = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(inc, d, 64);
      if (lane >= d) inc += t;
    }
    s_rs[w][lane] = start;
    s_pre[w][lane + 1] = inc;
    if (lane == 0) s_pre[w][0] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int T = wave_uniform(__shfl(inc, 63, 64));
    // 3) the flat candidate range, 64 at a time
    int ptr = 0;
    for (int p0 = 0; p0 < T; p0 += 64) {
      const int pp = min(p0 + lane, T - 1);
      while (pp >= s_pre[w][ptr + 1]) ptr++;
      const int p = s_rs[w][ptr] + (pp - s_pre[w][ptr]);
      const double4 xj = xb[p];
      const int tj = NT1 ? 1 : tb[p];
      const int j = (int)xj.w;
      bool near = false;
#pragma unroll
      for (int k = 0; k < CI; k++) {
        const double dx = xi[k].x - xj.x, dy = xi[k].y - xj.y, dz = xi[k].z - xj.z;
        const double rsq = dx * dx + dy * dy + dz * dz;
        near |= rsq <= (NT1 ? cns1 : s_cns[ti[k] * nt1 + tj]);
      }
      const bool hit = (p0 + lane < T) && near && (!HALF || j >= nlocal || j >= i0);
      const unsigned long long m = __ballot(hit);
      if (row) {
        const int qq = pos + __popcll(m & below);
        if (hit && qq < stride) row[qq] = j;
      }
      pos += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();  // s_rs/s_pre are rewritten by the next round
  }
  if (lane == 0) {
    cnt[c] = pos;
    if (row && pos > stride) atomicOr(ovf, 1);
  }
}

// ---- pair passes -------------------------------------------------------------------------
struct ClArgs {
  int n, nall, ntot, stride;  // owned atoms, owned + ghosts, list extent, row stride
  const int *cnt, *nbr;       // cluster rows
  double4 *xf, *vr;
  const int *ty;
  const double *en;
  const Coefs *cf;
  double4 *fo;  // {f, drho}: zeroed, then accumulated with atomics
  double *de;
  double *racc;  // rhosum accumulator (zeroed)
  double gx, gy, gz;
  int exp;  // study variants (SPH_CLX bits): 1 = no j-side atomics, 2 = no j-side sums
};

// sph/rhosum (pair_sph_rhosum.cpp:80-160): racc[i] += sum_j m_j W_ij over the clusters;
// the self term and the EOS epilogue are k_cl_rho_final.
template <int CI, bool HALF, bool NT1>
__global__ void __launch_bounds__(256) k_cl_rhosum(ClArgs a) {
  constexpr int J = 64 / CI;
  __shared__ RhoPair s_c[NT1 ? 1 : NT2];
  const Coefs *cf = a.cf;
  const int nt1 = cf->ntypes + 1;
  if (!NT1) {
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) s_c[t] = cf->rho[t];
    __syncthreads();
  }
  const int c = wave_uniform((int)((xcd_block() * blockDim.x + threadIdx.x) >> 6));
  const int i0 = c * CI;
  if (i0 >= a.n) return;  // wave-uniform
  const int lane = threadIdx.x & 63, il = lane & (CI - 1), sl = lane / CI;
  const int i = i0 + il;
  const bool ilive = i < a.n;
  const Rsrc rn = make_rsrc(a.nbr, nbytes<int>(a.ntot));
  const Rsrc rx = make_rsrc(a.xf, nbytes<double4>(a.nall));
  const Rsrc rt = make_rsrc(a.ty, nbytes<int>(a.nall));
  const double4 xi = a.xf[ilive ? i : i0];
  const int it = NT1 ? 1 : a.ty[ilive ? i : i0];
  const RhoPair c1 = NT1 ? cf->rho[3] : RhoPair{};
  const int beg = c * a.stride, end = beg + a.cnt[c];
  double acc = 0.0;
  int jn = ld_i32(rn, (unsigned)(beg + sl) * 4u);
  for (int k0 = beg; k0 < end; k0 += J) {  // wave-uniform trip count
    const int j = jn;
    const bool valid = k0 + sl < end;
    const double3 xj = ld_d3(rx, (unsigned)j * 32u);
    const int tj = NT1 ? 1 : ld_i32(rt, (unsigned)j * 4u);
    jn = ld_i32(rn, (unsigned)(k0 + J + sl) * 4u);
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    const RhoPair cc = NT1 ? c1 : s_c[it * nt1 + tj];
    double wf = 1.0 - rsq * cc.ihsq;
    wf = wf * wf;
    wf = wf * wf;
    const unsigned jl = (unsigned)(j - i0);
    const bool pair = HALF ? (jl >= (unsigned)CI || (unsigned)il < jl) : jl != (unsigned)il;
    const bool in = valid && ilive && rsq < cc.cutsq && pair;
    const double wv = in ? wf : 0.0;
    acc += cc.mK * wv;
    if (!HALF) continue;
    const unsigned long long bm = __ballot(in);
    const bool any = ((bm >> (sl * CI)) & ((1ull << CI) - 1ull)) != 0ull;
    double wj = (NT1 ? cc.mK : s_c[tj * nt1 + it].mK) * wv;
    if (!(a.exp & 2)) wj = slot_sum<CI>(wj);
    if (il == 0 && any && j < a.n && !(a.exp & 1)) atomicAdd(&a.racc[j], wj);
  }
  acc = atom_sum<CI>(acc);
  if (HALF) {
    if (sl == 0 && ilive) atomicAdd(&a.racc[i], acc);
  } else if (sl == 0 && ilive) {  // complete: rho = self + sum, EOS (k_cl_rho_final)
    const double rho = cf->self_rho[it] + acc;
    a.vr[i].w = rho;
    a.xf[i].w = tait_p_over_rho2(rho, cf->rho0[it], cf->B[it]);
  }
}

// rho = self + sum (pair_sph_rhosum.cpp:116-138); EOS: also P/rho^2 into xf.w (the row
// kernels' fused epilogue)
template <bool EOS>
__global__ void __launch_bounds__(256)
k_cl_rho_final(int n, const double *__restrict__ racc, const int *__restrict__ ty,
               const Coefs *__restrict__ cf, double4 *__restrict__ xf, double4 *__restrict__ vr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int it = ty[i];
  const double rho = cf->self_rho[it] + racc[i];
  vr[i].w = rho;
  if (EOS) xf[i].w = tait_p_over_rho2(rho, cf->rho0[it], cf->B[it]);
}

// sph/taitwater[/morris] (+ sph/heatconduction): forces, drho, de over the clusters, in
// the reference's per-pair arithmetic (pair_sph_taitwater.cpp:136-191,
// pair_sph_taitwater_morris.cpp:130-185, pair_sph_heatconduction.cpp:103-129) with the
// Newton-3 updates of j.  Gravity (m g) is added with i's own sums.
template <int CI, int VISC, int MODE, bool NT1, bool HALF>
__global__ void __launch_bounds__(256) k_cl_force(ClArgs a) {
  constexpr int J = 64 / CI;
  constexpr bool TAIT = (MODE & M_TAIT) != 0;
  constexpr bool HEAT = (MODE & M_HEAT) != 0;
  __shared__ TaitPair s_t[(TAIT && !NT1) ? NT2 : 1];
  __shared__ HeatPair s_h[(HEAT && !NT1) ? NT2 : 1];
  const Coefs *cf = a.cf;
  const int nt1 = cf->ntypes + 1;
  if (!NT1) {
    for (int t = threadIdx.x; t < nt1 * nt1; t += blockDim.x) {
      if (TAIT) s_t[t] = cf->tait[t];
      if (HEAT) s_h[t] = cf->heat[t];
    }
    __syncthreads();
  }
  const int c = wave_uniform((int)((xcd_block() * blockDim.x + threadIdx.x) >> 6));
  const int i0 = c * CI;
  if (i0 >= a.n) return;  // wave-uniform
  const int lane = threadIdx.x & 63, il = lane & (CI - 1), sl = lane / CI;
  const int i = i0 + il;
  const bool ilive = i < a.n;
  const int ii = ilive ? i : i0;
  const Rsrc rn = make_rsrc(a.nbr, nbytes<int>(a.ntot));
  const Rsrc rx = make_rsrc(a.xf, nbytes<double4>(a.nall));
  const Rsrc rv = make_rsrc(a.vr, nbytes<double4>(a.nall));
  const Rsrc rt = make_rsrc(a.ty, nbytes<int>(a.nall));
  const Rsrc re = make_rsrc(a.en, HEAT ? nbytes<double>(a.nall) : 0u);
  const double4 xi = a.xf[ii];
  const double4 vi = a.vr[ii];
  const double ei = HEAT ? a.en[ii] : 0.0;
  const int it = NT1 ? 1 : a.ty[ii];
  TaitPair t1{};
  HeatPair h1{};
  if (NT1) {
    if (TAIT) t1 = cf->tait[3];
    if (HEAT) h1 = cf->heat[3];
  }
  const int beg = c * a.stride, end = beg + a.cnt[c];
  double fx = 0.0, fy = 0.0, fz = 0.0, drho = 0.0, dE = 0.0;
  int jn = ld_i32(rn, (unsigned)(beg + sl) * 4u);
  for (int k0 = beg; k0 < end; k0 += J) {  // wave-uniform trip count
    const int j = jn;
    const bool valid = k0 + sl < end;
    const unsigned o = (unsigned)j;
    const double4 xj = ld_d4(rx, o * 32u);
    const double4 vj = ld_d4(rv, o * 32u);
    const double ej = HEAT ? ld_d1(re, o * 8u) : 0.0;
    const int tj = NT1 ? 1 : ld_i32(rt, o * 4u);
    jn = ld_i32(rn, (unsigned)(k0 + J + sl) * 4u);
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    const int pidx = NT1 ? 3 : it * nt1 + tj;
    const unsigned jl = (unsigned)(j - i0);
    const bool ok = valid && ilive &&
                    (HALF ? (jl >= (unsigned)CI || (unsigned)il < jl) : jl != (unsigned)il);
    const double r = sqrt1(rsq);
    // j-side sums: -force, drho_j, de_j
    double gfx = 0.0, gfy = 0.0, gfz = 0.0, jdrho = 0.0, jdE = 0.0;
    bool in = false;
    if (TAIT) {
      const TaitPair cc = NT1 ? t1 : s_t[pidx];
      const bool hit = ok && rsq < cc.cutsq;
      in = hit;
      double wfd = cc.h - r;
      wfd = cc.wK * (wfd * wfd);
      wfd = hit ? wfd : 0.0;  // zeroes every term below
      const double velx = vi.x - vj.x, vely = vi.y - vj.y, velz = vi.z - vj.z;
      const double dvdr = dx * velx + dy * vely + dz * velz;
      if (VISC == SPH_VISC_MONAGHAN) {
        const double qv = (cc.viscC * dvdr) * rcp1((rsq + cc.eps) * (vi.w + vj.w));
        const double fvisc = dvdr < 0. ? qv : 0.0;
        const double fpair = cc.mm * (xi.w + xj.w + fvisc) * wfd;
        gfx = dx * fpair;
        gfy = dy * fpair;
        gfz = dz * fpair;
        jdE = -0.5 * fpair * dvdr;
      } else {
        double fvisc = cc.viscC * rcp1(vi.w * vj.w);
        fvisc = hit ? fvisc * ((-cc.mm) * wfd) : 0.0;  // 1/(rho_i rho_j) of a masked slot
        const double fpair = cc.mm * (xi.w + xj.w) * wfd;
        gfx = dx * fpair + velx * fvisc;
        gfy = dy * fpair + vely * fvisc;
        gfz = dz * fpair + velz * fvisc;
        jdE = -0.5 * (fpair * dvdr + fvisc * (velx * velx + vely * vely + velz * velz));
      }
      fx += gfx;
      fy += gfy;
      fz += gfz;
      drho += cc.mj * dvdr * wfd;
      jdrho = cc.mi * dvdr * wfd;
      dE += jdE;
    }
    if (HEAT) {
      const HeatPair cc = NT1 ? h1 : s_h[pidx];
      const bool hit = ok && rsq < cc.cutsq;
      in = in || hit;
      double wfd = cc.h - r;
      wfd = cc.wK * (wfd * wfd);
      wfd = hit ? wfd : 0.0;
      double deltaE = cc.hmD;
      deltaE *= (vi.w + vj.w) * rcp1(vi.w * vj.w);
      deltaE = hit ? deltaE * ((ei - ej) * wfd) : 0.0;
      dE += deltaE;
      jdE -= deltaE;
    }
    if (!HALF) continue;
    const unsigned long long bm = __ballot(in);
    const bool any = ((bm >> (sl * CI)) & ((1ull << CI) - 1ull)) != 0ull;
    if (__builtin_amdgcn_ballot_w64(any) == 0ull) continue;  // no pair of the batch in range
    if (a.exp & 2) {
      fx += gfx + gfy + gfz + jdrho + jdE;
      continue;
    }
    if (TAIT) {
      gfx = slot_sum<CI>(gfx);
      gfy = slot_sum<CI>(gfy);
      gfz = slot_sum<CI>(gfz);
      jdrho = slot_sum<CI>(jdrho);
    }
    jdE = slot_sum<CI>(jdE);
    if (any && j < a.n && !(a.exp & 1)) {
      // lane il of the slot adds component il: fx, fy, fz, drho [, de when CI = 8]
      if (TAIT && il < 4) {
        const double v = il == 0 ? -gfx : il == 1 ? -gfy : il == 2 ? -gfz : jdrho;
        atomicAdd(reinterpret_cast<double *>(&a.fo[j]) + il, v);
      }
      if (il == (CI == 8 && TAIT ? 4 : 0)) atomicAdd(&a.de[j], jdE);
    }
  }
  if (TAIT) {
    fx = atom_sum<CI>(fx);
    fy = atom_sum<CI>(fy);
    fz = atom_sum<CI>(fz);
    drho = atom_sum<CI>(drho);
  }
  dE = atom_sum<CI>(dE);
  if (!HALF) {  // complete sums: plain stores, as the row kernels
    if (ilive && sl == 0) {
      if (TAIT) {
        const double m = cf->mass[it];
        a.fo[i] = make_double4(fx + m * a.gx, fy + m * a.gy, fz + m * a.gz, drho);
      }
      a.de[i] = dE;
    }
    return;
  }
  if (ilive && sl < 5) {  // slot sl adds component sl of atom i
    if (sl < 4) {
      if (TAIT) {
        const double m = cf->mass[it];
        const double v = sl == 0 ? fx + m * a.gx : sl == 1 ? fy + m * a.gy : sl == 2 ? fz + m * a.gz : drho;
        atomicAdd(reinterpret_cast<double *>(&a.fo[i]) + sl, v);
      }
    } else {
      atomicAdd(&a.de[i], dE);
    }
  }
}

}  // namespace sph
