// sph_phasechange.hip -- fix phase_change (FixPhaseChange::pre_exchange,
// src/USER-SPH/fix_phase_change.cpp:167-352) behind include/sph_hip.h section 1c.
//
// Split by what the work is:
//  * device, parallel over atoms: the candidate test (type == to_type, T = e/cv >= Tc),
//    and for every candidate one walk of its full-list row giving isfromphasearound()
//    (:538-563) and the quintic weights of the from_type donors with their weighted
//    velocity sums (:233-289) -- everything that does not depend on the random stream;
//  * host, sequential over the (few) candidates in atom order: the Park-Miller draws
//    (RanPark::uniform, random_park.cpp:42-49), the insertion positions (create_newpos /
//    create_newpos_simple, :466-520) and the sub-domain test (insert_one_atom, :425-456),
//    which must consume the stream exactly in the reference's order;
//  * device again: the mass taken from the donors (dmass[j] += to_mass w_j / W) for the
//    candidates that did change phase, scattered with fp64 atomics onto owned and ghost j.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <vector>

#include "sph_ctx.h"
#include "sph_util.h"

namespace {

constexpr int PCG = 8;  // lanes per list row

struct PcDev {
  int dim, from_type, to_type;
  double Tc, to_mass, cutoff;
};

static __global__ void k_pc_flags(int inum, const int *__restrict__ ilist,
                                  const int *__restrict__ ty, const double *__restrict__ en,
                                  const double *__restrict__ cv, PcDev p,
                                  int *__restrict__ flag) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= inum) return;
  const int i = ilist[r];
  const double Ti = en[i] / cv[i];
  flag[r] = (!(Ti < p.Tc) && ty[i] == p.to_type) ? 1 : 0;
}

__device__ __forceinline__ double pc_w(int dim, double r) {
  return quintic_w(dim, r);  // sph_kernel_quintic{2,3}d(sqrt(rsq)*cutoff), :247-251
}

// one record per candidate: {around, W, Sv[3], Svest[3]}
template <int G>
__global__ void __launch_bounds__(256)
k_pc_candidates(int ncand, const int *__restrict__ cand, const int *__restrict__ ilist,
                const int *__restrict__ off, const int *__restrict__ nbr,
                const double4 *__restrict__ xf, const double4 *__restrict__ vr,
                const double *__restrict__ vel, const int *__restrict__ ty,
                const double *__restrict__ rm, PcDev p, double *__restrict__ rec) {
  const int k = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (k >= ncand) return;
  const int row = cand[k];
  const int i = ilist[row];
  const double4 xi = xf[i];
  const double cut2 = p.cutoff * p.cutoff;
  int around = 0;
  double W = 0.0, sv0 = 0.0, sv1 = 0.0, sv2 = 0.0, se0 = 0.0, se1 = 0.0, se2 = 0.0;
  for (int q = off[row] + lane; q < off[row + 1]; q += G) {
    const int j = nbr[q];
    if (ty[j] != p.from_type) continue;
    const double4 xj = xf[j];
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    if (rsq <= cut2) around = 1;
    if (rm[j] > 0.5 * p.to_mass) {
      const double w = pc_w(p.dim, sqrt(rsq) * p.cutoff);
      const double4 vj = vr[j];
      W += w;
      sv0 += w * vel[3 * j];
      sv1 += w * vel[3 * j + 1];
      sv2 += w * vel[3 * j + 2];
      se0 += w * vj.x;
      se1 += w * vj.y;
      se2 += w * vj.z;
    }
  }
  around = group_sum_i<G>(around);
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
  }
}

// dmass[j] += to_mass * w_j / W over the donors of every inserted candidate
template <int G>
__global__ void __launch_bounds__(256)
k_pc_dmass(int nins, const int *__restrict__ rows, const double *__restrict__ Wtot,
           const int *__restrict__ ilist, const int *__restrict__ off,
           const int *__restrict__ nbr, const double4 *__restrict__ xf,
           const int *__restrict__ ty, const double *__restrict__ rm, PcDev p,
           double *__restrict__ dmass) {
  const int k = (int)((xcd_block() * blockDim.x + threadIdx.x) / G);
  const int lane = threadIdx.x & (G - 1);
  if (k >= nins) return;
  const int row = rows[k];
  const int i = ilist[row];
  const double4 xi = xf[i];
  const double W = Wtot[k];
  for (int q = off[row] + lane; q < off[row + 1]; q += G) {
    const int j = nbr[q];
    if (ty[j] != p.from_type || !(rm[j] > 0.5 * p.to_mass)) continue;
    const double4 xj = xf[j];
    const double dx = xi.x - xj.x, dy = xi.y - xj.y, dz = xi.z - xj.z;
    const double rsq = dx * dx + dy * dy + dz * dz;
    atomicAdd(&dmass[j], p.to_mass * pc_w(p.dim, sqrt(rsq) * p.cutoff) / W);
  }
}

// ---- host side: the random stream, in the reference's order ----------------------------
double park_uniform(int &seed) {  // RanPark::uniform, random_park.cpp:42-49
  const int IA = 16807, IM = 2147483647, IQ = 127773, IR = 2836;
  const double AM = 1.0 / IM;
  const int k = seed / IQ;
  seed = IA * (seed - k * IQ) - IR * k;
  if (seed < 0) seed += IM;
  return AM * seed;
}

bool owns(const sph_phasechange_params &p, int dim, const double *c) {  // :441-452
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

void newpos_simple(int &seed, const double *x, double delta, double *c) {  // :466-470
  c[0] = x[0] + (park_uniform(seed) - 0.5) * delta;
  c[1] = x[1] + (park_uniform(seed) - 0.5) * delta;
  c[2] = x[2] + (park_uniform(seed) - 0.5) * delta;
}

void newpos(int dim, int &seed, const double *x, const double *cg, double delta,
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

}  // namespace

extern "C" {

int sph_hip_phasechange(sph_hip_ctx *c, const sph_phasechange_params *p, int *seed,
                        const double *v, const double *cg, double *e, double *dmass, int cap,
                        int *nins_out, double *new_atoms, int *parent) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && p && seed && v && cg && e && dmass && nins_out, SPH_HIP_EINVAL,
              "sph_hip_phasechange: NULL argument");
  SPH_REQUIRE(cap == 0 || (new_atoms && parent), SPH_HIP_EINVAL,
              "sph_hip_phasechange: cap > 0 needs new_atoms and parent");
  SPH_REQUIRE(*seed > 0, SPH_HIP_EINVAL, "Invalid seed for Park random # generator");
  SPH_REQUIRE(c->list_kind == SPH_LIST_FULL, SPH_HIP_EINVAL,
              "sph_hip_phasechange: needs the fix's FULL neighbor list staged");
  SPH_REQUIRE(c->have_mp_atoms, SPH_HIP_EINVAL,
              "sph_hip_phasechange: per-atom rmass/cv not staged (sph_hip_atoms_multiphase)");
  SPH_REQUIRE(p->to_mass > 0.0 && p->maxattempt >= 1, SPH_HIP_EINVAL,
              "sph_hip_phasechange: bad parameters");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const int nlocal = c->nlocal, nall = c->nlocal + c->nghost;
  for (int i = 0; i < nall; i++) dmass[i] = 0.0;  // :193-196 (newton on: all atoms)
  *nins_out = 0;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  PcDev pd{c->dim, p->from_type, p->to_type, p->Tc, p->to_mass, p->cutoff};
  const int inum = c->inum;
  // 1. candidates in row order
  DBuf<int> flag, cand, ncand_d, rows;
  DBuf<double> vel, rec, Wd, dm;
  flag.reserve(inum);
  cand.reserve(inum);
  ncand_d.reserve(1);
  hipLaunchKernelGGL(k_pc_flags, dim3((inum + 255) / 256), dim3(256), 0, c->stream, inum,
                     c->ilist.p, c->ty.p, c->en.p, c->cv.p, pd, flag.p);
  hipcub::CountingInputIterator<int> it(0);
  size_t tb = 0;
  SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, flag.p, cand.p, ncand_d.p, inum, c->stream));
  DBuf<unsigned char> tmp;
  tmp.reserve(tb);
  SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, it, flag.p, cand.p, ncand_d.p, inum, c->stream));
  int ncand = 0;
  SPH_HIP_TRY(hipMemcpyAsync(&ncand, ncand_d.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  auto release = [&]() {
    flag.release();
    cand.release();
    ncand_d.release();
    rows.release();
    vel.release();
    rec.release();
    Wd.release();
    dm.release();
    tmp.release();
  };
  if (ncand == 0) {
    release();
    return SPH_HIP_OK;
  }
  // 2. per-candidate list walk (stream independent)
  vel.reserve((size_t)3 * nall);
  rec.reserve((size_t)8 * ncand);
  SPH_HIP_TRY(hipMemcpyAsync(vel.p, v, (size_t)3 * nall * sizeof(double), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_pc_candidates<PCG>,
                     dim3((unsigned)(((long long)ncand * PCG + 255) / 256)), dim3(256), 0,
                     c->stream, ncand, cand.p, c->ilist.p, c->off.p, c->nbr.p, c->xf.p,
                     c->vr.p, vel.p, c->ty.p, c->rm.p, pd, rec.p);
  SPH_HIP_TRY(hipGetLastError());
  std::vector<int> hcand(ncand);
  std::vector<double> hrec((size_t)8 * ncand);
  std::vector<double> he(nall), hcv(nall);
  SPH_HIP_TRY(hipMemcpyAsync(hcand.data(), cand.p, ncand * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hrec.data(), rec.p, hrec.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(he.data(), c->en.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hcv.data(), c->cv.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  std::vector<double4> hxf(nall), hvr(nall);
  SPH_HIP_TRY(hipMemcpyAsync(hxf.data(), c->xf.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hvr.data(), c->vr.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  // 3. the random stream, candidate by candidate in atom order (:198-321)
  int s = *seed;
  std::vector<int> ins_rows;
  std::vector<double> ins_W;
  int nins = 0;
  for (int k = 0; k < ncand; k++) {
    const int i = c->hilist[hcand[k]];
    const double *r = &hrec[(size_t)8 * k];
    const double Ti = he[i] / hcv[i];
    const bool around = r[0] != 0.0;
    bool change;
    if (p->energy_chance) {
      const double threshold = (he[i] - p->Tc * hcv[i]) / p->Hwv * p->dt * p->rate;
      change = (park_uniform(s) < threshold) && around;
    } else {
      change = (park_uniform(s) < p->change_chance) && (Ti > p->Tt) && around;
    }
    if (!change) continue;
    const double xi[3] = {hxf[i].x, hxf[i].y, hxf[i].z};
    double coord[3];
    bool ok = false;
    double delta = p->dr;
    int na = 0;
    do {
      newpos(c->dim, s, xi, cg + 3 * (size_t)i, delta, coord);
      ok = owns(*p, c->dim, coord);
      delta = 0.75 * delta;
      na++;
    } while (!ok && na < p->maxattempt);
    if (!ok) {
      delta = p->dr;
      na = 0;
      do {
        newpos_simple(s, xi, delta, coord);
        ok = owns(*p, c->dim, coord);
        delta = 0.75 * delta;
        na++;
      } while (!ok && na < p->maxattempt);
    }
    if (!ok) continue;
    const double W = r[1];
    const double energy_aux = 0.5 * (he[i] - p->Hwv);  // :317-320
    if (nins < cap) {
      double *o = new_atoms + 13 * (size_t)nins;
      o[0] = coord[0];
      o[1] = coord[1];
      o[2] = coord[2];
      for (int d = 0; d < 3; d++) {
        o[3 + d] = (r[2 + d] * p->to_mass / W) / p->to_mass;  // dmom / to_mass (:300-302)
        o[6 + d] = (r[5 + d] * p->to_mass / W) / p->to_mass;  // dmomest / to_mass
      }
      o[9] = energy_aux;
      o[10] = p->to_mass;
      o[11] = hvr[i].w;
      o[12] = hcv[i];
      parent[nins] = i;
    }
    e[i] = energy_aux;
    he[i] = energy_aux;
    ins_rows.push_back(hcand[k]);
    ins_W.push_back(W);
    nins++;
  }
  *seed = s;
  *nins_out = nins;
  // 4. mass taken from the donors
  if (nins > 0) {
    rows.reserve(nins);
    Wd.reserve(nins);
    dm.reserve(nall);
    SPH_HIP_TRY(hipMemcpyAsync(rows.p, ins_rows.data(), nins * sizeof(int), hipMemcpyHostToDevice, c->stream));
    SPH_HIP_TRY(hipMemcpyAsync(Wd.p, ins_W.data(), nins * sizeof(double), hipMemcpyHostToDevice, c->stream));
    SPH_HIP_TRY(hipMemsetAsync(dm.p, 0, nall * sizeof(double), c->stream));
    hipLaunchKernelGGL(k_pc_dmass<PCG>, dim3((unsigned)(((long long)nins * PCG + 255) / 256)),
                       dim3(256), 0, c->stream, nins, rows.p, Wd.p, c->ilist.p, c->off.p,
                       c->nbr.p, c->xf.p, c->ty.p, c->rm.p, pd, dm.p);
    SPH_HIP_TRY(hipGetLastError());
    SPH_HIP_TRY(hipMemcpyAsync(dmass, dm.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  }
  // the staged e follows the update (a later pair pass sees the new energies)
  SPH_HIP_TRY(hipMemcpyAsync(c->en.p, he.data(), nlocal * sizeof(double), hipMemcpyHostToDevice, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  release();
  SPH_API_END
}

int sph_hip_phasechange_finish(int nlocal, const double *dmass, double *rmass, double *e) {
  SPH_API_BEGIN
  SPH_REQUIRE(nlocal >= 0 && (nlocal == 0 || (dmass && rmass && e)), SPH_HIP_EINVAL,
              "sph_hip_phasechange_finish: bad argument");
  for (int i = 0; i < nlocal; i++) {
    const double mold = rmass[i];
    rmass[i] -= dmass[i];
    SPH_REQUIRE(rmass[i] > 0.0, SPH_HIP_ERUNTIME, "atom %d lost all its mass (rmass %g)", i,
                rmass[i]);
    e[i] = e[i] * mold / rmass[i];
  }
  SPH_API_END
}

}  // extern "C"
