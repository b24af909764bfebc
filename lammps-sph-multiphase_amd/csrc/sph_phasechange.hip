// sph_phasechange.hip -- fix phase_change (FixPhaseChange::pre_exchange,
// src/USER-SPH/fix_phase_change.cpp:167-352) behind include/sph_hip.h section 1c: the
// staged atoms and the fix's full list of the pair-style layer through the shared
// candidate kernels and stream replay of sph_pc.h.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <vector>

#include "sph_ctx.h"
#include "sph_pc.h"
#include "sph_util.h"

namespace {
constexpr int PCG = 8;  // lanes per list row
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
  SPH_REQUIRE((long long)c->nlocal + c->nghost < MP_MAXALL, SPH_HIP_EOVERFLOW,
              "sph_hip_phasechange: at most 2^28 atoms");
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
  DBuf<int> flag, cand, ncand_d, rows, minr, one;
  DBuf<double> vel, rec, Wd, dm, rec1;
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
    minr.release();
    one.release();
    rec1.release();
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
  // the staged atoms are in LAMMPS order: ghost j sits in slot j - nlocal (sph_pc.h)
  const PcRank rk{nlocal, 0, nullptr};
  vel.reserve((size_t)3 * nall);
  rec.reserve((size_t)8 * ncand);
  minr.reserve(ncand);
  SPH_HIP_TRY(hipMemcpyAsync(vel.p, v, (size_t)3 * nall * sizeof(double), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_pc_candidates<PCG>,
                     dim3((unsigned)(((long long)ncand * PCG + 255) / 256)), dim3(256), 0,
                     c->stream, ncand, cand.p, c->ilist.p, c->off.p, c->nbr.p, c->xf.p,
                     c->vr.p, vel.p, 3, c->ty.p, c->rm.p, pd, rec.p, 0, (const int *)nullptr,
                     rk, 0, 0, minr.p);
  SPH_HIP_TRY(hipGetLastError());
  std::vector<int> hcand(ncand), hminr(ncand);
  std::vector<double> hrec((size_t)8 * ncand);
  std::vector<double> he(nall), hcv(nall);
  SPH_HIP_TRY(hipMemcpyAsync(hcand.data(), cand.p, ncand * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hminr.data(), minr.p, ncand * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hrec.data(), rec.p, hrec.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(he.data(), c->en.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hcv.data(), c->cv.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  std::vector<double4> hxf(nall), hvr(nall);
  SPH_HIP_TRY(hipMemcpyAsync(hxf.data(), c->xf.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(hvr.data(), c->vr.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  // 3. the random stream, candidate by candidate in atom order (:198-321)
  std::vector<PcCand> cands(ncand);
  for (int k = 0; k < ncand; k++) {
    const int i = c->hilist[hcand[k]];
    PcCand &a = cands[k];
    a.x[0] = hxf[i].x;
    a.x[1] = hxf[i].y;
    a.x[2] = hxf[i].z;
    for (int d = 0; d < 3; d++) a.cg[d] = cg[3 * (size_t)i + d];
    a.e = he[i];
    a.cv = hcv[i];
    a.rho = hvr[i].w;
    for (int q = 0; q < 8; q++) a.rec[q] = hrec[(size_t)8 * k + q];
    a.minr = hminr[k];
  }
  // a candidate whose row meets a slot already overwritten by a created atom: its walk again
  // on the device without those slots
  auto recompute = [&](size_t k, int dead_a, int dead_w, double *out) {
    one.reserve(1);
    rec1.reserve(8);
    SPH_HIP_TRY(hipMemcpyAsync(one.p, &hcand[k], sizeof(int), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_pc_candidates<PCG>, dim3(1), dim3(256), 0, c->stream, 1, one.p,
                       c->ilist.p, c->off.p, c->nbr.p, c->xf.p, c->vr.p, vel.p, 3, c->ty.p,
                       c->rm.p, pd, rec1.p, 0, (const int *)nullptr, rk, dead_a, dead_w,
                       (int *)nullptr);
    SPH_HIP_TRY(hipMemcpyAsync(out, rec1.p, 8 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  };
  int s = *seed;
  std::vector<int> ins_k;
  std::vector<double> ins_rec, ins_Wv;
  pc_replay(*p, c->dim, s, cands, ins_k, ins_Wv, ins_rec, recompute);
  const int nins = (int)ins_k.size();
  std::vector<int> ins_rows(nins);
  std::vector<double> ins_W(nins);
  for (int q = 0; q < nins; q++) {
    const int k = ins_k[q];
    const int i = c->hilist[hcand[k]];
    const double *o = &ins_rec[(size_t)13 * q];
    if (q < cap) {
      for (int d = 0; d < 13; d++) new_atoms[13 * (size_t)q + d] = o[d];
      parent[q] = i;
    }
    e[i] = o[9];
    he[i] = o[9];
    ins_rows[q] = hcand[k];
    ins_W[q] = ins_Wv[q];
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
    long long cap = 0;  // the inserted candidates' row lengths
    for (int q = 0; q < nins; q++) cap += c->hoff[ins_rows[q] + 1] - c->hoff[ins_rows[q]];
    DBuf<unsigned long long> k0, k1;
    DBuf<double> v0, v1;
    DBuf<int> cnt;
    pc_dmass_ordered<PCG>(c->stream, nins, rows.p, Wd.p, c->ilist.p, c->off.p, c->nbr.p,
                          c->xf.p, c->ty.p, c->rm.p, pd, 0, (const int *)nullptr, rk, cap, k0,
                          k1, v0, v1, cnt, tmp, dm.p);
    SPH_HIP_TRY(hipMemcpyAsync(dmass, dm.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SPH_HIP_TRY(hipStreamSynchronize(c->stream));
    k0.release();
    k1.release();
    v0.release();
    v1.release();
    cnt.release();
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
