// sph_multiphase.hip -- multiphase styles of the pair-style layer (include/sph_hip.h,
// section 1b): what PairSPHRhoSumMultiphase, PairSPHTaitwaterMultiphase,
// PairSPHHeatConductionPhaseChange, PairSPHColorGradient and PairSPHSurfaceTension call
// from compute().
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <vector>

#include "sph_ctx.h"
#include "sph_util.h"

namespace {

constexpr int MPG = 8;  // lanes per list row

// upper-triangle (coeff() i <= j) table mirrored like init_one
template <typename T>
void mirror(T *dst, const T *src, int nt) {
  const int n1 = nt + 1;
  for (int i = 0; i <= nt; i++)
    for (int j = 0; j <= nt; j++) dst[i * n1 + j] = (j >= i) ? src[i * n1 + j] : src[j * n1 + i];
}

MpArgs mp_args(sph_hip_ctx *c) {
  MpArgs a{};
  a.inum = c->inum;
  a.nlocal = c->nlocal;
  a.newton = c->newton;
  a.dim = c->dim;
  a.half = c->list_kind == SPH_LIST_HALF;
  a.ilist = c->ilist.p;
  a.off = c->off.p;
  a.nbr = c->nbr.p;
  a.xf = c->xf.p;
  a.vr = c->vr.p;
  a.ty = c->ty.p;
  a.rm = c->rm.p;
  a.en = c->en.p;
  a.cv = c->cv.p;
  a.mc = c->dm;
#ifdef SPH_STUDY  // study variants (SPH_MPX), study builds only
  static const int mpx = [] {
    const char *v = getenv("SPH_MPX");
    return v ? atoi(v) : 0;
  }();
#else
  const int mpx = 0;
#endif
  a.exp = mpx;
  return a;
}

void mp_ready(sph_hip_ctx *c, const char *who, bool have) {
  SPH_REQUIRE(have, SPH_HIP_EINVAL, "%s: coefficients not set", who);
  SPH_REQUIRE(c->list_kind >= 0, SPH_HIP_EINVAL, "%s: no neighbor list staged", who);
  SPH_REQUIRE(c->have_mp_atoms, SPH_HIP_EINVAL,
              "%s: per-atom rmass/cv not staged (sph_hip_atoms_multiphase)", who);
  SPH_REQUIRE((long long)c->nlocal + c->nghost < MP_MAXALL, SPH_HIP_EOVERFLOW,
              "%s: the multiphase kernels index at most 2^28 atoms", who);
  SPH_HIP_TRY(hipSetDevice(c->device));
  if (!c->dm) SPH_HIP_TRY(hipMalloc(&c->dm, sizeof(MpCoefs)));
  c->hm.ntypes = c->ntypes;
  c->hm.dim = c->dim;
  c->upload_mp();
}

dim3 mp_grid(int inum) { return dim3((unsigned)(((long long)inum * MPG + 255) / 256)); }

// one half-list style: forward rows (+ reverse rows when gathering the j share)
template <int STYLE>
void run_half(sph_hip_ctx *c, MpArgs a) {
  const bool rev = a.half && sph_rev_on();
  c->tstart();  // the reverse build (first half-list style after a list upload) is timed too
  if (rev) {
    c->build_rev();
    a.rev = 1;
    a.roff = c->roff.p;
    a.rnbr = c->rnbr.p;
    a.nrows = c->newton ? c->nlocal + c->nghost : c->nlocal;
  }
  hipLaunchKernelGGL((k_mp_half<MPG, STYLE, false>), mp_grid(c->inum), dim3(256), 0, c->stream, a);
  if (rev && a.nrows > 0)
    hipLaunchKernelGGL((k_mp_half<MPG, STYLE, true>), mp_grid(a.nrows), dim3(256), 0, c->stream,
                       a);
  c->tstop();
}

}  // namespace

extern "C" {

int sph_hip_atoms_multiphase(sph_hip_ctx *c, const double *rmass, const double *cv) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && rmass, SPH_HIP_EINVAL, "sph_hip_atoms_multiphase: bad argument");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const size_t nall = (size_t)c->nlocal + c->nghost;
  c->have_mp_atoms = true;
  if (nall == 0) return SPH_HIP_OK;
  for (size_t i = 0; i < nall; i++)
    SPH_REQUIRE(rmass[i] > 0.0, SPH_HIP_EINVAL, "atom %zu has rmass %g <= 0", i, rmass[i]);
  c->rm.reserve(nall);
  c->cv.reserve(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->rm.p, rmass, nall * sizeof(double), hipMemcpyHostToDevice, c->stream));
  std::vector<double> h(nall, 1.0);
  if (cv)
    for (size_t i = 0; i < nall; i++) h[i] = cv[i];
  SPH_HIP_TRY(hipMemcpyAsync(c->cv.p, h.data(), nall * sizeof(double), hipMemcpyHostToDevice, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  SPH_API_END
}

int sph_hip_rhosum_multiphase_coeff(sph_hip_ctx *c, const double *cut) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && cut, SPH_HIP_EINVAL, "sph_hip_rhosum_multiphase_coeff: NULL argument");
  mirror(c->hm.rcut, cut, c->ntypes);
  for (int k = 0; k < NT2; k++) c->hm.rcutsq[k] = c->hm.rcut[k] * c->hm.rcut[k];
  c->have_mp_rho = true;
  c->mp_dirty = true;
  SPH_API_END
}

int sph_hip_rhosum_multiphase(sph_hip_ctx *c, double *rho) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && rho, SPH_HIP_EINVAL, "sph_hip_rhosum_multiphase: bad argument");
  mp_ready(c, "sph_hip_rhosum_multiphase", c->have_mp_rho);
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  c->rho_out.reserve(nall);
  MpArgs a = mp_args(c);
  a.rho = c->rho_out.p;
  c->tstart();
  hipLaunchKernelGGL(k_mp_rhosum<MPG>, mp_grid(c->inum), dim3(256), 0, c->stream, a);
  c->tstop();
  SPH_HIP_TRY(hipGetLastError());
  c->h1.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h1.data(), c->rho_out.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  for (int r = 0; r < c->inum; r++) rho[c->hilist[r]] = c->h1[c->hilist[r]];
  SPH_API_END
}

int sph_hip_taitwater_multiphase_coeff(sph_hip_ctx *c, const double *rho0,
                                       const double *soundspeed, const double *gamma,
                                       const double *rbackground, const double *viscosity,
                                       const double *cut) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && rho0 && soundspeed && gamma && rbackground && viscosity && cut,
              SPH_HIP_EINVAL, "sph_hip_taitwater_multiphase_coeff: NULL argument");
  for (int t = 1; t <= c->ntypes; t++) {
    SPH_REQUIRE(gamma[t] != 0.0 && rho0[t] != 0.0, SPH_HIP_EINVAL,
                "type %d: gamma and rho0 must be non-zero", t);
    c->hm.rho0[t] = rho0[t];
    c->hm.gamma[t] = gamma[t];
    c->hm.rbg[t] = rbackground[t];
    // B = c^2 rho0 / gamma, pair_sph_taitwater_multiphase.cpp:243-250
    c->hm.B[t] = soundspeed[t] * soundspeed[t] * rho0[t] / gamma[t];
  }
  mirror(c->hm.tvisc, viscosity, c->ntypes);
  mirror(c->hm.tcut, cut, c->ntypes);
  for (int k = 0; k < NT2; k++) c->hm.tcutsq[k] = c->hm.tcut[k] * c->hm.tcut[k];
  c->have_mp_tait = true;
  c->mp_dirty = true;
  SPH_API_END
}

int sph_hip_taitwater_multiphase(sph_hip_ctx *c, double *f) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && f, SPH_HIP_EINVAL, "sph_hip_taitwater_multiphase: bad argument");
  mp_ready(c, "sph_hip_taitwater_multiphase", c->have_mp_tait);
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  c->fo.reserve(nall);
  SPH_HIP_TRY(hipMemsetAsync(c->fo.p, 0, nall * sizeof(double4), c->stream));
  MpArgs a = mp_args(c);
  a.fo = c->fo.p;
  run_half<MP_TAIT>(c, a);
  SPH_HIP_TRY(hipGetLastError());
  c->h4.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h4.data(), c->fo.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  auto add = [&](int i) {
    f[3 * i] += c->h4[i].x;
    f[3 * i + 1] += c->h4[i].y;
    f[3 * i + 2] += c->h4[i].z;
  };
  if (a.half)
    for (int i = 0; i < nall; i++) add(i);
  else
    for (int r = 0; r < c->inum; r++) add(c->hilist[r]);
  SPH_API_END
}

int sph_hip_heatconduction_phasechange_coeff(sph_hip_ctx *c, const double *alpha,
                                             const int *fixflag, const double *tc,
                                             const double *cut) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && alpha && cut, SPH_HIP_EINVAL,
              "sph_hip_heatconduction_phasechange_coeff: NULL argument");
  mirror(c->hm.halpha, alpha, c->ntypes);
  mirror(c->hm.hcut, cut, c->ntypes);
  for (int k = 0; k < NT2; k++) {
    c->hm.hcutsq[k] = c->hm.hcut[k] * c->hm.hcut[k];
    c->hm.hfix[k] = 0;
    c->hm.htc[k] = 0.0;
  }
  if (fixflag) mirror(c->hm.hfix, fixflag, c->ntypes);
  if (tc) mirror(c->hm.htc, tc, c->ntypes);
  c->have_mp_heat = true;
  c->mp_dirty = true;
  SPH_API_END
}

int sph_hip_heatconduction_phasechange(sph_hip_ctx *c, double *de) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && de, SPH_HIP_EINVAL, "sph_hip_heatconduction_phasechange: bad argument");
  mp_ready(c, "sph_hip_heatconduction_phasechange", c->have_mp_heat);
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  c->de.reserve(nall);
  SPH_HIP_TRY(hipMemsetAsync(c->de.p, 0, nall * sizeof(double), c->stream));
  MpArgs a = mp_args(c);
  a.de = c->de.p;
  run_half<MP_HEAT>(c, a);
  SPH_HIP_TRY(hipGetLastError());
  c->h1.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h1.data(), c->de.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  if (a.half)
    for (int i = 0; i < nall; i++) de[i] += c->h1[i];
  else
    for (int r = 0; r < c->inum; r++) de[c->hilist[r]] += c->h1[c->hilist[r]];
  SPH_API_END
}

int sph_hip_colorgradient_coeff(sph_hip_ctx *c, const double *alpha, const double *cut) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && alpha && cut, SPH_HIP_EINVAL, "sph_hip_colorgradient_coeff: NULL argument");
  mirror(c->hm.calpha, alpha, c->ntypes);
  mirror(c->hm.ccut, cut, c->ntypes);
  for (int k = 0; k < NT2; k++) c->hm.ccutsq[k] = c->hm.ccut[k] * c->hm.ccut[k];
  c->have_mp_cg = true;
  c->mp_dirty = true;
  SPH_API_END
}

int sph_hip_colorgradient(sph_hip_ctx *c, double *cg) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && cg, SPH_HIP_EINVAL, "sph_hip_colorgradient: bad argument");
  mp_ready(c, "sph_hip_colorgradient", c->have_mp_cg);
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  c->cg.reserve(nall);
  MpArgs a = mp_args(c);
  a.cg = c->cg.p;
  c->tstart();
  hipLaunchKernelGGL(k_mp_colorgradient<MPG>, mp_grid(c->inum), dim3(256), 0, c->stream, a);
  c->tstop();
  SPH_HIP_TRY(hipGetLastError());
  c->h4.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h4.data(), c->cg.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  for (int r = 0; r < c->inum; r++) {
    const int i = c->hilist[r];
    cg[3 * i] = c->h4[i].x;
    cg[3 * i + 1] = c->h4[i].y;
    cg[3 * i + 2] = c->h4[i].z;
  }
  SPH_API_END
}

int sph_hip_surfacetension_coeff(sph_hip_ctx *c, const double *cut) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && cut, SPH_HIP_EINVAL, "sph_hip_surfacetension_coeff: NULL argument");
  mirror(c->hm.scut, cut, c->ntypes);
  for (int k = 0; k < NT2; k++) c->hm.scutsq[k] = c->hm.scut[k] * c->hm.scut[k];
  c->have_mp_st = true;
  c->mp_dirty = true;
  SPH_API_END
}

int sph_hip_surfacetension(sph_hip_ctx *c, const double *cg, double *f) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && cg && f, SPH_HIP_EINVAL, "sph_hip_surfacetension: bad argument");
  mp_ready(c, "sph_hip_surfacetension", c->have_mp_st);
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  c->h4in.resize(nall);
  for (int i = 0; i < nall; i++)
    c->h4in[i] = make_double4(cg[3 * i], cg[3 * i + 1], cg[3 * i + 2], 0.0);
  c->cgin.reserve(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->cgin.p, c->h4in.data(), nall * sizeof(double4), hipMemcpyHostToDevice, c->stream));
  c->fo.reserve(nall);
  SPH_HIP_TRY(hipMemsetAsync(c->fo.p, 0, nall * sizeof(double4), c->stream));
  MpArgs a = mp_args(c);
  a.fo = c->fo.p;
  a.cgi = c->cgin.p;
  run_half<MP_SURF>(c, a);
  SPH_HIP_TRY(hipGetLastError());
  c->h4.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h4.data(), c->fo.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  auto add = [&](int i) {
    f[3 * i] += c->h4[i].x;
    f[3 * i + 1] += c->h4[i].y;
    f[3 * i + 2] += c->h4[i].z;
  };
  if (a.half)
    for (int i = 0; i < nall; i++) add(i);
  else
    for (int r = 0; r < c->inum; r++) add(c->hilist[r]);
  SPH_API_END
}

}  // extern "C"
