// sph_pair_api.hip -- pair-style layer of the C ABI (include/sph_hip.h, section 1).
//
// What a LAMMPS `sph/<style>/hip` Pair class calls from compute(): LAMMPS' host arrays
// and NeighList are staged into the HBM layout of sph_kernels.h, the style's loop runs as
// a gfx950 kernel, and the results are added back into the caller's arrays.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdlib>
#include <vector>

#include "sph_coef.h"
#include "sph_ctx.h"
#include "sph_dispatch.h"
#include "sph_util.h"

namespace sph {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int group_lanes() {
  static int g = [] {
    const char *s = getenv("SPH_GROUP");
    int v = s ? atoi(s) : 8;
    if (v != 4 && v != 8 && v != 16) v = 8;
    return v;
  }();
  return g;
}

void require_device(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  SPH_REQUIRE(e == hipSuccess && n > 0, SPH_HIP_ENODEV,
              "no HIP device available (hipGetDeviceCount: %s, count %d)",
              hipGetErrorString(e), n);
  SPH_REQUIRE(device >= 0 && device < n, SPH_HIP_ENODEV, "device %d out of range (%d devices)",
              device, n);
  SPH_HIP_TRY(hipSetDevice(device));
}

}  // namespace sph

using namespace sph;

extern "C" {

const char *sph_hip_last_error(void) { return sph::g_err; }
int sph_hip_abi_version(void) { return SPH_HIP_ABI_VERSION; }
int sph_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int sph_hip_create(int device, int dim, int ntypes, int newton_pair, sph_hip_ctx **out) {
  SPH_API_BEGIN
  SPH_REQUIRE(out, SPH_HIP_EINVAL, "sph_hip_create: out is NULL");
  SPH_REQUIRE(dim == 2 || dim == 3, SPH_HIP_EINVAL, "dimension must be 2 or 3");
  SPH_REQUIRE(ntypes >= 1 && ntypes <= SPH_MAXTYPES, SPH_HIP_EINVAL,
              "ntypes %d outside [1,%d]", ntypes, SPH_MAXTYPES);
  require_device(device);
  sph_hip_ctx *c = new sph_hip_ctx;
  c->device = device;
  c->dim = dim;
  c->ntypes = ntypes;
  c->newton = newton_pair ? 1 : 0;
  c->hc.ntypes = ntypes;
  c->hc.dim = dim;
  SPH_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  SPH_HIP_TRY(hipMalloc(&c->dc, sizeof(Coefs)));
  *out = c;
  SPH_API_END
}

int sph_hip_set_timing(sph_hip_ctx *c, int on) {
  SPH_API_BEGIN
  SPH_REQUIRE(c, SPH_HIP_EINVAL, "sph_hip_set_timing: NULL context");
  SPH_HIP_TRY(hipSetDevice(c->device));
  if (on && !c->ev0) {
    SPH_HIP_TRY(hipEventCreate(&c->ev0));
    SPH_HIP_TRY(hipEventCreate(&c->ev1));
  }
  c->timing = on != 0;
  c->kernel_ms = 0.0;
  SPH_API_END
}

int sph_hip_last_kernel_ms(sph_hip_ctx *c, double *ms) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && ms, SPH_HIP_EINVAL, "sph_hip_last_kernel_ms: bad argument");
  *ms = c->kernel_ms;
  SPH_API_END
}

int sph_hip_destroy(sph_hip_ctx *c) {
  if (!c) return SPH_HIP_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  c->xf.release();
  c->vr.release();
  c->fo.release();
  c->rkey.release();
  c->rnbr.release();
  c->rown.release();
  c->roff.release();
  c->tmp.release();
  c->en.release();
  c->ty.release();
  c->de.release();
  c->rho_out.release();
  c->virial.release();
  c->ilist.release();
  c->off.release();
  c->nbr.release();
  c->rm.release();
  c->cv.release();
  c->cg.release();
  if (c->dm) (void)hipFree(c->dm);
  if (c->dc) (void)hipFree(c->dc);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return SPH_HIP_OK;
}

int sph_hip_rhosum_coeff(sph_hip_ctx *c, const double *cut, const double *mass) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && cut && mass, SPH_HIP_EINVAL, "sph_hip_rhosum_coeff: NULL argument");
  coef_rhosum(c->hc, c->dim, c->ntypes, cut, mass);
  for (int t = 0; t <= c->ntypes; t++) c->hc.mass[t] = mass[t];
  c->have_rho = true;
  c->coef_dirty = true;
  SPH_API_END
}

int sph_hip_taitwater_coeff(sph_hip_ctx *c, int visc_variant, const double *rho0,
                            const double *soundspeed, const double *B,
                            const double *viscosity, const double *cut, const double *mass) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && rho0 && soundspeed && B && viscosity && cut && mass, SPH_HIP_EINVAL,
              "sph_hip_taitwater_coeff: NULL argument");
  SPH_REQUIRE(visc_variant == SPH_VISC_MONAGHAN || visc_variant == SPH_VISC_MORRIS,
              SPH_HIP_EINVAL, "unknown viscosity variant %d", visc_variant);
  coef_tait(c->hc, c->dim, c->ntypes, visc_variant, rho0, soundspeed, B, viscosity, cut, mass);
  for (int t = 0; t <= c->ntypes; t++) c->hc.mass[t] = mass[t];
  c->tait_visc = visc_variant;
  c->have_tait = true;
  c->coef_dirty = true;
  SPH_API_END
}

int sph_hip_heatconduction_coeff(sph_hip_ctx *c, const double *alpha, const double *cut,
                                 const double *mass) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && alpha && cut && mass, SPH_HIP_EINVAL,
              "sph_hip_heatconduction_coeff: NULL argument");
  coef_heat(c->hc, c->dim, c->ntypes, alpha, cut, mass);
  for (int t = 0; t <= c->ntypes; t++) c->hc.mass[t] = mass[t];
  c->have_heat = true;
  c->coef_dirty = true;
  SPH_API_END
}

int sph_hip_atoms(sph_hip_ctx *c, int nlocal, int nghost, const double *x, const double *vest,
                  const double *rho, const double *e, const int *type) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && x && type && nlocal >= 0 && nghost >= 0, SPH_HIP_EINVAL,
              "sph_hip_atoms: bad argument");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const size_t nall = (size_t)nlocal + nghost;
  c->nlocal = nlocal;
  c->nghost = nghost;
  c->have_mp_atoms = false;  // rmass/cv must be restaged for the new atom set
  if (nall == 0) return SPH_HIP_OK;
  for (size_t i = 0; i < nall; i++)
    SPH_REQUIRE(type[i] >= 1 && type[i] <= c->ntypes, SPH_HIP_EINVAL,
                "atom %zu has type %d outside [1,%d]", i, type[i], c->ntypes);
  c->xf.reserve(nall);
  c->vr.reserve(nall);
  c->en.reserve(nall);
  c->ty.reserve(nall);
  c->h4.resize(nall);
  for (size_t i = 0; i < nall; i++)
    c->h4[i] = make_double4(x[3 * i], x[3 * i + 1], x[3 * i + 2], 0.0);
  SPH_HIP_TRY(hipMemcpyAsync(c->xf.p, c->h4.data(), nall * sizeof(double4), hipMemcpyHostToDevice, c->stream));
  SPH_HIP_TRY(hipMemcpyAsync(c->ty.p, type, nall * sizeof(int), hipMemcpyHostToDevice, c->stream));
  std::vector<double4> hv(nall);
  for (size_t i = 0; i < nall; i++)
    hv[i] = make_double4(vest ? vest[3 * i] : 0.0, vest ? vest[3 * i + 1] : 0.0,
                         vest ? vest[3 * i + 2] : 0.0, rho ? rho[i] : 0.0);
  SPH_HIP_TRY(hipMemcpyAsync(c->vr.p, hv.data(), nall * sizeof(double4), hipMemcpyHostToDevice, c->stream));
  c->h1.assign(nall, 0.0);
  if (e)
    for (size_t i = 0; i < nall; i++) c->h1[i] = e[i];
  SPH_HIP_TRY(hipMemcpyAsync(c->en.p, c->h1.data(), nall * sizeof(double), hipMemcpyHostToDevice, c->stream));
  // staging vectors must outlive the async copies
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  SPH_API_END
}

static void upload_list(sph_hip_ctx *c, int kind, int inum) {
  const size_t tot = (size_t)c->hoff[inum];
  SPH_REQUIRE(tot < (size_t)0x7fffffff, SPH_HIP_EOVERFLOW, "neighbor list too long (%zu)", tot);
  const size_t nall = (size_t)c->nlocal + c->nghost;
  for (size_t k = 0; k < tot; k++)
    SPH_REQUIRE(c->hnbr[k] >= 0 && (size_t)c->hnbr[k] < nall, SPH_HIP_EINVAL,
                "neighbor index %d outside [0,%zu)", c->hnbr[k], nall);
  for (int r = 0; r < inum; r++)
    SPH_REQUIRE(c->hilist[r] >= 0 && c->hilist[r] < c->nlocal, SPH_HIP_EINVAL,
                "ilist[%d] = %d is not an owned atom", r, c->hilist[r]);
  c->off.reserve(inum + 1);
  c->nbr.reserve(tot > 0 ? tot : 1);
  c->ilist.reserve(inum > 0 ? inum : 1);
  SPH_HIP_TRY(hipMemcpyAsync(c->off.p, c->hoff.data(), (inum + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (tot) SPH_HIP_TRY(hipMemcpyAsync(c->nbr.p, c->hnbr.data(), tot * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (inum) SPH_HIP_TRY(hipMemcpyAsync(c->ilist.p, c->hilist.data(), inum * sizeof(int), hipMemcpyHostToDevice, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->list_kind = kind;
  c->inum = inum;
  c->rev_ok = false;
}

int sph_hip_list(sph_hip_ctx *c, int kind, int inum, const int *ilist, const int *numneigh,
                 const int *const *firstneigh) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && (inum == 0 || (ilist && numneigh && firstneigh)), SPH_HIP_EINVAL,
              "sph_hip_list: bad argument");
  SPH_REQUIRE(kind == SPH_LIST_FULL || kind == SPH_LIST_HALF, SPH_HIP_EINVAL, "bad list kind");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const int NEIGHMASK = 0x3FFFFFFF;  // src/lmptype.h / neighbor.h: SBBITS = 30
  c->hoff.resize(inum + 1);
  c->hilist.assign(ilist, ilist + inum);
  size_t tot = 0;
  for (int r = 0; r < inum; r++) {
    c->hoff[r] = (int)tot;
    tot += (size_t)numneigh[ilist[r]];
  }
  c->hoff[inum] = (int)tot;
  c->hnbr.resize(tot);
  for (int r = 0; r < inum; r++) {
    const int i = ilist[r];
    const int *jl = firstneigh[i];
    for (int k = 0; k < numneigh[i]; k++) c->hnbr[c->hoff[r] + k] = jl[k] & NEIGHMASK;
  }
  upload_list(c, kind, inum);
  SPH_API_END
}

int sph_hip_list_csr(sph_hip_ctx *c, int kind, int inum, const int64_t *off, const int *neigh) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && off && (inum == 0 || neigh || off[inum] == 0), SPH_HIP_EINVAL,
              "sph_hip_list_csr: bad argument");
  SPH_REQUIRE(kind == SPH_LIST_FULL || kind == SPH_LIST_HALF, SPH_HIP_EINVAL, "bad list kind");
  SPH_HIP_TRY(hipSetDevice(c->device));
  c->hoff.resize(inum + 1);
  c->hilist.resize(inum);
  for (int r = 0; r <= inum; r++) c->hoff[r] = (int)off[r];
  for (int r = 0; r < inum; r++) c->hilist[r] = r;
  const size_t tot = (size_t)off[inum];
  c->hnbr.assign(neigh, neigh + tot);
  upload_list(c, kind, inum);
  SPH_API_END
}

int sph_hip_rhosum(sph_hip_ctx *c, double *rho) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && rho, SPH_HIP_EINVAL, "sph_hip_rhosum: bad argument");
  SPH_REQUIRE(c->have_rho, SPH_HIP_EINVAL, "sph_hip_rhosum: coefficients not set");
  SPH_REQUIRE(c->list_kind >= 0, SPH_HIP_EINVAL, "sph_hip_rhosum: no neighbor list staged");
  SPH_HIP_TRY(hipSetDevice(c->device));
  c->upload_coefs();
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return SPH_HIP_OK;
  c->rho_out.reserve(nall);
  RhoArgs ra{c->inum, c->ilist.p, c->off.p, c->nbr.p, c->xf.p, c->ty.p, c->vr.p, c->rho_out.p,
             c->dc};
  c->tstart();
  launch_rhosum(c->dim, false, c->ntypes == 1, c->stream, ra);
  c->tstop();
  SPH_HIP_TRY(hipGetLastError());
  c->h1.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h1.data(), c->rho_out.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  for (int r = 0; r < c->inum; r++) {
    const int i = c->hilist[r];
    rho[i] = c->h1[i];
  }
  SPH_API_END
}

static void run_force(sph_hip_ctx *c, int mode, double *f, double *drho, double *de,
                      double *virial) {
  SPH_HIP_TRY(hipSetDevice(c->device));
  c->upload_coefs();
  const int nall = c->nlocal + c->nghost;
  if (c->inum == 0 || nall == 0) return;
  c->fo.reserve(nall);
  c->de.reserve(nall);
  SPH_HIP_TRY(hipMemsetAsync(c->fo.p, 0, nall * sizeof(double4), c->stream));
  SPH_HIP_TRY(hipMemsetAsync(c->de.p, 0, nall * sizeof(double), c->stream));
  if (virial) {
    c->virial.reserve(6);
    SPH_HIP_TRY(hipMemsetAsync(c->virial.p, 0, 6 * sizeof(double), c->stream));
  }
  c->tstart();
  if (mode & M_TAIT)  // p/rho^2 of every atom (owned + ghost) from the staged rho
    hipLaunchKernelGGL(k_eos, dim3((nall + 255) / 256), dim3(256), 0, c->stream, nall, c->xf.p,
                       c->vr.p, c->ty.p, c->dc);
  ForceArgs a{};
  a.inum = c->inum;
  a.nlocal = c->nlocal;
  a.newton = c->newton;
  a.ilist = c->ilist.p;
  a.off = c->off.p;
  a.nbr = c->nbr.p;
  a.xf = c->xf.p;
  a.vr = c->vr.p;
  a.ty = c->ty.p;
  a.en = c->en.p;
  a.fo = c->fo.p;
  a.de = c->de.p;
  a.accum = 0;
  a.cf = c->dc;
  a.virial = virial ? c->virial.p : nullptr;
  const bool rev = c->list_kind == SPH_LIST_HALF && sph_rev_on();
  if (rev) c->build_rev();  // timed with the kernels (once per list upload)
  if (c->list_kind == SPH_LIST_HALF) mode |= M_HALF;
  a.nojside = rev ? 1 : 0;
  launch_force(c->dim, c->ntypes == 1, c->stream, c->tait_visc, mode, a);
  if (rev && c->rev_rows() > 0) {
    // the j share: FULL-mode gather over the reverse half list, added to the i shares
    ForceArgs b = a;
    b.inum = c->rev_rows();
    b.ilist = nullptr;
    b.off = c->roff.p;
    b.nbr = c->rnbr.p;
    b.accum = 1;
    b.virial = nullptr;
    b.nojside = 0;
    launch_force(c->dim, c->ntypes == 1, c->stream, c->tait_visc, mode & ~M_HALF, b);
  }
  c->tstop();
  SPH_HIP_TRY(hipGetLastError());
  double hv[6] = {0, 0, 0, 0, 0, 0};
  if (mode & M_TAIT) {
    c->h4.resize(nall);
    SPH_HIP_TRY(hipMemcpyAsync(c->h4.data(), c->fo.p, nall * sizeof(double4), hipMemcpyDeviceToHost, c->stream));
  }
  c->h1.resize(nall);
  SPH_HIP_TRY(hipMemcpyAsync(c->h1.data(), c->de.p, nall * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (virial) SPH_HIP_TRY(hipMemcpyAsync(hv, c->virial.p, 6 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->tread();
  const int n = (c->list_kind == SPH_LIST_HALF) ? nall : 0;
  auto add_atom = [&](int i) {
    if (mode & M_TAIT) {
      f[3 * i] += c->h4[i].x;
      f[3 * i + 1] += c->h4[i].y;
      f[3 * i + 2] += c->h4[i].z;
      if (drho) drho[i] += c->h4[i].w;
    }
    if (de) de[i] += c->h1[i];
  };
  if (c->list_kind == SPH_LIST_HALF) {
    for (int i = 0; i < n; i++) add_atom(i);
  } else {
    for (int r = 0; r < c->inum; r++) add_atom(c->hilist[r]);
  }
  if (virial)
    for (int k = 0; k < 6; k++) virial[k] += hv[k];
}

int sph_hip_taitwater(sph_hip_ctx *c, double *f, double *drho, double *de, double *virial) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && f && drho && de, SPH_HIP_EINVAL, "sph_hip_taitwater: bad argument");
  SPH_REQUIRE(c->have_tait, SPH_HIP_EINVAL, "sph_hip_taitwater: coefficients not set");
  SPH_REQUIRE(c->list_kind >= 0, SPH_HIP_EINVAL, "sph_hip_taitwater: no neighbor list staged");
  run_force(c, M_TAIT, f, drho, de, virial);
  SPH_API_END
}

int sph_hip_heatconduction(sph_hip_ctx *c, double *de) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && de, SPH_HIP_EINVAL, "sph_hip_heatconduction: bad argument");
  SPH_REQUIRE(c->have_heat, SPH_HIP_EINVAL, "sph_hip_heatconduction: coefficients not set");
  SPH_REQUIRE(c->list_kind >= 0, SPH_HIP_EINVAL, "sph_hip_heatconduction: no neighbor list staged");
  run_force(c, M_HEAT, nullptr, nullptr, de, nullptr);
  SPH_API_END
}

}  // extern "C"
