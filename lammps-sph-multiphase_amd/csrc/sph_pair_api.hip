// sph_pair_api.hip -- pair-style layer of the C ABI (include/sph_hip.h, section 1).
//
// What a LAMMPS `sph/<style>/hip` Pair class calls from compute(): LAMMPS' host arrays
// and NeighList are staged into the HBM layout of sph_kernels.h, the style's loop runs as
// a gfx950 kernel, and the results are added back into the caller's arrays.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdlib>
#include <algorithm>
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

// lanes per row of the pair layer's kernels: 8; study builds take SPH_GROUP (4, 8, 16)
int group_lanes() {
#ifdef SPH_STUDY
  static int g = [] {
    const char *s = getenv("SPH_GROUP");
    int v = s ? atoi(s) : 8;
    if (v != 4 && v != 8 && v != 16) v = 8;
    return v;
  }();
  return g;
#else
  return 8;
#endif
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
  c->unmap_all();
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
  c->release_lists();
  c->lbad.release();
  c->raw.release();
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

// LAMMPS' per-atom arrays (x, vest: nall*3; rho, e: nall; NULL = zeros) -> the gather
// records, with the type range checked on the way (bad |= 1)
static __global__ void k_pack_atoms(int nall, const double *__restrict__ x,
                                    const double *__restrict__ v, const double *__restrict__ rho,
                                    const double *__restrict__ e, const int *__restrict__ ty,
                                    int ntypes, double4 *__restrict__ xf, double4 *__restrict__ vr,
                                    double *__restrict__ en, int *__restrict__ bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nall) return;
  xf[i] = make_double4(x[3 * i], x[3 * i + 1], x[3 * i + 2], 0.0);
  vr[i] = make_double4(v ? v[3 * i] : 0.0, v ? v[3 * i + 1] : 0.0, v ? v[3 * i + 2] : 0.0,
                       rho ? rho[i] : 0.0);
  en[i] = e ? e[i] : 0.0;
  const int t = ty[i];
  if (t < 1 || t > ntypes) atomicOr(bad, 1);
}
static __global__ void k_pack_atoms_notype(int nall, const double *__restrict__ x,
                                           const double *__restrict__ v,
                                           const double *__restrict__ rho,
                                           const double *__restrict__ e,
                                           double4 *__restrict__ xf, double4 *__restrict__ vr,
                                           double *__restrict__ en) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nall) return;
  xf[i] = make_double4(x[3 * i], x[3 * i + 1], x[3 * i + 2], 0.0);
  vr[i] = make_double4(v ? v[3 * i] : 0.0, v ? v[3 * i + 1] : 0.0, v ? v[3 * i + 2] : 0.0,
                       rho ? rho[i] : 0.0);
  if (e) en[i] = e[i];
}
// results straight into the caller's (mapped host) arrays: rows r -> atom ilist[r] (nullptr:
// r itself); rho written, f / drho / de added
static __global__ void k_out_rho(int n, const int *__restrict__ ilist,
                                 const double *__restrict__ src, double *__restrict__ rho) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int i = ilist ? ilist[r] : r;
  rho[i] = src[i];
}
static __global__ void k_out_add(int n, const int *__restrict__ ilist,
                                 const double4 *__restrict__ fo, const double *__restrict__ dd,
                                 double *__restrict__ f, double *__restrict__ drho,
                                 double *__restrict__ de) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int i = ilist ? ilist[r] : r;
  if (f) {
    const double4 a = fo[i];
    f[3 * i] += a.x;
    f[3 * i + 1] += a.y;
    f[3 * i + 2] += a.z;
    if (drho) drho[i] += a.w;
  }
  if (de) de[i] += dd[i];
}
static __global__ void k_set_rho(int nall, const double *__restrict__ rho,
                                 double4 *__restrict__ vr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nall) vr[i].w = rho[i];
}

int sph_hip_host_arrays(sph_hip_ctx *c, int nmax, double *x, double *vest, double *rho,
                        double *e, double *f, double *drho, double *de) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && nmax >= 0, SPH_HIP_EINVAL, "sph_hip_host_arrays: bad argument");
  SPH_HIP_TRY(hipSetDevice(c->device));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));  // (nothing in flight reads the old ones)
  c->unmap_all();
  if (nmax == 0) return SPH_HIP_OK;
  const struct {
    void *p;
    size_t n;
  } arr[7] = {{x, 3}, {vest, 3}, {rho, 1}, {e, 1}, {f, 3}, {drho, 1}, {de, 1}};
  for (const auto &a : arr) {
    if (!a.p || c->mapped(a.p, a.n * nmax * sizeof(double))) continue;
    const size_t bytes = a.n * (size_t)nmax * sizeof(double);
    if (hipHostRegister(a.p, bytes, hipHostRegisterMapped) != hipSuccess) {
      (void)hipGetLastError();  // (not registrable: that array takes the copy path)
      continue;
    }
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, a.p, 0) != hipSuccess || !d) {
      (void)hipGetLastError();
      (void)hipHostUnregister(a.p);
      continue;
    }
    c->hmaps.push_back(sph_hip_ctx::HostMap{a.p, bytes, d});
  }
  SPH_API_END
}

// mapped-host inputs -> the gather records (k_pack_atoms reads them over PCIe)
static const double *in_dev(sph_hip_ctx *c, const double *h, size_t n) {
  return static_cast<const double *>(c->mapped(h, n * sizeof(double)));
}

int sph_hip_atoms(sph_hip_ctx *c, int nlocal, int nghost, const double *x, const double *vest,
                  const double *rho, const double *e, const int *type) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && x && type && nlocal >= 0 && nghost >= 0, SPH_HIP_EINVAL,
              "sph_hip_atoms: bad argument");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const size_t nall = (size_t)nlocal + nghost;
  if (nlocal != c->nlocal || nghost != c->nghost) c->drop_lists();  // (indices refer to nall)
  c->nlocal = nlocal;
  c->nghost = nghost;
  c->have_mp_atoms = false;  // rmass/cv must be restaged for the new atom set
  c->have_atoms = false;
  if (nall == 0) {
    c->have_atoms = true;
    return SPH_HIP_OK;
  }
  // raw arrays up (one copy each), packed into the gather records on the device
  c->xf.reserve(nall);
  c->vr.reserve(nall);
  c->en.reserve(nall);
  c->ty.reserve(nall);
  c->raw.reserve(8 * nall);
  c->lbad.reserve(1);
  double *const rx = c->raw.p, *const rv = rx + 3 * nall, *const rr = rv + 3 * nall,
               *const re = rr + nall;
  // each array read straight from mapped host memory by the pack kernel when registered
  // (sph_hip_host_arrays), else copied up first
  auto up = [&](const double *h, size_t n, double *staging) -> const double * {
    if (!h) return nullptr;
    if (const double *d = in_dev(c, h, n)) return d;
    SPH_HIP_TRY(hipMemcpyAsync(staging, h, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return staging;
  };
  const double *dx = up(x, 3 * nall, rx), *dv = up(vest, 3 * nall, rv),
               *dr = up(rho, nall, rr), *de_ = up(e, nall, re);
  SPH_HIP_TRY(hipMemcpyAsync(c->ty.p, type, nall * sizeof(int), hipMemcpyHostToDevice, c->stream));
  SPH_HIP_TRY(hipMemsetAsync(c->lbad.p, 0, sizeof(int), c->stream));
  hipLaunchKernelGGL(k_pack_atoms, dim3((unsigned)((nall + 255) / 256)), dim3(256), 0, c->stream,
                     (int)nall, dx, dv, dr, de_, c->ty.p, c->ntypes, c->xf.p, c->vr.p, c->en.p,
                     c->lbad.p);
  int bad = 0;
  SPH_HIP_TRY(hipMemcpyAsync(&bad, c->lbad.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  if (bad)
    for (size_t i = 0; i < nall; i++)  // (the culprit, for the message)
      SPH_REQUIRE(type[i] >= 1 && type[i] <= c->ntypes, SPH_HIP_EINVAL,
                  "atom %zu has type %d outside [1,%d]", i, type[i], c->ntypes);
  c->have_atoms = true;
  SPH_API_END
}

int sph_hip_atoms_update(sph_hip_ctx *c, const double *x, const double *vest,
                         const double *rho, const double *e) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && x, SPH_HIP_EINVAL, "sph_hip_atoms_update: bad argument");
  SPH_REQUIRE(c->have_atoms, SPH_HIP_EINVAL, "sph_hip_atoms_update: no atoms staged");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const size_t nall = (size_t)c->nlocal + c->nghost;
  if (nall == 0) return SPH_HIP_OK;  // (rmass / cv of the same atom set stay staged)
  c->raw.reserve(8 * nall);
  double *const rx = c->raw.p, *const rv = rx + 3 * nall, *const rr = rv + 3 * nall,
               *const re = rr + nall;
  auto up = [&](const double *h, size_t n, double *staging) -> const double * {
    if (!h) return nullptr;
    if (const double *d = in_dev(c, h, n)) return d;
    SPH_HIP_TRY(hipMemcpyAsync(staging, h, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return staging;
  };
  const double *dx = up(x, 3 * nall, rx), *dv = up(vest, 3 * nall, rv),
               *dr = up(rho, nall, rr), *de_ = up(e, nall, re);
  hipLaunchKernelGGL(k_pack_atoms_notype, dim3((unsigned)((nall + 255) / 256)), dim3(256), 0,
                     c->stream, (int)nall, dx, dv, dr, de_, c->xf.p, c->vr.p, c->en.p);
  SPH_HIP_TRY(hipGetLastError());
  SPH_API_END
}

int sph_hip_atoms_rho(sph_hip_ctx *c, const double *rho) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && rho, SPH_HIP_EINVAL, "sph_hip_atoms_rho: bad argument");
  SPH_REQUIRE(c->have_atoms, SPH_HIP_EINVAL, "sph_hip_atoms_rho: no atoms staged");
  SPH_HIP_TRY(hipSetDevice(c->device));
  const size_t nall = (size_t)c->nlocal + c->nghost;
  if (nall == 0) return SPH_HIP_OK;
  c->raw.reserve(8 * nall);
  const double *dr = in_dev(c, rho, nall);
  if (!dr) {
    SPH_HIP_TRY(hipMemcpyAsync(c->raw.p, rho, nall * sizeof(double), hipMemcpyHostToDevice, c->stream));
    dr = c->raw.p;
  }
  hipLaunchKernelGGL(k_set_rho, dim3((unsigned)((nall + 255) / 256)), dim3(256), 0, c->stream,
                     (int)nall, dr, c->vr.p);
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  SPH_API_END
}

// bad[0] |= 1 for a neighbor index outside [0, nall), |= 2 for an ilist entry that is not
// an owned atom (the kernels index atom arrays with both: checked once per upload, on the
// device, instead of a host loop over every entry)
static __global__ void k_list_check(long tot, const int *__restrict__ nbr, int nall, int inum,
                                    const int *__restrict__ ilist, int nlocal,
                                    int *__restrict__ bad) {
  int f = 0;
  for (long k = blockIdx.x * (long)blockDim.x + threadIdx.x; k < tot;
       k += (long)gridDim.x * blockDim.x) {
    const int j = nbr[k];
    if (j < 0 || j >= nall) f |= 1;
  }
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < inum; r += gridDim.x * blockDim.x) {
    const int i = ilist[r];
    if (i < 0 || i >= nlocal) f |= 2;
  }
  if (f) atomicOr(bad, f);
}

static void upload_list(sph_hip_ctx *c, int kind, int inum, int64_t key) {
  const size_t tot = (size_t)c->hoff[inum];
  SPH_REQUIRE(tot < (size_t)0x7fffffff, SPH_HIP_EOVERFLOW, "neighbor list too long (%zu)", tot);
  const int nall = c->nlocal + c->nghost;
  c->list_key = -1;  // (until the upload is checked)
  c->list_devbuilt = false;
  c->off.reserve(inum + 1);
  c->nbr.reserve(tot > 0 ? tot : 1);
  c->ilist.reserve(inum > 0 ? inum : 1);
  c->lbad.reserve(1);
  SPH_HIP_TRY(hipMemcpyAsync(c->off.p, c->hoff.data(), (inum + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (tot) SPH_HIP_TRY(hipMemcpyAsync(c->nbr.p, c->hnbr.data(), tot * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (inum) SPH_HIP_TRY(hipMemcpyAsync(c->ilist.p, c->hilist.data(), inum * sizeof(int), hipMemcpyHostToDevice, c->stream));
  SPH_HIP_TRY(hipMemsetAsync(c->lbad.p, 0, sizeof(int), c->stream));
  if (tot || inum) {
    const long work = std::max<long>((long)tot, inum);
    const unsigned grid = (unsigned)std::min<long>((work + 255) / 256, 4096);
    hipLaunchKernelGGL(k_list_check, dim3(grid), dim3(256), 0, c->stream, (long)tot, c->nbr.p,
                       nall, inum, c->ilist.p, c->nlocal, c->lbad.p);
  }
  int bad = 0;
  SPH_HIP_TRY(hipMemcpyAsync(&bad, c->lbad.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  SPH_HIP_TRY(hipStreamSynchronize(c->stream));
  c->list_kind = kind;
  c->inum = inum;
  c->rev_ok = false;
  if (bad) {
    c->list_kind = -1;  // (nothing may run on it)
    SPH_REQUIRE(!(bad & 1), SPH_HIP_EINVAL, "neighbor index outside [0,%d)", nall);
    SPH_REQUIRE(false, SPH_HIP_EINVAL, "ilist holds an index that is not an owned atom");
  }
  c->list_key = key;
}

int sph_hip_list(sph_hip_ctx *c, int kind, int inum, const int *ilist, const int *numneigh,
                 const int *const *firstneigh) {
  return sph_hip_list_keyed(c, kind, -1, inum, ilist, numneigh, firstneigh);
}

int sph_hip_list_keyed(sph_hip_ctx *c, int kind, int64_t key, int inum, const int *ilist,
                       const int *numneigh, const int *const *firstneigh) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && inum >= 0 && (inum == 0 || (ilist && numneigh && firstneigh)), SPH_HIP_EINVAL,
              "sph_hip_list: bad argument");
  SPH_REQUIRE(kind == SPH_LIST_FULL || kind == SPH_LIST_HALF, SPH_HIP_EINVAL, "bad list kind");
  SPH_HIP_TRY(hipSetDevice(c->device));
  c->select_list(kind);
  size_t tot = 0;
  for (int r = 0; r < inum; r++) tot += (size_t)numneigh[ilist[r]];
  // reuse: same build, same rows and entry count (two lists of one kind from one build --
  // a pair style's and a fix's full list -- are copies of each other in LAMMPS)
  if (key >= 0 && c->list_key == key && c->inum == inum && !c->hoff.empty() &&
      (size_t)c->hoff[inum] == tot)
    return SPH_HIP_OK;
  const int NEIGHMASK = 0x3FFFFFFF;  // src/lmptype.h / neighbor.h: SBBITS = 30
  c->hoff.resize(inum + 1);
  c->hilist.assign(ilist, ilist + inum);
  tot = 0;
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
  upload_list(c, kind, inum, key);
  SPH_API_END
}

int sph_hip_list_csr(sph_hip_ctx *c, int kind, int inum, const int64_t *off, const int *neigh) {
  SPH_API_BEGIN
  SPH_REQUIRE(c && off && (inum == 0 || neigh || off[inum] == 0), SPH_HIP_EINVAL,
              "sph_hip_list_csr: bad argument");
  SPH_REQUIRE(kind == SPH_LIST_FULL || kind == SPH_LIST_HALF, SPH_HIP_EINVAL, "bad list kind");
  SPH_HIP_TRY(hipSetDevice(c->device));
  c->select_list(kind);
  c->hoff.resize(inum + 1);
  c->hilist.resize(inum);
  for (int r = 0; r <= inum; r++) c->hoff[r] = (int)off[r];
  for (int r = 0; r < inum; r++) c->hilist[r] = r;
  const size_t tot = (size_t)off[inum];
  c->hnbr.assign(neigh, neigh + tot);
  upload_list(c, kind, inum, -1);
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
  if (double *dr = static_cast<double *>(c->mapped(rho, (size_t)nall * sizeof(double)))) {
    // straight into the caller's (mapped) rho
    hipLaunchKernelGGL(k_out_rho, dim3((c->inum + 255) / 256), dim3(256), 0, c->stream, c->inum,
                       (const int *)c->ilist.p, (const double *)c->rho_out.p, dr);
    SPH_HIP_TRY(hipStreamSynchronize(c->stream));
    c->tread();
    return SPH_HIP_OK;
  }
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
  {  // results added straight into the caller's (mapped) arrays when every one is registered
    const size_t nb = (size_t)nall * sizeof(double);
    double *mf = (mode & M_TAIT) ? static_cast<double *>(c->mapped(f, 3 * nb)) : nullptr;
    double *md = (mode & M_TAIT) && drho ? static_cast<double *>(c->mapped(drho, nb)) : nullptr;
    double *me = de ? static_cast<double *>(c->mapped(de, nb)) : nullptr;
    const bool ok = (!(mode & M_TAIT) || (mf && (md || !drho))) && (me || !de);
    if (ok) {
      const bool half = c->list_kind == SPH_LIST_HALF;
      const int rows = half ? nall : c->inum;
      hipLaunchKernelGGL(k_out_add, dim3((rows + 255) / 256), dim3(256), 0, c->stream, rows,
                         half ? (const int *)nullptr : (const int *)c->ilist.p,
                         (const double4 *)c->fo.p, (const double *)c->de.p, mf, md, me);
      if (virial) SPH_HIP_TRY(hipMemcpyAsync(hv, c->virial.p, 6 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
      SPH_HIP_TRY(hipStreamSynchronize(c->stream));
      c->tread();
      if (virial)
        for (int k = 0; k < 6; k++) virial[k] += hv[k];
      return;
    }
  }
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
