// sph_ctx.h -- the pair-style layer's context (include/sph_hip.h section 1), shared by
// the translation units that implement its entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <vector>

#include "sph_kernels.h"
#include "sph_mp_kernels.h"
#include "sph_util.h"

using namespace sph;

// SPH_MPREV (default 1): half-list styles gather the j share through the reverse half list
// instead of scattering it with fp64 atomics
inline bool sph_rev_on() {
  static const bool v = [] {
    const char *e = getenv("SPH_MPREV");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

struct sph_hip_ctx {
  int device = 0, dim = 3, ntypes = 1, newton = 1;
  hipStream_t stream = nullptr;
  Coefs hc{};
  Coefs *dc = nullptr;
  bool have_rho = false, have_tait = false, have_heat = false;
  int tait_visc = SPH_VISC_MONAGHAN;
  int nlocal = 0, nghost = 0;
  int list_kind = -1, inum = 0;
  DBuf<double4> xf, vr, fo;
  DBuf<double> en, de, rho_out, virial;
  DBuf<int> ty, ilist, off, nbr;
  // multiphase styles (atom_style meso/multiphase): per-atom rmass and cv, own coefficients
  DBuf<double> rm, cv;
  DBuf<double4> cg, cgin;
  bool have_mp_atoms = false;
  bool have_mp_rho = false, have_mp_tait = false, have_mp_heat = false, have_mp_cg = false;
  bool have_mp_st = false;
  // reverse of the staged half list (k_mp_half REV), built on first use after a list upload
  DBuf<int> rkey, rnbr, rown, roff;
  DBuf<unsigned char> tmp;
  bool rev_ok = false;
  std::vector<double4> h4in;
  MpCoefs hm{};
  MpCoefs *dm = nullptr;
  bool mp_dirty = true;
  std::vector<double4> h4;
  std::vector<double> h1;
  std::vector<int> hoff, hnbr, hilist;
  bool coef_dirty = true;
  // optional device timing of each style call's kernels (sph_hip_set_timing)
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double kernel_ms = 0.0;
  void tstart() {
    if (timing) SPH_HIP_TRY(hipEventRecord(ev0, stream));
  }
  void tstop() {
    if (timing) SPH_HIP_TRY(hipEventRecord(ev1, stream));
  }
  // after the stream synchronised
  void tread() {
    if (!timing) return;
    float ms = 0.f;
    SPH_HIP_TRY(hipEventElapsedTime(&ms, ev0, ev1));
    kernel_ms = ms;
  }

  // Reverse of the staged half list: entries sorted by j (stable radix sort of (j, row
  // atom) pairs), CSR offsets over the reverse rows (nall with newton_pair, else nlocal:
  // without newton the reference gives ghosts no share).  Built once per list upload.
  int rev_rows() const { return newton ? nlocal + nghost : nlocal; }
  void build_rev() {
    if (rev_ok) return;
    const int nall = nlocal + nghost;
    const int tot = hoff[inum];
    const int nrows = rev_rows();
    rkey.reserve(tot > 0 ? tot : 1);
    rnbr.reserve(tot > 0 ? tot : 1);
    rown.reserve(tot > 0 ? tot : 1);
    roff.reserve((size_t)nrows + 1);
    if (inum)
      hipLaunchKernelGGL(k_entry_owner, dim3((inum + 255) / 256), dim3(256), 0, stream, inum,
                         off.p, ilist.p, rown.p);
    int endbit = 1;
    while ((1u << endbit) < (unsigned)(nall + 1) && endbit < 31) endbit++;
    if (tot) {
      size_t tb = 0;
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, nbr.p, rkey.p, rown.p, rnbr.p,
                                                     tot, 0, endbit, stream));
      tmp.reserve(tb);
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, nbr.p, rkey.p, rown.p, rnbr.p,
                                                     tot, 0, endbit, stream));
    }
    hipLaunchKernelGGL(k_rev_offsets, dim3((nrows + 1 + 255) / 256), dim3(256), 0, stream,
                       nrows, tot, rkey.p, roff.p);
    SPH_HIP_TRY(hipGetLastError());
    rev_ok = true;
  }
  void upload_mp() {
    if (!mp_dirty) return;
    SPH_HIP_TRY(hipMemcpyAsync(dm, &hm, sizeof(MpCoefs), hipMemcpyHostToDevice, stream));
    mp_dirty = false;
  }
  void upload_coefs() {
    if (!coef_dirty) return;
    SPH_HIP_TRY(hipMemcpyAsync(dc, &hc, sizeof(Coefs), hipMemcpyHostToDevice, stream));
    coef_dirty = false;
  }
};

