// sph_ctx.h -- the pair-style layer's context (include/sph_hip.h section 1), shared by
// the translation units that implement its entry points.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "sph_kernels.h"
#include "sph_mp_kernels.h"
#include "sph_util.h"

using namespace sph;

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

