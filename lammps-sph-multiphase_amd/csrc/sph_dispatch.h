// sph_dispatch.h -- runtime -> template dispatch for the CSR pair kernels.
#pragma once
#include "sph_kernels.h"
#include "sph_util.h"

namespace sph {

// lanes per neighbor-list row; SPH_GROUP env var overrides (tuning), default 8
int group_lanes();

inline unsigned grid_for_rows(long rows, int G, int block = 256) {
  return (unsigned)((rows * (long)G + block - 1) / block);
}

struct RhoArgs {
  int inum;
  const int *ilist, *off, *nbr;
  double4 *xf;
  const int *ty;
  double4 *vr;
  double *rho_out;
  const Coefs *cf;
};

template <int G, int DIM, bool EOS, bool NT1>
inline void launch_rhosum_t(hipStream_t s, const RhoArgs &a) {
  hipLaunchKernelGGL((k_rhosum<G, DIM, EOS, NT1>), dim3(grid_for_rows(a.inum, G)), dim3(256),
                     0, s, a.inum, a.ilist, a.off, a.nbr, a.xf, a.ty, a.vr, a.rho_out, a.cf);
}

template <int G>
inline void launch_rhosum_g(int dim, bool eos, bool nt1, hipStream_t s, const RhoArgs &a) {
  const int code = (dim == 3 ? 4 : 0) | (eos ? 2 : 0) | (nt1 ? 1 : 0);
  switch (code) {
    case 7: launch_rhosum_t<G, 3, true, true>(s, a); break;
    case 6: launch_rhosum_t<G, 3, true, false>(s, a); break;
    case 5: launch_rhosum_t<G, 3, false, true>(s, a); break;
    case 4: launch_rhosum_t<G, 3, false, false>(s, a); break;
    case 3: launch_rhosum_t<G, 2, true, true>(s, a); break;
    case 2: launch_rhosum_t<G, 2, true, false>(s, a); break;
    case 1: launch_rhosum_t<G, 2, false, true>(s, a); break;
    default: launch_rhosum_t<G, 2, false, false>(s, a); break;
  }
}

inline void launch_rhosum(int dim, bool eos, bool nt1, hipStream_t s, const RhoArgs &a) {
  if (a.inum <= 0) return;
  switch (group_lanes()) {
    case 4: launch_rhosum_g<4>(dim, eos, nt1, s, a); break;
    case 16: launch_rhosum_g<16>(dim, eos, nt1, s, a); break;
    default: launch_rhosum_g<8>(dim, eos, nt1, s, a); break;
  }
}

struct ForceArgs {
  int inum, nlocal, newton;
  const int *ilist, *off, *nbr;
  const double4 *xf, *vr;
  const int *ty;
  const double *en;
  double4 *fo;
  double *de;
  int accum;
  const Coefs *cf;
  double gx, gy, gz;
  double *virial;
  int nojside = 0;  // HALF: i share only, no atomics (two-pass reverse-list mode)
  // setup step, full list: owned atoms' vest before setup_pre_force, ghosts' vest as
  // borders() left it (k_force's setup comment); nullptr otherwise
  const double4 *vso = nullptr, *vsg = nullptr;
};

template <int G, int DIM, int VISC, int MODE, bool NT1>
inline void launch_force_t(hipStream_t s, const ForceArgs &a) {
  hipLaunchKernelGGL((k_force<G, DIM, VISC, MODE, NT1>), dim3(grid_for_rows(a.inum, G)),
                     dim3(256), 0, s, a.inum, a.nlocal, a.newton, a.ilist, a.off, a.nbr, a.xf,
                     a.vr, a.ty, a.en, a.fo, a.de, a.accum, a.cf, a.gx, a.gy, a.gz, a.virial,
                     a.nojside, a.vso, a.vsg);
}

template <int G, int DIM, bool NT1>
inline void launch_force_gdn(hipStream_t s, int visc, int mode, const ForceArgs &a) {
  const bool mor = visc == SPH_VISC_MORRIS;
  switch (mode) {
    case M_TAIT:
      if (mor) launch_force_t<G, DIM, 1, M_TAIT, NT1>(s, a);
      else launch_force_t<G, DIM, 0, M_TAIT, NT1>(s, a);
      break;
    case M_TAIT | M_HEAT:
      if (mor) launch_force_t<G, DIM, 1, M_TAIT | M_HEAT, NT1>(s, a);
      else launch_force_t<G, DIM, 0, M_TAIT | M_HEAT, NT1>(s, a);
      break;
    case M_HEAT: launch_force_t<G, DIM, 0, M_HEAT, NT1>(s, a); break;
    case M_TAIT | M_HALF:
      if (mor) launch_force_t<G, DIM, 1, M_TAIT | M_HALF, NT1>(s, a);
      else launch_force_t<G, DIM, 0, M_TAIT | M_HALF, NT1>(s, a);
      break;
    case M_TAIT | M_HEAT | M_HALF:
      if (mor) launch_force_t<G, DIM, 1, M_TAIT | M_HEAT | M_HALF, NT1>(s, a);
      else launch_force_t<G, DIM, 0, M_TAIT | M_HEAT | M_HALF, NT1>(s, a);
      break;
    case M_HEAT | M_HALF: launch_force_t<G, DIM, 0, M_HEAT | M_HALF, NT1>(s, a); break;
    default: SPH_REQUIRE(false, SPH_HIP_EINVAL, "unsupported force mode %d", mode);
  }
}

template <int G>
inline void launch_force_g(int dim, bool nt1, hipStream_t s, int visc, int mode,
                           const ForceArgs &a) {
  if (dim == 3) {
    if (nt1) launch_force_gdn<G, 3, true>(s, visc, mode, a);
    else launch_force_gdn<G, 3, false>(s, visc, mode, a);
  } else {
    if (nt1) launch_force_gdn<G, 2, true>(s, visc, mode, a);
    else launch_force_gdn<G, 2, false>(s, visc, mode, a);
  }
}

inline void launch_force(int dim, bool nt1, hipStream_t s, int visc, int mode,
                         const ForceArgs &a) {
  if (a.inum <= 0) return;
  switch (group_lanes()) {
    case 4: launch_force_g<4>(dim, nt1, s, visc, mode, a); break;
    case 16: launch_force_g<16>(dim, nt1, s, visc, mode, a); break;
    default: launch_force_g<8>(dim, nt1, s, visc, mode, a); break;
  }
}

}  // namespace sph
