// sph_dispatch.h -- runtime -> template dispatch for the pair kernels.
#pragma once
#include "sph_kernels.h"
#include "sph_util.h"

namespace sph {

// lanes per neighbor-list row; SPH_GROUP env var overrides (tuning), default 8
int group_lanes();

inline unsigned grid_for_rows(long rows, int G, int block = 256) {
  return (unsigned)((rows * (long)G + block - 1) / block);
}

template <int G>
inline void launch_rhosum_g(int dim, bool eos, hipStream_t s, int inum, const int *ilist,
                            const int *off, const int *nbr, const double4 *xt, double4 *vr,
                            double2 *aux, double *rho_out, const Coefs *cf) {
  dim3 grid(grid_for_rows(inum, G)), block(256);
  if (dim == 3) {
    if (eos)
      hipLaunchKernelGGL((k_rhosum<G, 3, true>), grid, block, 0, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf);
    else
      hipLaunchKernelGGL((k_rhosum<G, 3, false>), grid, block, 0, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf);
  } else {
    if (eos)
      hipLaunchKernelGGL((k_rhosum<G, 2, true>), grid, block, 0, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf);
    else
      hipLaunchKernelGGL((k_rhosum<G, 2, false>), grid, block, 0, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf);
  }
}

inline void launch_rhosum(int dim, bool eos, hipStream_t s, int inum, const int *ilist,
                          const int *off, const int *nbr, const double4 *xt, double4 *vr,
                          double2 *aux, double *rho_out, const Coefs *cf) {
  if (inum <= 0) return;
  switch (group_lanes()) {
    case 4: launch_rhosum_g<4>(dim, eos, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf); break;
    case 16: launch_rhosum_g<16>(dim, eos, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf); break;
    case 32: launch_rhosum_g<32>(dim, eos, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf); break;
    default: launch_rhosum_g<8>(dim, eos, s, inum, ilist, off, nbr, xt, vr, aux, rho_out, cf); break;
  }
}

struct ForceArgs {
  int inum, nlocal, newton;
  const int *ilist, *off, *nbr;
  const double4 *xt, *vr;
  const double2 *aux;
  double4 *fo;
  double *de;
  int accum;
  const Coefs *cf;
  double gx, gy, gz;
  double *virial;
};

template <int G, int DIM, int VISC, int MODE>
inline void launch_force_t(hipStream_t s, const ForceArgs &a) {
  dim3 grid(grid_for_rows(a.inum, G)), block(256);
  hipLaunchKernelGGL((k_force<G, DIM, VISC, MODE>), grid, block, 0, s, a.inum, a.nlocal, a.newton,
                     a.ilist, a.off, a.nbr, a.xt, a.vr, a.aux, a.fo, a.de, a.accum, a.cf, a.gx,
                     a.gy, a.gz, a.virial);
}

template <int G, int DIM>
inline void launch_force_gd(hipStream_t s, int visc, int mode, const ForceArgs &a) {
  // supported mode combinations
  if (mode == M_TAIT) {
    if (visc == SPH_VISC_MORRIS) launch_force_t<G, DIM, 1, M_TAIT>(s, a);
    else launch_force_t<G, DIM, 0, M_TAIT>(s, a);
  } else if (mode == (M_TAIT | M_HEAT)) {
    if (visc == SPH_VISC_MORRIS) launch_force_t<G, DIM, 1, M_TAIT | M_HEAT>(s, a);
    else launch_force_t<G, DIM, 0, M_TAIT | M_HEAT>(s, a);
  } else if (mode == M_HEAT) {
    launch_force_t<G, DIM, 0, M_HEAT>(s, a);
  } else if (mode == (M_TAIT | M_HALF)) {
    if (visc == SPH_VISC_MORRIS) launch_force_t<G, DIM, 1, M_TAIT | M_HALF>(s, a);
    else launch_force_t<G, DIM, 0, M_TAIT | M_HALF>(s, a);
  } else if (mode == (M_TAIT | M_HEAT | M_HALF)) {
    if (visc == SPH_VISC_MORRIS) launch_force_t<G, DIM, 1, M_TAIT | M_HEAT | M_HALF>(s, a);
    else launch_force_t<G, DIM, 0, M_TAIT | M_HEAT | M_HALF>(s, a);
  } else if (mode == (M_HEAT | M_HALF)) {
    launch_force_t<G, DIM, 0, M_HEAT | M_HALF>(s, a);
  } else {
    SPH_REQUIRE(false, SPH_HIP_EINVAL, "unsupported force mode %d", mode);
  }
}

template <int G>
inline void launch_force_g(int dim, hipStream_t s, int visc, int mode, const ForceArgs &a) {
  if (dim == 3) launch_force_gd<G, 3>(s, visc, mode, a);
  else launch_force_gd<G, 2>(s, visc, mode, a);
}

inline void launch_force(int dim, hipStream_t s, int visc, int mode, const ForceArgs &a) {
  if (a.inum <= 0) return;
  switch (group_lanes()) {
    case 4: launch_force_g<4>(dim, s, visc, mode, a); break;
    case 16: launch_force_g<16>(dim, s, visc, mode, a); break;
    case 32: launch_force_g<32>(dim, s, visc, mode, a); break;
    default: launch_force_g<8>(dim, s, visc, mode, a); break;
  }
}

}  // namespace sph
