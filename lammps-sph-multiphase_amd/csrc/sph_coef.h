// sph_coef.h -- build the device coefficient records from LAMMPS-style tables.
// Each builder mirrors the style's coeff()+init_one()+Pair::init() semantics: the caller
// gives (ntypes+1)^2 tables whose upper triangle (j >= i) was set by pair_coeff; the
// lower triangle is mirrored as init_one() does, and cutsq = cut*cut (pair.cpp:221-229).
#pragma once
#include <cmath>

#include "sph_kernels.h"

namespace sph {

inline double upper(const double *t, int nt, int i, int j) {
  return (j >= i) ? t[i * (nt + 1) + j] : t[j * (nt + 1) + i];
}

// pair_sph_rhosum.cpp:116-138 (self) and :172-192 (pair); quadric kernel norms
inline void coef_rhosum(Coefs &c, int dim, int nt, const double *cut, const double *mass) {
  for (int i = 1; i <= nt; i++) {
    const double h = upper(cut, nt, i, i);
    const double wf = (dim == 3) ? 2.1541870227086614782 / (h * h * h)
                                 : 1.5915494309189533576e0 / (h * h);
    c.self_rho[i] = h > 0.0 ? mass[i] * wf : 0.0;
    // no pair of this type has a rhosum coefficient: the type is skipped (hybrid/overlay)
    bool any = false;
    for (int j = 1; j <= nt; j++) any = any || upper(cut, nt, i, j) > 0.0;
    if (!any) c.rho_keep |= 1 << i;
    for (int j = 1; j <= nt; j++) {
      const double hh = upper(cut, nt, i, j);
      const double ih = 1.0 / hh, ihsq = ih * ih;
      RhoPair &r = c.rho[i * (nt + 1) + j];
      r.cutsq = hh * hh;
      r.ihsq = ihsq;
      r.mK = mass[j] * ((dim == 3) ? 2.1541870227086614782e0 * ihsq * ih
                                   : 1.5915494309189533576e0 * ihsq);
      // a pair without coefficients (cut 0) contributes nothing: finite zero factors, as
      // the kernels weight every pair arithmetically instead of branching on the cut
      if (hh <= 0.0) r = RhoPair{0.0, 0.0, 0.0};
    }
  }
}

// pair_sph_taitwater.cpp:136-191 / pair_sph_taitwater_morris.cpp:134-191
inline void coef_tait(Coefs &c, int dim, int nt, int visc_variant, const double *rho0,
                      const double *c0, const double *B, const double *visc,
                      const double *cut, const double *mass) {
  for (int i = 0; i <= nt; i++) {
    c.rho0[i] = rho0[i];
    c.B[i] = B[i];
  }
  for (int i = 1; i <= nt; i++)
    for (int j = 1; j <= nt; j++) {
      const double h = upper(cut, nt, i, j);
      const double ih = 1.0 / h, ihsq = ih * ih;
      TaitPair &t = c.tait[i * (nt + 1) + j];
      t.cutsq = h * h;
      t.h = h;
      t.wK = (dim == 3) ? -25.066903536973515383e0 * ihsq * ihsq * ihsq * ih
                        : -19.098593171027440292e0 * ihsq * ihsq * ihsq;
      t.mm = -mass[i] * mass[j];
      t.mj = mass[j];
      t.mi = mass[i];
      const double v = upper(visc, nt, i, j);
      t.viscC = (visc_variant == SPH_VISC_MONAGHAN) ? -v * (c0[i] + c0[j]) * h : 2 * v;
      t.eps = 0.01 * h * h;
      if (h <= 0.0) {  // no coefficients: zero weight, finite factors (see coef_rhosum)
        t.wK = 0.0;
        t.viscC = 0.0;
        t.eps = 1.0;
      }
    }
}

// pair_sph_heatconduction.cpp:103-124
inline void coef_heat(Coefs &c, int dim, int nt, const double *alpha, const double *cut,
                      const double *mass) {
  for (int i = 1; i <= nt; i++)
    for (int j = 1; j <= nt; j++) {
      const double h = upper(cut, nt, i, j);
      const double ih = 1.0 / h, ihsq = ih * ih;
      HeatPair &p = c.heat[i * (nt + 1) + j];
      p.cutsq = h * h;
      p.h = h;
      p.wK = (dim == 3) ? -25.066903536973515383e0 * ihsq * ihsq * ihsq * ih
                        : -19.098593171027440292e0 * ihsq * ihsq * ihsq;
      p.hmD = 2.0 * mass[i] * mass[j] / (mass[i] + mass[j]) * upper(alpha, nt, i, j);
      if (h <= 0.0) p.wK = 0.0;  // no coefficients (see coef_rhosum)
    }
}

// neighbor.cpp:251-268: cutoff = sqrt(cutsq) with cutsq = cut*cut, cut += skin, squared
// margin: the block path's inner rows keep pairs within cut + margin (k_blk_inner)
inline double coef_cutneigh(Coefs &c, int nt, const double *cutmax, double skin,
                            double margin = 0.0) {
  double cmax = 0.0;
  for (int i = 1; i <= nt; i++)
    for (int j = 1; j <= nt; j++) {
      const double cu = upper(cutmax, nt, i, j);
      const double cutoff = std::sqrt(cu * cu);
      const double cut = cutoff + (cutoff > 0.0 ? skin : 0.0);
      c.cutneighsq[i * (nt + 1) + j] = cut * cut;
      const double ci = cutoff + (cutoff > 0.0 ? margin : 0.0);
      c.cutinsq[i * (nt + 1) + j] = ci * ci;
      if (cut > cmax) cmax = cut;
    }
  return cmax;
}

}  // namespace sph
