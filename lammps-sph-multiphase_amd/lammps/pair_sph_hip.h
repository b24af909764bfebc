/* -*- c++ -*- ----------------------------------------------------------------------------
   LAMMPS-side binding of the MI355X USER-SPH engine (include/sph_hip.h, pair-style layer).
   Drop into src/USER-SPH next to the reference styles; "-sf hip" or "pair_style
   sph/taitwater/hip" selects them (force.cpp:148-166).  Each class inherits the reference
   style's settings()/coeff()/init_one()/init_style() unchanged (same arguments, same error
   messages) and replaces only compute() (pair.h:135) by a call through the C ABI.
------------------------------------------------------------------------------------------ */
#ifdef PAIR_CLASS

PairStyle(sph/rhosum/hip,PairSPHRhoSumHIP)
PairStyle(sph/taitwater/hip,PairSPHTaitwaterHIP)
PairStyle(sph/taitwater/morris/hip,PairSPHTaitwaterMorrisHIP)
PairStyle(sph/heatconduction/hip,PairSPHHeatConductionHIP)
PairStyle(sph/rhosum/multiphase/hip,PairSPHRhoSumMultiphaseHIP)
PairStyle(sph/taitwater/multiphase/hip,PairSPHTaitwaterMultiphaseHIP)
PairStyle(sph/heatconduction/phasechange/hip,PairSPHHeatConductionPhaseChangeHIP)
PairStyle(sph/colorgradient/hip,PairSPHColorGradientHIP)
PairStyle(sph/surfacetension/hip,PairSPHSurfaceTensionHIP)

#else

#ifndef LMP_PAIR_SPH_HIP_H
#define LMP_PAIR_SPH_HIP_H

#include "pair_sph_colorgradient.h"
#include "pair_sph_heatconduction.h"
#include "pair_sph_heatconduction_phasechange.h"
#include "pair_sph_rhosum.h"
#include "pair_sph_rhosum_multiphase.h"
#include "pair_sph_surfacetension.h"
#include "pair_sph_taitwater.h"
#include "pair_sph_taitwater_morris.h"
#include "pair_sph_taitwater_multiphase.h"

struct sph_hip_ctx;

namespace LAMMPS_NS {

// one device context per MPI rank, shared by every sph/<style>/hip style and fix
sph_hip_ctx *sph_hip_rank_ctx(class LAMMPS *lmp);
// stage atom->x/vest/rho/e/type (and rmass/cv for meso/multiphase) plus a NeighList
void sph_hip_stage(class LAMMPS *lmp, sph_hip_ctx *ctx, class NeighList *list, int kind,
                   bool multiphase);
// turn an ABI status into error->one (src/GPU/pair_lj_cut_gpu.cpp:114-115 precedent)
void sph_hip_check(class LAMMPS *lmp, int rc, const char *where);
// a new run/minimize/rerun is being set up (Pair::init -> init_style, Fix::init): atoms and
// lists staged before it are never reused after it, even at the same timestep and list
// build count (Verlet::setup resets neighbor->ncalls, verlet.cpp:113)
void sph_hip_new_run();

class PairSPHRhoSumHIP : public PairSPHRhoSum {
 public:
  PairSPHRhoSumHIP(class LAMMPS *lmp) : PairSPHRhoSum(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHTaitwaterHIP : public PairSPHTaitwater {
 public:
  PairSPHTaitwaterHIP(class LAMMPS *lmp) : PairSPHTaitwater(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHTaitwaterMorrisHIP : public PairSPHTaitwaterMorris {
 public:
  PairSPHTaitwaterMorrisHIP(class LAMMPS *lmp) : PairSPHTaitwaterMorris(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHHeatConductionHIP : public PairSPHHeatConduction {
 public:
  PairSPHHeatConductionHIP(class LAMMPS *lmp) : PairSPHHeatConduction(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHRhoSumMultiphaseHIP : public PairSPHRhoSumMultiphase {
 public:
  PairSPHRhoSumMultiphaseHIP(class LAMMPS *lmp) : PairSPHRhoSumMultiphase(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHTaitwaterMultiphaseHIP : public PairSPHTaitwaterMultiphase {
 public:
  PairSPHTaitwaterMultiphaseHIP(class LAMMPS *lmp) : PairSPHTaitwaterMultiphase(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHHeatConductionPhaseChangeHIP : public PairSPHHeatConductionPhaseChange {
 public:
  PairSPHHeatConductionPhaseChangeHIP(class LAMMPS *lmp)
      : PairSPHHeatConductionPhaseChange(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHColorGradientHIP : public PairSPHColorGradient {
 public:
  PairSPHColorGradientHIP(class LAMMPS *lmp) : PairSPHColorGradient(lmp) {}
  void compute(int, int);
  void init_style();
};

class PairSPHSurfaceTensionHIP : public PairSPHSurfaceTension {
 public:
  PairSPHSurfaceTensionHIP(class LAMMPS *lmp) : PairSPHSurfaceTension(lmp) {}
  void compute(int, int);
  void init_style();
};

}  // namespace LAMMPS_NS

#endif
#endif
