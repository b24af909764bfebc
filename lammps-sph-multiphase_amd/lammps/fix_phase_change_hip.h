/* -*- c++ -*- ----------------------------------------------------------------------------
   fix phase_change/hip: FixPhaseChange (fix_phase_change.cpp) with pre_exchange() run by
   the MI355X engine (include/sph_hip.h section 1c).  Same arguments and errors as the
   reference (fix_phase_change.cpp:46-121, options :358-390); FixPhaseChange's members are
   private, so the argument parsing is restated here instead of inherited.
------------------------------------------------------------------------------------------ */
#ifdef FIX_CLASS

FixStyle(phase_change/hip,FixPhaseChangeHIP)

#else

#ifndef LMP_FIX_PHASE_CHANGE_HIP_H
#define LMP_FIX_PHASE_CHANGE_HIP_H

#include "fix.h"

namespace LAMMPS_NS {

class FixPhaseChangeHIP : public Fix {
 public:
  FixPhaseChangeHIP(class LAMMPS *, int, char **);
  ~FixPhaseChangeHIP();
  int setmask();
  void init();
  void init_list(int, class NeighList *);
  void pre_exchange();
  int pack_reverse_comm(int, int, double *);
  void unpack_reverse_comm(int, int *, double *);

 private:
  int from_type, to_type, nfreq, seed, iregion, maxattempt;
  char *idregion;
  double Tc, Tt, Hwv, dr, to_mass, cutoff, change_chance, phase_change_rate;
  bool energy_chance_flag;
  int rng;                   // Park-Miller state (RanPark::seed)
  class NeighList *list;
  double *dmass;
  int nmax_dmass;
};

}  // namespace LAMMPS_NS

#endif
#endif
