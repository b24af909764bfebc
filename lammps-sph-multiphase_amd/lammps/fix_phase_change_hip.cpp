/* ----------------------------------------------------------------------------------------
   fix phase_change/hip -- see fix_phase_change_hip.h.  pre_exchange() follows
   FixPhaseChange::pre_exchange (fix_phase_change.cpp:167-352): the engine returns the new
   particles and the mass taken from the donors; atom creation, the reverse comm of that
   mass, and the natoms/tag bookkeeping stay with LAMMPS exactly as in the reference.
------------------------------------------------------------------------------------------ */
#include "fix_phase_change_hip.h"

#include <cstdlib>
#include <cstring>
#include <vector>

#include "atom.h"
#include "atom_vec.h"
#include "comm.h"
#include "domain.h"
#include "error.h"
#include "force.h"
#include "memory.h"
#include "modify.h"
#include "neigh_list.h"
#include "neigh_request.h"
#include "neighbor.h"
#include "pair_sph_hip.h"
#include "region.h"
#include "sph_hip.h"
#include "update.h"

using namespace LAMMPS_NS;
using namespace FixConst;

FixPhaseChangeHIP::FixPhaseChangeHIP(LAMMPS *lmp, int narg, char **arg)
    : Fix(lmp, narg, arg), idregion(NULL), list(NULL), dmass(NULL), nmax_dmass(0) {
  comm_reverse = 1;
  int nnarg = 14;
  if (narg < nnarg) error->all(FLERR, "Illegal fix phase_change command");
  restart_global = 1;
  time_depend = 1;
  int m = 3;
  Tc = atof(arg[m++]);
  Tt = atof(arg[m++]);
  Hwv = atof(arg[m++]);
  dr = atof(arg[m++]);
  to_mass = atof(arg[m++]);
  cutoff = atof(arg[m++]);
  from_type = atoi(arg[m++]);
  to_type = atoi(arg[m++]);
  nfreq = atoi(arg[m++]);
  seed = atoi(arg[m++]);
  if (seed <= 0) error->all(FLERR, "Illegal value for seed");
  if (strcmp(arg[m++], "ENERGY") == 0) {
    energy_chance_flag = true;
    phase_change_rate = atof(arg[m++]);
    nnarg = 15;
  } else {
    energy_chance_flag = false;
    change_chance = atof(arg[m - 1]);
    if (change_chance < 0) error->all(FLERR, "Illegal value for change_chance");
  }
  iregion = -1;
  maxattempt = 10;
  for (int iarg = nnarg; iarg < narg;) {   // FixPhaseChange::options, :358-390
    if (strcmp(arg[iarg], "region") == 0 && iarg + 2 <= narg) {
      iregion = domain->find_region(arg[iarg + 1]);
      if (iregion == -1) error->all(FLERR, "Region ID for fix phase_change does not exist");
      idregion = new char[strlen(arg[iarg + 1]) + 1];
      strcpy(idregion, arg[iarg + 1]);
      iarg += 2;
    } else if (strcmp(arg[iarg], "attempt") == 0 && iarg + 2 <= narg) {
      maxattempt = atoi(arg[iarg + 1]);
      iarg += 2;
    } else if (strcmp(arg[iarg], "units") == 0 && iarg + 2 <= narg) {
      // the reference rejects 'units lattice' itself (fix_phase_change.cpp:381-386), and its
      // scaleflag (:83) is read nowhere: no length of the fix is lattice-scaled either way
      if (strcmp(arg[iarg + 1], "lattice") == 0)
        error->all(FLERR, "Illegal fix phase_change command: 'units lattice' is not implemented");
      else if (strcmp(arg[iarg + 1], "box") != 0)
        error->all(FLERR, "Illegal fix phase_change command");
      iarg += 2;
    } else {
      error->all(FLERR, "Illegal fix phase_change command");
    }
  }
  if (iregion == -1) error->all(FLERR, "Must specify a region in fix phase_change");
  if (domain->regions[iregion]->bboxflag == 0)
    error->all(FLERR, "Fix phase_change region does not support a bounding box");
  if (domain->regions[iregion]->dynamic_check())
    error->all(FLERR, "Fix phase_change region cannot be dynamic");
  // the region's extent must lie inside the box (:97-114)
  Region *r = domain->regions[iregion];
  const double *lo = domain->triclinic ? domain->boxlo_bound : domain->boxlo;
  const double *hi = domain->triclinic ? domain->boxhi_bound : domain->boxhi;
  if (r->extent_xlo < lo[0] || r->extent_xhi > hi[0] || r->extent_ylo < lo[1] ||
      r->extent_yhi > hi[1] || r->extent_zlo < lo[2] || r->extent_zhi > hi[2])
    error->all(FLERR, "Phase change region extends outside simulation box");
  rng = seed;  // RanPark(lmp, seed)
  force_reneighbor = 1;
  next_reneighbor = update->ntimestep + 1;
}

FixPhaseChangeHIP::~FixPhaseChangeHIP() {
  delete[] idregion;
  memory->destroy(dmass);
}

int FixPhaseChangeHIP::setmask() { return PRE_EXCHANGE; }

void FixPhaseChangeHIP::init() {
  iregion = domain->find_region(idregion);
  if (iregion == -1) error->all(FLERR, "Region ID for fix phase_change does not exist");
  sph_hip_new_run();
  // full list, rebuilt whenever re-neighboring occurs (fix_phase_change.cpp:151-156)
  int irequest = neighbor->request((void *)this);
  neighbor->requests[irequest]->pair = 0;
  neighbor->requests[irequest]->fix = 1;
  neighbor->requests[irequest]->half = 0;
  neighbor->requests[irequest]->full = 1;
}

void FixPhaseChangeHIP::init_list(int, NeighList *ptr) { list = ptr; }

void FixPhaseChangeHIP::pre_exchange() {
  if (next_reneighbor != update->ntimestep) return;
  const int nlocal = atom->nlocal;
  const int nall = nlocal + atom->nghost;
  if (nall > nmax_dmass) {
    nmax_dmass = atom->nmax;
    memory->destroy(dmass);
    memory->create(dmass, nmax_dmass, "phase_change/hip:dmass");
  }
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_phasechange_params p;
  memset(&p, 0, sizeof(p));
  p.Tc = Tc;
  p.Tt = Tt;
  p.Hwv = Hwv;
  p.dr = dr;
  p.to_mass = to_mass;
  p.cutoff = cutoff;
  p.from_type = from_type;
  p.to_type = to_type;
  p.energy_chance = energy_chance_flag ? 1 : 0;
  p.change_chance = change_chance;
  p.rate = phase_change_rate;
  p.dt = update->dt;
  p.maxattempt = maxattempt;
  for (int d = 0; d < 3; d++) {
    p.sublo[d] = domain->sublo[d];
    p.subhi[d] = domain->subhi[d];
    p.boxhi[d] = domain->boxhi[d];
    p.top[d] = comm->myloc[d] == comm->procgrid[d] - 1;
  }
  std::vector<double> rec;
  std::vector<int> parent;
  int nins = 0, cap = 64;
  for (;;) {
    const int s0 = rng;
    rec.assign((size_t)13 * cap, 0.0);
    parent.assign(cap, 0);
    std::vector<double> e_save(atom->e, atom->e + nall);
    sph_hip_stage(lmp, ctx, list, SPH_LIST_FULL, true);
    sph_hip_check(lmp,
                  sph_hip_phasechange(ctx, &p, &rng, nall ? &atom->v[0][0] : NULL,
                                      nall ? &atom->colorgradient[0][0] : NULL, atom->e, dmass,
                                      cap, &nins, rec.data(), parent.data()),
                  "sph_hip_phasechange");
    if (nins <= cap) break;
    rng = s0;  // more insertions than room: replay the same stream with enough room
    std::copy(e_save.begin(), e_save.end(), atom->e);
    cap = nins;
  }
  for (int k = 0; k < nins; k++) {   // insert_one_atom (:425-462) + the new atom's fields (:303-320)
    const double *r = &rec[(size_t)13 * k];
    double coord[3] = {r[0], r[1], r[2]};
    atom->avec->create_atom(to_type, coord);
    const int m = atom->nlocal - 1;
    atom->type[m] = to_type;
    atom->mask[m] = 1 | groupbit;
    for (int j = 0; j < modify->nfix; j++)
      if (modify->fix[j]->create_attribute) modify->fix[j]->set_arrays(m);
    for (int d = 0; d < 3; d++) {
      atom->v[m][d] = r[3 + d];
      atom->vest[m][d] = r[6 + d];
    }
    atom->e[m] = r[9];
    atom->rmass[m] = r[10];
    atom->rho[m] = r[11];
    atom->cv[m] = r[12];
  }
  comm->reverse_comm_fix(this);   // ghost donors' mass back to their owners
  sph_hip_check(lmp, sph_hip_phasechange_finish(nlocal, dmass, atom->rmass, atom->e),
                "sph_hip_phasechange_finish");
  next_reneighbor += nfreq;
  int ninsall;
  MPI_Allreduce(&nins, &ninsall, 1, MPI_INT, MPI_SUM, world);
  if (ninsall > 0) {
    atom->natoms += ninsall;
    if (atom->tag_enable) atom->tag_extend();
    atom->nghost = 0;
    if (atom->map_style) {
      atom->map_init();
      atom->map_set();
    }
  }
}

int FixPhaseChangeHIP::pack_reverse_comm(int n, int first, double *buf) {
  int m = 0;
  for (int i = first; i < first + n; i++) buf[m++] = dmass[i];
  return m;
}

void FixPhaseChangeHIP::unpack_reverse_comm(int n, int *list_, double *buf) {
  int m = 0;
  for (int i = 0; i < n; i++) dmass[list_[i]] += buf[m++];
}
