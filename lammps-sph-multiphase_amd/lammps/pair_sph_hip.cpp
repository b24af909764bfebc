/* ----------------------------------------------------------------------------------------
   LAMMPS-side binding of the MI355X USER-SPH engine: compute() of the sph/<style>/hip pair styles.
   Each compute() stages the rank's atoms and the style's NeighList into the device
   context and calls the style's C-ABI entry point (include/sph_hip.h); the loops it
   replaces are cited per class.  Everything else (settings, coeff, init_one, comm) is the
   reference style's own code, inherited.
------------------------------------------------------------------------------------------ */
#include "pair_sph_hip.h"

#include <cmath>
#include <cstdio>
#include <vector>

#include "atom.h"
#include "comm.h"
#include "domain.h"
#include "error.h"
#include "force.h"
#include "memory.h"
#include "neigh_list.h"
#include "neighbor.h"
#include "pair.h"
#include "sph_hip.h"
#include "update.h"

using namespace LAMMPS_NS;

namespace {
sph_hip_ctx *g_ctx = NULL;
// what the context's atoms were staged at: a later compute of the same step (hybrid/overlay
// sub-styles after forward_comm_pair) restages rho only.  Within one run borders happen only
// with a list build, so (ntimestep, neighbor->ncalls, nlocal, nghost) pins the atom set and
// positions; across runs it does not (Verlet::setup and setup_minimal reset ncalls to 0,
// verlet.cpp:113, :172, and FixMeso::setup_pre_force rewrites vest), so the key also holds
// the run epoch that every init (Pair::init -> init_style, Fix::init) advances.
struct StageKey {
  bigint epoch, step, ncalls;
  int nlocal, nghost;
  bool mp;
};
bigint g_epoch = 0;
StageKey g_key = {-1, -1, -1, -1, -1, false};
// lists built on the device (sph_hip_build_list) instead of copied from the NeighList
bool g_device_lists = true;
std::vector<double> g_cns;
// the device list of a kind is reused while this key is unchanged
int64_t list_key(LAMMPS *lmp) { return (int64_t)(g_epoch << 40) + (int64_t)lmp->neighbor->ncalls; }
}

void LAMMPS_NS::sph_hip_new_run() { g_epoch++; }

extern "C" void sph_hip_shim_set_device_lists(int on) { g_device_lists = on != 0; }

sph_hip_ctx *LAMMPS_NS::sph_hip_rank_ctx(LAMMPS *lmp) {
  // one context per rank; made again when the system it was made for changed (a `clear`
  // followed by a new box with another dimension / number of types / newton setting)
  static int made_for[3] = {0, 0, 0};
  const int want[3] = {lmp->domain->dimension, lmp->atom->ntypes, lmp->force->newton_pair};
  if (g_ctx && (want[0] != made_for[0] || want[1] != made_for[1] || want[2] != made_for[2])) {
    sph_hip_destroy(g_ctx);
    g_ctx = NULL;
    g_key.epoch = -1;
  }
  if (!g_ctx) {
    for (int k = 0; k < 3; k++) made_for[k] = want[k];
    const int ndev = sph_hip_device_count();
    if (ndev < 1) lmp->error->one(FLERR, "sph/<style>/hip styles need a HIP device");
    sph_hip_check(lmp,
                  sph_hip_create(lmp->comm->me % ndev, lmp->domain->dimension,
                                 lmp->atom->ntypes, lmp->force->newton_pair, &g_ctx),
                  "sph_hip_create");
  }
  return g_ctx;
}

void LAMMPS_NS::sph_hip_check(LAMMPS *lmp, int rc, const char *where) {
  if (rc == SPH_HIP_OK) return;
  char msg[1200];
  snprintf(msg, sizeof(msg), "%s failed (%d): %s", where, rc, sph_hip_last_error());
  lmp->error->one(FLERR, msg);
}

void LAMMPS_NS::sph_hip_stage(LAMMPS *lmp, sph_hip_ctx *ctx, NeighList *list, int kind,
                              bool multiphase) {
  Atom *atom = lmp->atom;
  const int nlocal = atom->nlocal, nghost = atom->nghost;
  const int nall = nlocal + nghost;
  const StageKey key = {g_epoch, lmp->update->ntimestep, lmp->neighbor->ncalls, nlocal, nghost,
                        multiphase};
  // LAMMPS' per-atom arrays as mapped host memory (sph_hip_host_arrays): the device reads
  // x / vest / rho / e and writes rho, adds f / drho / de in place over PCIe.  Registered
  // again whenever AtomVec::grow moved them (nmax or a pointer changed) and at every run
  // (a `clear` may hand out the same addresses for new arrays).
  {
    static bigint reg_epoch = -1;
    double *const p[7] = {atom->x ? &atom->x[0][0] : NULL, atom->vest ? &atom->vest[0][0] : NULL,
                          atom->rho, atom->e, atom->f ? &atom->f[0][0] : NULL, atom->drho,
                          atom->de};
    static double *reg[7] = {NULL, NULL, NULL, NULL, NULL, NULL, NULL};
    static int reg_nmax = -1;
    static sph_hip_ctx *reg_ctx = NULL;
    bool same = reg_nmax == atom->nmax && reg_ctx == ctx && reg_epoch == g_epoch;
    for (int k = 0; k < 7; k++) same = same && reg[k] == p[k];
    if (!same && atom->nmax > 0) {
      sph_hip_check(lmp, sph_hip_host_arrays(ctx, atom->nmax, p[0], p[1], p[2], p[3], p[4], p[5],
                                             p[6]),
                    "sph_hip_host_arrays");
      for (int k = 0; k < 7; k++) reg[k] = p[k];
      reg_nmax = atom->nmax;
      reg_ctx = ctx;
      reg_epoch = g_epoch;
    }
  }
  if (key.epoch == g_key.epoch && key.step == g_key.step && key.ncalls == g_key.ncalls &&
      key.nlocal == g_key.nlocal && key.nghost == g_key.nghost && (g_key.mp || !multiphase) &&
      nall && atom->rho) {
    sph_hip_check(lmp, sph_hip_atoms_rho(ctx, atom->rho), "sph_hip_atoms_rho");
  } else if (key.epoch == g_key.epoch && key.ncalls == g_key.ncalls &&
             key.nlocal == g_key.nlocal && key.nghost == g_key.nghost &&
             (g_key.mp || !multiphase) && nall) {
    // a new step of the same atom set (no reneighbor since): positions, vest, rho, e only
    sph_hip_check(lmp,
                  sph_hip_atoms_update(ctx, &atom->x[0][0], atom->vest ? &atom->vest[0][0] : NULL,
                                       atom->rho, atom->e),
                  "sph_hip_atoms_update");
    g_key = key;
  } else {
    // x and vest are memory->create 2-D arrays: contiguous nmax*3 backing (memory.h:124-137)
    sph_hip_check(lmp,
                  sph_hip_atoms(ctx, nlocal, nghost, nall ? &atom->x[0][0] : NULL,
                                (nall && atom->vest) ? &atom->vest[0][0] : NULL, atom->rho,
                                atom->e, atom->type),
                  "sph_hip_atoms");
    if (multiphase)
      sph_hip_check(lmp, sph_hip_atoms_multiphase(ctx, atom->rmass, atom->cv),
                    "sph_hip_atoms_multiphase");
    g_key = key;
  }
  // the list build is the key (run epoch + neighbor->ncalls, neighbor.cpp:1423): between
  // rebuilds the staged device copy of this kind is reused -- no host copy, no upload, and a
  // half list keeps its reverse list; sub-styles of hybrid/overlay on the other kind keep
  // theirs.  Device-list path (default): the list is built on the device from
  // the staged atoms with Neighbor::init's cutneighsq, (sqrt(pair->cutsq) + skin)^2
  // (neighbor.cpp:251-268), full_bin membership and half_from_full_newton's half.
  // Only where the device list IS the list LAMMPS would hand this caller: not for a
  // hybrid/overlay sub-style's skip list (pair_hybrid.cpp:428-485: types or type pairs the
  // sub-style has no coefficients for are left out, and its coefficient tables are
  // uninitialised there) and not with neigh_modify exclude (neighbor.cpp's exclusion tests) --
  // those take the NeighList upload below.
  Pair *pair = lmp->force->pair;
  const bool skip_list = list && (list->iskip || list->ijskip);
  if (g_device_lists && pair && pair->cutsq && !skip_list && !lmp->neighbor->exclude_setting()) {
    const int nt = atom->ntypes;
    g_cns.assign((size_t)(nt + 1) * (nt + 1), 0.0);
    for (int i = 1; i <= nt; i++)
      for (int j = 1; j <= nt; j++) {
        const double cutoff = sqrt(pair->cutsq[i][j]);
        const double cut = cutoff + (cutoff > 0.0 ? lmp->neighbor->skin : 0.0);
        g_cns[(size_t)i * (nt + 1) + j] = cut * cut;
      }
    sph_hip_check(lmp, sph_hip_build_list(ctx, kind, list_key(lmp), g_cns.data()),
                  "sph_hip_build_list");
    return;
  }
  sph_hip_check(lmp,
                sph_hip_list_keyed(ctx, kind, list_key(lmp), list->inum, list->ilist,
                                   list->numneigh, list->firstneigh),
                "sph_hip_list_keyed");
}

namespace {

// (nt+1)^2 row-major view of a memory->create 2-D table (contiguous backing)
const double *tab(double **t) { return &t[0][0]; }

// (vflag_atom / vflag_global are meaningful only after ev_setup, i.e. when evflag is set:
// Pair's constructor leaves them uninitialised, pair.cpp:684-692)
double *virial_target(LAMMPS *lmp, Pair *p) {
  if (!p->evflag) return NULL;
  if (p->vflag_atom) lmp->error->all(FLERR, "sph/<style>/hip styles do not tally per-atom virials");
  return p->vflag_global ? p->virial : NULL;
}

}  // namespace

/* pair_sph_rhosum.cpp:66-204 */
void PairSPHRhoSumHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  if (nstep != 0 && (update->ntimestep % nstep) == 0) {
    sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
    sph_hip_check(lmp, sph_hip_rhosum_coeff(ctx, tab(cut), atom->mass), "sph_hip_rhosum_coeff");
    sph_hip_stage(lmp, ctx, list, SPH_LIST_FULL, false);
    sph_hip_check(lmp, sph_hip_rhosum(ctx, atom->rho), "sph_hip_rhosum");
  }
  comm->forward_comm_pair(this);
}

/* pair_sph_taitwater.cpp:53-200 */
void PairSPHTaitwaterHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_hip_check(lmp,
                sph_hip_taitwater_coeff(ctx, SPH_VISC_MONAGHAN, rho0, soundspeed, B,
                                        tab(viscosity), tab(cut), atom->mass),
                "sph_hip_taitwater_coeff");
  sph_hip_stage(lmp, ctx, list, SPH_LIST_HALF, false);
  if (atom->nlocal + atom->nghost)
    sph_hip_check(lmp,
                  sph_hip_taitwater(ctx, &atom->f[0][0], atom->drho, atom->de,
                                    virial_target(lmp, this)),
                  "sph_hip_taitwater");
  if (vflag_fdotr) virial_fdotr_compute();
}

/* pair_sph_taitwater_morris.cpp:52-200 */
void PairSPHTaitwaterMorrisHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_hip_check(lmp,
                sph_hip_taitwater_coeff(ctx, SPH_VISC_MORRIS, rho0, soundspeed, B,
                                        tab(viscosity), tab(cut), atom->mass),
                "sph_hip_taitwater_coeff");
  sph_hip_stage(lmp, ctx, list, SPH_LIST_HALF, false);
  if (atom->nlocal + atom->nghost)
    sph_hip_check(lmp,
                  sph_hip_taitwater(ctx, &atom->f[0][0], atom->drho, atom->de,
                                    virial_target(lmp, this)),
                  "sph_hip_taitwater");
  if (vflag_fdotr) virial_fdotr_compute();
}

/* pair_sph_heatconduction.cpp:47-134 */
void PairSPHHeatConductionHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_hip_check(lmp, sph_hip_heatconduction_coeff(ctx, tab(alpha), tab(cut), atom->mass),
                "sph_hip_heatconduction_coeff");
  sph_hip_stage(lmp, ctx, list, SPH_LIST_HALF, false);
  sph_hip_check(lmp, sph_hip_heatconduction(ctx, atom->de), "sph_hip_heatconduction");
}

/* pair_sph_rhosum_multiphase.cpp:68-174 */
void PairSPHRhoSumMultiphaseHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  if (nstep != 0 && (update->ntimestep % nstep) == 0) {
    sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
    sph_hip_check(lmp, sph_hip_rhosum_multiphase_coeff(ctx, tab(cut)),
                  "sph_hip_rhosum_multiphase_coeff");
    sph_hip_stage(lmp, ctx, list, SPH_LIST_FULL, true);
    sph_hip_check(lmp, sph_hip_rhosum_multiphase(ctx, atom->rho), "sph_hip_rhosum_multiphase");
  }
  comm->forward_comm_pair(this);
}

/* pair_sph_taitwater_multiphase.cpp:55-186 */
void PairSPHTaitwaterMultiphaseHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_hip_check(lmp,
                sph_hip_taitwater_multiphase_coeff(ctx, rho0, soundspeed, gamma, rbackground,
                                                   tab(viscosity), tab(cut)),
                "sph_hip_taitwater_multiphase_coeff");
  sph_hip_stage(lmp, ctx, list, SPH_LIST_HALF, true);
  if (atom->nlocal + atom->nghost)
    sph_hip_check(lmp, sph_hip_taitwater_multiphase(ctx, &atom->f[0][0]),
                  "sph_hip_taitwater_multiphase");
  if (vflag_fdotr) virial_fdotr_compute();
}

/* pair_sph_heatconduction_phasechange.cpp:52-141 */
void PairSPHHeatConductionPhaseChangeHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_hip_check(lmp,
                sph_hip_heatconduction_phasechange_coeff(ctx, tab(alpha), &fixflag[0][0],
                                                         tab(tc), tab(cut)),
                "sph_hip_heatconduction_phasechange_coeff");
  sph_hip_stage(lmp, ctx, list, SPH_LIST_HALF, true);
  sph_hip_check(lmp, sph_hip_heatconduction_phasechange(ctx, atom->de),
                "sph_hip_heatconduction_phasechange");
}

/* pair_sph_colorgradient.cpp:70-191 */
void PairSPHColorGradientHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  if (nstep != 0 && (update->ntimestep % nstep) == 0) {
    sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
    sph_hip_check(lmp, sph_hip_colorgradient_coeff(ctx, tab(alpha), tab(cut)),
                  "sph_hip_colorgradient_coeff");
    sph_hip_stage(lmp, ctx, list, SPH_LIST_FULL, true);
    if (atom->nlocal)
      sph_hip_check(lmp, sph_hip_colorgradient(ctx, &atom->colorgradient[0][0]),
                    "sph_hip_colorgradient");
  }
  comm->forward_comm_pair(this);
}

/* pair_sph_surfacetension.cpp:50-192 (no virial tally there either) */
void PairSPHSurfaceTensionHIP::compute(int eflag, int vflag) {
  if (eflag || vflag) ev_setup(eflag, vflag);
  else evflag = vflag_fdotr = 0;
  sph_hip_ctx *ctx = sph_hip_rank_ctx(lmp);
  sph_hip_check(lmp, sph_hip_surfacetension_coeff(ctx, tab(cut)), "sph_hip_surfacetension_coeff");
  sph_hip_stage(lmp, ctx, list, SPH_LIST_HALF, true);
  if (atom->nlocal + atom->nghost)
    sph_hip_check(lmp,
                  sph_hip_surfacetension(ctx, &atom->colorgradient[0][0], &atom->f[0][0]),
                  "sph_hip_surfacetension");
}

/* Pair::init -> init_style (pair.cpp:211): the reference style's own request, then a new run
   epoch for the device mirrors */
void PairSPHRhoSumHIP::init_style() {
  PairSPHRhoSum::init_style();
  sph_hip_new_run();
}
void PairSPHTaitwaterHIP::init_style() {
  PairSPHTaitwater::init_style();
  sph_hip_new_run();
}
void PairSPHTaitwaterMorrisHIP::init_style() {
  PairSPHTaitwaterMorris::init_style();
  sph_hip_new_run();
}
void PairSPHHeatConductionHIP::init_style() {
  PairSPHHeatConduction::init_style();
  sph_hip_new_run();
}
void PairSPHRhoSumMultiphaseHIP::init_style() {
  PairSPHRhoSumMultiphase::init_style();
  sph_hip_new_run();
}
void PairSPHTaitwaterMultiphaseHIP::init_style() {
  PairSPHTaitwaterMultiphase::init_style();
  sph_hip_new_run();
}
void PairSPHHeatConductionPhaseChangeHIP::init_style() {
  PairSPHHeatConductionPhaseChange::init_style();
  sph_hip_new_run();
}
void PairSPHColorGradientHIP::init_style() {
  PairSPHColorGradient::init_style();
  sph_hip_new_run();
}
void PairSPHSurfaceTensionHIP::init_style() {
  PairSPHSurfaceTension::init_style();
  sph_hip_new_run();
}
