/*
 * sph_oracle.h -- CPU restatement of the USER-SPH hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU baseline -- never as the
 * thing measured or shipped.  The product path (libsph_hip.so) never links it.
 *
 * Every function restates one reference routine (paths relative to /root/reference):
 *   orc_pbc                    src/domain.cpp:478-560          Domain::pbc (orthogonal box)
 *   orc_borders                src/comm_brick.cpp:151-380,696-864  setup()+borders(), 1 proc
 *   orc_forward_comm           src/USER-SPH/atom_vec_meso.cpp:246-288  pack_comm/unpack_comm
 *   orc_reverse_comm           src/USER-SPH/atom_vec_meso.cpp:387-418  pack/unpack_reverse
 *   orc_neigh_full             src/neigh_full.cpp:241-344      Neighbor::full_bin membership
 *   orc_neigh_half_from_full   src/neigh_derive.cpp:83-150     Neighbor::half_from_full_newton
 *   orc_cutneighsq             src/neighbor.cpp:251-268 + src/pair.cpp:221-229
 *   orc_rhosum                 src/USER-SPH/pair_sph_rhosum.cpp:66-204
 *   orc_taitwater              src/USER-SPH/pair_sph_taitwater.cpp:53-200
 *   orc_taitwater_morris       src/USER-SPH/pair_sph_taitwater_morris.cpp:52-200
 *   orc_heatconduction         src/USER-SPH/pair_sph_heatconduction.cpp:47-134
 *   orc_meso_initial/final     src/USER-SPH/fix_meso.cpp:91-180
 *   orc_kernel_quintic{2,3}d, orc_dw_quintic{2,3}d  src/USER-SPH/sph_kernel_quintic.cpp:17-73
 *   orc_rhosum_multiphase      src/USER-SPH/pair_sph_rhosum_multiphase.cpp:68-174
 *   orc_taitwater_multiphase   src/USER-SPH/pair_sph_taitwater_multiphase.cpp:55-186
 *   orc_heatconduction_phasechange src/USER-SPH/pair_sph_heatconduction_phasechange.cpp:52-141
 *   orc_colorgradient          src/USER-SPH/pair_sph_colorgradient.cpp:70-191
 *   orc_surfacetension         src/USER-SPH/pair_sph_surfacetension.cpp:50-192
 *
 * Data model mirrors LAMMPS: per-atom arrays hold nlocal owned atoms followed by nghost
 * ghosts; vectors (x, v, vest, f) are AoS double[n][3] like atom->x's contiguous backing
 * (src/memory.h:124-137); per-type tables are (ntypes+1) long and per-type-pair tables are
 * (ntypes+1)^2 row-major, 1-based like LAMMPS.  Neighbor lists are CSR: for owned atom i
 * (ilist is the identity, as full_bin builds it) its neighbors are neigh[off[i] .. off[i+1]).
 */
#ifndef SPH_ORACLE_H
#define SPH_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int dim;              /* 2 or 3 (domain->dimension) */
  double boxlo[3];
  double boxhi[3];
  int periodic[3];
} orc_domain;

/* ---- domain / comm ---------------------------------------------------------------- */
void orc_pbc(const orc_domain *d, int nlocal, double *x);

/* Build ghosts for a single process (procgrid 1x1x1) exactly in CommBrick's swap order.
   x/type must have room for nmax atoms; ghosts are appended after nlocal.
   ghost_owner[g]  = owned atom the ghost images (after composing hops),
   ghost_image[3g+k] = -1/0/+1 periodic image in dim k.
   Returns nghost, or -1 if nmax would be exceeded. */
int orc_borders(const orc_domain *d, double cutghost, int nlocal, double *x, int *type,
                int nmax, int *ghost_owner, int *ghost_image);
/* orc_borders plus CommBrick's swap structure: ghost_src[g] = sendlist entry the ghost was
   copied from, swap_first[0..nswap] = first ghost of each swap (nullable outputs) */
int orc_borders_ex(const orc_domain *d, double cutghost, int nlocal, double *x, int *type,
                   int nmax, int *ghost_owner, int *ghost_image, int *ghost_src,
                   int *swap_first, int *nswap);
/* CommBrick::reverse_comm_fix over self swaps (comm_brick.cpp:999-1030), one double/atom */
void orc_reverse_swaps(int nlocal, int nswap, const int *swap_first, const int *ghost_src,
                       double *a);

/* ghost <- owner (+ image*prd on x), for x, rho, e, vest (AtomVecMeso::pack_comm). any of
   rho/e/vest may be NULL. */
void orc_forward_comm(const orc_domain *d, int nlocal, int nghost, const int *ghost_owner,
                      const int *ghost_image, double *x, double *rho, double *e, double *vest);

/* owner += ghost for f (3), drho, de; ghosts left untouched.  any may be NULL. */
void orc_reverse_comm(int nlocal, int nghost, const int *ghost_owner, double *f,
                      double *drho, double *de);

/* ---- neighbor lists ----------------------------------------------------------------- */
/* cutneighsq[i][j] = (sqrt(cut*cut) + skin)^2 with cut = max sub-style cutoff for i,j */
void orc_cutneighsq(int ntypes, const double *cutmax /*(nt+1)^2*/, double skin,
                    double *cutneighsq /*(nt+1)^2*/, double *cutneighmax);

/* Full list of owned atoms over owned+ghost atoms, rsq <= cutneighsq[it][jt], j != i.
   off must hold nlocal+1 ints; neigh capacity cap.  Returns total entries or -1 if cap
   is exceeded (off is then filled with counts only when neigh==NULL). */
long orc_neigh_full(int dim, int nlocal, int nall, const double *x, const int *type,
                    int ntypes, const double *cutneighsq, long *off, int *neigh, long cap);

/* Half (newton on) list derived from a full list, Neighbor::half_from_full_newton. */
long orc_neigh_half_from_full(int nlocal, const double *x, const long *foff,
                              const int *fneigh, long *hoff, int *hneigh);

/* ---- pair styles -------------------------------------------------------------------- */
void orc_rhosum(int dim, int nlocal, const double *x, const int *type, int ntypes,
                const double *mass, const double *cut, const double *cutsq,
                const long *off, const int *neigh, double *rho);

void orc_taitwater(int dim, int nlocal, int newton_pair, const double *x,
                   const double *vest, const double *rho, const int *type, int ntypes,
                   const double *mass, const double *rho0, const double *soundspeed,
                   const double *B, const double *viscosity, const double *cut,
                   const double *cutsq, const long *off, const int *neigh, double *f,
                   double *drho, double *de, double *virial /*6 or NULL*/);

void orc_taitwater_morris(int dim, int nlocal, int newton_pair, const double *x,
                          const double *vest, const double *rho, const int *type,
                          int ntypes, const double *mass, const double *rho0,
                          const double *soundspeed, const double *B,
                          const double *viscosity, const double *cut, const double *cutsq,
                          const long *off, const int *neigh, double *f, double *drho,
                          double *de, double *virial);

void orc_heatconduction(int dim, int nlocal, int newton_pair, const double *x,
                        const double *e, const double *rho, const int *type, int ntypes,
                        const double *mass, const double *alpha, const double *cut,
                        const double *cutsq, const long *off, const int *neigh,
                        double *de);

/* ---- quintic kernel helpers & multiphase styles ------------------------------------ */
double orc_kernel_quintic2d(double r);
double orc_kernel_quintic3d(double r);
double orc_dw_quintic2d(double r);
double orc_dw_quintic3d(double r);

void orc_rhosum_multiphase(int dim, int nlocal, const double *x, const int *type,
                           int ntypes, const double *rmass, const double *cut,
                           const double *cutsq, const long *off, const int *neigh,
                           double *rho);

void orc_taitwater_multiphase(int dim, int nlocal, int newton_pair, const double *x,
                              const double *vest, const double *rho, const int *type,
                              int ntypes, const double *rmass, const double *rho0,
                              const double *soundspeed, const double *B,
                              const double *gamma, const double *rbackground,
                              const double *viscosity, const double *cut,
                              const double *cutsq, const long *off, const int *neigh,
                              double *f);

void orc_heatconduction_phasechange(int dim, int nlocal, int newton_pair, const double *x,
                                    const double *e, const double *cv, const double *rho,
                                    const double *rmass, const int *type, int ntypes,
                                    const double *alpha, const int *fixflag,
                                    const double *tc, const double *cut,
                                    const double *cutsq, const long *off,
                                    const int *neigh, double *de);

void orc_colorgradient(int dim, int nlocal, const double *x, const double *rho,
                       const double *rmass, const int *type, int ntypes,
                       const double *alpha, const double *cut, const double *cutsq,
                       const long *off, const int *neigh, double *colorgradient);

/* cg: nall*3 colorgradient (owned + ghosts); f (nall*3) accumulated, Newton-3 onto j when
   newton_pair or j < nlocal (half lists) */
void orc_surfacetension(int dim, int nlocal, int newton_pair, const double *x,
                        const double *rho, const double *rmass, const int *type, int ntypes,
                        const double *cg, const double *cut, const double *cutsq,
                        const long *off, const int *neigh, double *f);

/* ---- integrators (fix meso, fix meso/stationary, fix gravity) ------------------------
   tmask: the fix's group as a type mask (bit t: type t in the group; 0 = all atoms) */
void orc_meso_setup(int nlocal, const double *v, double *vest);
void orc_meso_setup_g(int nlocal, const int *type, int tmask, const double *v, double *vest);
void orc_meso_initial_g(int nlocal, double dtv, double dtf, const int *type, int tmask,
                        const double *mass, const double *rmass, double *x, double *v,
                        const double *f, double *vest, double *rho, const double *drho,
                        double *e, const double *de);
void orc_meso_final_g(int nlocal, double dtf, const int *type, int tmask, const double *mass,
                      const double *rmass, double *v, const double *f, double *rho,
                      const double *drho, double *e, const double *de);
/* FixMesoStationary::initial_integrate == ::final_integrate (fix_meso_stationary.cpp:71-112) */
void orc_meso_stationary(int nlocal, double dtf, const int *type, int tmask, double *rho,
                         const double *drho, double *e, const double *de);
/* FixGravity::post_force, style vector (fix_gravity.cpp:244-295, :320-336): f += m*acc */
void orc_gravity(int nlocal, const int *type, int tmask, const double *mass,
                 const double *rmass, const double *acc, double *f);
void orc_meso_initial(int nlocal, double dtv, double dtf, const int *type,
                      const double *mass, const double *rmass, double *x, double *v,
                      const double *f, double *vest, double *rho, const double *drho,
                      double *e, const double *de);
void orc_meso_final(int nlocal, double dtf, const int *type, const double *mass,
                    const double *rmass, double *v, const double *f, double *rho,
                    const double *drho, double *e, const double *de);

/* ---- fix phase_change (FixPhaseChange::pre_exchange, fix_phase_change.cpp:167-352) ---- */
typedef struct {
  int dim;
  double Tc, Tt, Hwv, dr, to_mass, cutoff;   /* required args, fix_phase_change.cpp:58-67 */
  int from_type, to_type;
  int energy_chance;                          /* "ENERGY rate" form (:70-73) */
  double change_chance, rate, dt;             /* dt = update->dt */
  int maxattempt;                             /* option "attempt", default 10 (:364) */
  double sublo[3], subhi[3], boxhi[3];
  int top[3];                                 /* comm->myloc[d] == procgrid[d]-1 */
} orc_pc_params;

/* RanPark::uniform, src/random_park.cpp:42-49 (seed updated in place) */
double orc_park_uniform(int *seed);

/* One pre_exchange call on one rank.  Arrays hold nall = nlocal + nghost atoms (x, v,
   vest, cg: 3 per atom); the list is the fix's FULL list (rows 0..nlocal).  e is updated
   in place for the atoms that change phase; dmass[0..nall) receives the mass taken from
   from_type atoms (ghost entries still to be reverse-communicated).  New atoms (at most
   cap) are written as records of 13 doubles {x[3], v[3], vest[3], e, rmass, rho, cv} with
   the index of the parent atom in parent[].  Returns the number inserted. */
int orc_phasechange(const orc_pc_params *p, int *seed, int nlocal, int nall, const double *x,
                    const double *v, const double *vest, const double *cg, double *e,
                    const double *rmass, const double *rho, const double *cv,
                    const int *type, const long *off, const int *neigh, double *dmass,
                    int cap, double *new_atoms, int *parent);
/* after reverse comm of dmass: rmass -= dmass, e renormalised (fix_phase_change.cpp:327-334) */
void orc_phasechange_finish(int nlocal, const double *dmass, double *rmass, double *e);
/* The whole pre_exchange with the reference's memory behaviour (created atoms written over
   ghost slots, reverse comm along CommBrick's swaps); see sph_oracle.c.  Returns the new
   nlocal or -1. */
int orc_pre_exchange_ref(const orc_pc_params *p, int *seed, int nlocal, int nghost, int nmax,
                         double *x, double *v, double *vest, double *cg, double *e,
                         double *rmass, double *rho, double *cv, int *type, const long *off,
                         const int *neigh, int nswap, const int *swap_first,
                         const int *ghost_src, double *dmass);

#ifdef __cplusplus
}
#endif
#endif
