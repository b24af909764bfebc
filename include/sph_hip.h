/*
 * sph_hip.h -- C ABI of the MI355X-native USER-SPH pair engine (libsph_hip.so).
 *
 * Two layers, both plain C (pointers + sizes, no torch/HIP types):
 *
 *  1. Pair-style layer (sph_hip_*): what a LAMMPS `sph/<style>/hip` Pair class calls from
 *     its compute(), with LAMMPS' own host arrays and NeighList.  Replaces the CPU loops of
 *       PairSPHRhoSum::compute          src/USER-SPH/pair_sph_rhosum.cpp:66-204
 *       PairSPHTaitwater::compute       src/USER-SPH/pair_sph_taitwater.cpp:53-200
 *       PairSPHTaitwaterMorris::compute src/USER-SPH/pair_sph_taitwater_morris.cpp:52-200
 *       PairSPHHeatConduction::compute  src/USER-SPH/pair_sph_heatconduction.cpp:47-134
 *     (paths relative to the reference tree).  Coefficients follow each style's coeff() /
 *     init_one() semantics (tables already filled and symmetrised by LAMMPS).
 *
 *  2. Device-resident engine (sph_engine_*): the whole Verlet step of an SPH run
 *     (FixMeso integrate, pbc, borders/ghost images, binned neighbor build, rhosum ->
 *     forward comm -> taitwater[/morris] [+heatconduction], integrate) kept in HBM,
 *     optionally sharded over several GPUs by brick decomposition with the halo carried on
 *     RCCL.  Replaces, for device-resident runs, Verlet::run (src/verlet.cpp:207-309)
 *     around the same pair styles; Neighbor::full_bin (src/neigh_full.cpp:241-344);
 *     CommBrick::borders/forward_comm (src/comm_brick.cpp:444-506, 696-864);
 *     FixMeso::initial/final_integrate (src/USER-SPH/fix_meso.cpp:91-180).
 *
 * Every function returns 0 on success and a negative SPH_HIP_E* code on failure;
 * sph_hip_last_error() then describes the failure (thread-local).  As with the GPU
 * package precedent (src/GPU/pair_lj_cut_gpu.cpp:114-115) the caller turns a failure into
 * error->one(FLERR, ...).  There is no CPU fallback: without a usable HIP device every
 * compute entry point fails with SPH_HIP_ENODEV.
 *
 * Array conventions (identical to LAMMPS): per-atom vectors are AoS double[n][3]
 * (atom->x's contiguous backing, src/memory.h:124-137); per-type tables have ntypes+1
 * entries and per-type-pair tables (ntypes+1)^2 entries, row-major, 1-based types.
 */
#ifndef SPH_HIP_H
#define SPH_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPH_HIP_ABI_VERSION 2

#define SPH_HIP_OK 0
#define SPH_HIP_EINVAL (-1)   /* bad argument / not configured */
#define SPH_HIP_ENODEV (-2)   /* no usable HIP device */
#define SPH_HIP_ERUNTIME (-3) /* HIP runtime / kernel failure */
#define SPH_HIP_ENOMEM (-4)   /* device allocation failed ("Insufficient memory on accelerator") */
#define SPH_HIP_ECOMM (-5)    /* RCCL failure */
#define SPH_HIP_EOVERFLOW (-6)/* neighbor / ghost capacity exceeded */

/* list kinds, as NeighRequest half/full (src/neigh_request.h) */
#define SPH_LIST_FULL 0
#define SPH_LIST_HALF 1

/* viscosity variants of sph/taitwater */
#define SPH_VISC_MONAGHAN 0   /* sph/taitwater        (pair_sph_taitwater.cpp:162-169) */
#define SPH_VISC_MORRIS 1     /* sph/taitwater/morris (pair_sph_taitwater_morris.cpp:163-167) */

const char *sph_hip_last_error(void);
int sph_hip_abi_version(void);
/* number of visible HIP devices (0 without a GPU; never fails) */
int sph_hip_device_count(void);

/* ======================================================================================
 * 1. Pair-style layer
 * ==================================================================================== */
typedef struct sph_hip_ctx sph_hip_ctx;

/* One context per MPI rank / Pair instance set.  dim = domain->dimension, ntypes =
   atom->ntypes, newton_pair = force->newton_pair. */
int sph_hip_create(int device, int dim, int ntypes, int newton_pair, sph_hip_ctx **out);
int sph_hip_destroy(sph_hip_ctx *ctx);
/* Device time of the last style call's kernels, in ms (HIP events recorded around the
   launches on the context's stream; staging and result copies excluded), when enabled by
   sph_hip_set_timing(ctx, 1).  Measurement support; not part of the LAMMPS pair API. */
int sph_hip_set_timing(sph_hip_ctx *ctx, int on);
int sph_hip_last_kernel_ms(sph_hip_ctx *ctx, double *ms);

/* PairSPHRhoSum::coeff/init_one: cut (nt+1)^2 (h per type pair), mass = atom->mass. */
int sph_hip_rhosum_coeff(sph_hip_ctx *ctx, const double *cut, const double *mass);
/* PairSPHTaitwater[Morris]::coeff/init_one: rho0, soundspeed, B per type (nt+1),
   viscosity and cut per pair ((nt+1)^2). visc_variant = SPH_VISC_*. */
int sph_hip_taitwater_coeff(sph_hip_ctx *ctx, int visc_variant, const double *rho0,
                            const double *soundspeed, const double *B,
                            const double *viscosity, const double *cut, const double *mass);
/* PairSPHHeatConduction::coeff/init_one: alpha and cut per pair ((nt+1)^2). */
int sph_hip_heatconduction_coeff(sph_hip_ctx *ctx, const double *alpha, const double *cut,
                                 const double *mass);

/* Stage per-atom inputs: nlocal owned then nghost ghost atoms (atom->x, atom->vest,
   atom->rho, atom->e, atom->type).  vest/rho/e may be NULL when the next compute does
   not read them. */
int sph_hip_atoms(sph_hip_ctx *ctx, int nlocal, int nghost, const double *x,
                  const double *vest, const double *rho, const double *e, const int *type);
/* Restage rho only (nall values; x, vest, e, type, rmass, cv as last staged): the second
   and later pair computes of one step under hybrid/overlay, after forward_comm_pair of the
   density (the shim keys it on ntimestep + neighbor->ncalls + nlocal/nghost). */
int sph_hip_atoms_rho(sph_hip_ctx *ctx, const double *rho);
/* Restage x (and vest, rho, e where non-NULL) of the SAME atom set as the last
   sph_hip_atoms (same nlocal/nghost and types: a step between rebuilds) -- no type upload or
   check, staged lists kept. */
int sph_hip_atoms_update(sph_hip_ctx *ctx, const double *x, const double *vest,
                         const double *rho, const double *e);
/* Register the caller's per-atom arrays (capacity nmax atoms: x, vest, f nmax*3, the others
   nmax; any may be NULL) as mapped host memory: the staging kernels then read x/vest/rho/e
   straight from them over PCIe and the styles write rho / add f, drho, de straight into
   them, instead of a host copy, a PCIe copy and a host loop per call.  Call again whenever
   the arrays move (LAMMPS: atom->nmax or a pointer changed; the shim checks every compute);
   nmax = 0 unregisters.  An array the runtime refuses to register keeps the copy path. */
int sph_hip_host_arrays(sph_hip_ctx *ctx, int nmax, double *x, double *vest, double *rho,
                        double *e, double *f, double *drho, double *de);

/* Stage a LAMMPS NeighList (list->inum, ilist, numneigh, firstneigh; NEIGHMASK bits are
   stripped).  kind = SPH_LIST_FULL (gather-only kernels, nothing written to ghosts) or
   SPH_LIST_HALF (the reference's Newton-3 semantics: the j share of every pair, ghosts
   included when newton_pair is on, is gathered through the reverse of the staged half list,
   built once per upload; SPH_MPREV=0 scatters it with fp64 atomics instead).  Entries are
   checked on the device (0 <= j < nall, ilist owned): SPH_HIP_EINVAL otherwise. */
int sph_hip_list(sph_hip_ctx *ctx, int kind, int inum, const int *ilist,
                 const int *numneigh, const int *const *firstneigh);
/* sph_hip_list with reuse (the device mirror keyed by the list build):
   key >= 0 identifies the build (LAMMPS: neighbor->ncalls).  The context keeps one staged
   list per kind, so hybrid/overlay sub-styles that alternate FULL and HALF lists each keep
   theirs; a call whose (kind, key, inum) matches the staged list of that kind returns
   without touching the host list (no copy, upload or check; the reverse list is kept).
   Restaging atoms with a different nlocal/nghost drops every staged list.  key < 0 always
   uploads (= sph_hip_list). */
int sph_hip_list_keyed(sph_hip_ctx *ctx, int kind, int64_t key, int inum, const int *ilist,
                       const int *numneigh, const int *const *firstneigh);
/* The list built on the DEVICE from the staged atoms (SURVEY 8(b) device-list path; the GPU
   package's GPU_NEIGH, src/GPU/pair_lj_cut_gpu.cpp:97-104): kind SPH_LIST_FULL =
   Neighbor::full_bin membership (neigh_full.cpp:241-344: j != i, rsq <= cutneighsq[it][jt]),
   SPH_LIST_HALF = half_from_full_newton of it (neigh_derive.cpp:83-150); owned rows, ilist
   the identity.  cutneighsq = neighbor->cutneighsq ((nt+1)^2).  key as sph_hip_list_keyed:
   a staged device-built list of this kind with the same key is reused (hybrid/overlay
   sub-styles, the fix's copy).  Replaces the host NeighList copy and upload per rebuild. */
int sph_hip_build_list(sph_hip_ctx *ctx, int kind, int64_t key, const double *cutneighsq);
/* Row lengths of the staged list (inum values, in ilist order): LAMMPS' numneigh. */
int sph_hip_list_numneigh(sph_hip_ctx *ctx, int *numneigh);
/* Same, from a CSR list (row i = neigh[off[i]..off[i+1]) for owned atom i). */
int sph_hip_list_csr(sph_hip_ctx *ctx, int kind, int inum, const int64_t *off,
                     const int *neigh);

/* rho[0..nlocal) <- self term + sum over list (pair_sph_rhosum.cpp:112-195).  The
   forward_comm_pair of ghost rho stays with the caller (comm->forward_comm_pair). */
int sph_hip_rhosum(sph_hip_ctx *ctx, double *rho);
/* f (nall*3), drho, de (nall) are ACCUMULATED into (force_clear semantics stay with the
   caller).  With a FULL list only owned entries change; with a HALF list ghosts receive
   their Newton-3 share exactly as in the reference and need reverse_comm. virial may be
   NULL, else 6 doubles accumulated in the ev_tally convention (pair.cpp:770-850). */
int sph_hip_taitwater(sph_hip_ctx *ctx, double *f, double *drho, double *de,
                      double *virial);
int sph_hip_heatconduction(sph_hip_ctx *ctx, double *de);

/* ======================================================================================
 * 1b. Multiphase styles (atom_style meso/multiphase: per-atom rmass; quintic kernel).
 *     Tables are (nt+1)^2 row-major; like coeff()+init_one() the upper triangle i <= j is
 *     read and mirrored.  Stage atoms with sph_hip_atoms (x, vest, rho, e, type) and then
 *     sph_hip_atoms_multiphase (rmass, cv: nlocal + nghost each; cv may be NULL).
 * ==================================================================================== */
int sph_hip_atoms_multiphase(sph_hip_ctx *ctx, const double *rmass, const double *cv);

/* PairSPHRhoSumMultiphase (pair_sph_rhosum_multiphase.cpp:112-167, coeff :194-216):
   cut = h per pair; rho[0..nlocal) <- rmass_i (W(0)/h_ii^d + sum_j W(r/h)/h^d).  Full list. */
int sph_hip_rhosum_multiphase_coeff(sph_hip_ctx *ctx, const double *cut);
int sph_hip_rhosum_multiphase(sph_hip_ctx *ctx, double *rho);

/* PairSPHTaitwaterMultiphase (pair_sph_taitwater_multiphase.cpp:95-183, coeff :225-262):
   per type rho0, soundspeed, gamma, rbackground (B = c^2 rho0 / gamma); per pair viscosity
   and cut.  f (nall*3) is ACCUMULATED; HALF lists scatter onto j (newton_pair) exactly as
   the reference, including its p_j = p(rho_j; gamma[itype]) asymmetry. */
int sph_hip_taitwater_multiphase_coeff(sph_hip_ctx *ctx, const double *rho0,
                                       const double *soundspeed, const double *gamma,
                                       const double *rbackground, const double *viscosity,
                                       const double *cut);
int sph_hip_taitwater_multiphase(sph_hip_ctx *ctx, double *f);

/* PairSPHHeatConductionPhaseChange (pair_sph_heatconduction_phasechange.cpp:81-138, coeff
   :177-225): alpha, cut per pair; fixflag (int, the type whose temperature is clamped, 0 =
   none) and tc per pair, either may be NULL (4-argument coeff form).  de (nall) is
   ACCUMULATED. */
int sph_hip_heatconduction_phasechange_coeff(sph_hip_ctx *ctx, const double *alpha,
                                             const int *fixflag, const double *tc,
                                             const double *cut);
int sph_hip_heatconduction_phasechange(sph_hip_ctx *ctx, double *de);

/* PairSPHColorGradient (pair_sph_colorgradient.cpp:118-187): alpha, cut per pair;
   cg[0..nlocal)*3 is OVERWRITTEN (the reference zeroes it first).  Full list. */
int sph_hip_colorgradient_coeff(sph_hip_ctx *ctx, const double *alpha, const double *cut);
int sph_hip_colorgradient(sph_hip_ctx *ctx, double *cg);

/* PairSPHSurfaceTension (pair_sph_surfacetension.cpp:50-192, coeff :222-247): cut = h per
   pair.  cg (nall*3, atom->colorgradient of owned atoms and ghosts) is read; f (nall*3) is
   ACCUMULATED; HALF lists (the style's default request) scatter onto j when newton_pair or
   j < nlocal, as the reference. */
int sph_hip_surfacetension_coeff(sph_hip_ctx *ctx, const double *cut);
int sph_hip_surfacetension(sph_hip_ctx *ctx, const double *cg, double *f);

/* ======================================================================================
 * 1c. fix phase_change (FixPhaseChange::pre_exchange, fix_phase_change.cpp:167-352)
 * ==================================================================================== */
typedef struct {
  double Tc, Tt, Hwv, dr, to_mass, cutoff;   /* required args (fix_phase_change.cpp:58-67) */
  int from_type, to_type;
  int energy_chance;                          /* 1: "ENERGY rate" form (:70-73) */
  double change_chance, rate;                 /* prob, or rate of the ENERGY form */
  double dt;                                  /* update->dt */
  int maxattempt;                             /* option "attempt" (default 10) */
  double sublo[3], subhi[3], boxhi[3];        /* domain->sublo/subhi/boxhi */
  int top[3];                                 /* comm->myloc[d] == comm->procgrid[d]-1 */
} sph_phasechange_params;

/* One pre_exchange on this rank.  Uses the staged atoms (sph_hip_atoms: x, vest, rho, e,
   type; sph_hip_atoms_multiphase: rmass, cv) and the fix's FULL list (sph_hip_list /
   sph_hip_list_csr with SPH_LIST_FULL).  v and cg (atom->v, atom->colorgradient) are nall*3.
   The Park-Miller stream (*seed, RanPark) is consumed in the reference's order, so the
   same seed gives the same insertions.  e[0..nlocal) is updated for atoms that changed
   phase; dmass[0..nall) receives the mass taken from from_type atoms (reverse-communicate
   the ghost part, then call sph_hip_phasechange_finish).  Up to cap new atoms are written
   as 13-double records {x[3], v[3], vest[3], e, rmass, rho, cv}, their parent atom index in
   parent[]; *nins = number inserted (may exceed cap: then call again with more room, the
   seed must be restored by the caller).  The caller creates them (avec->create_atom,
   type to_type) and updates natoms/tags as the reference does (:336-351). */
int sph_hip_phasechange(sph_hip_ctx *ctx, const sph_phasechange_params *p, int *seed,
                        const double *v, const double *cg, double *e, double *dmass, int cap,
                        int *nins, double *new_atoms, int *parent);
/* rmass[i] -= dmass[i]; e[i] *= mold / rmass[i] for i < nlocal (:327-334).  Host only. */
int sph_hip_phasechange_finish(int nlocal, const double *dmass, double *rmass, double *e);

/* ======================================================================================
 * 2. Device-resident engine
 * ==================================================================================== */
#define SPH_MAXTYPES 8

/* Multiphase stack of examples/USER/sph/bubble_growth/bubble.lmp:57-73 (atom_style
   meso/multiphase: per-atom rmass, cv, colorgradient; quintic kernel), run by the engine
   in place of the sph/rhosum, taitwater and heatconduction styles of sph_engine_config.
   Per-pair tables in the (SPH_MAXTYPES+1)^2 layout, upper triangle (i <= j) read and
   mirrored as init_one does.  Sequence per step (hybrid/overlay order): rhosum/multiphase
   and colorgradient over the full list (owned rows; their misnamed pack_comm moves
   nothing, so ghosts keep their comm-time rho and colorgradient), then
   taitwater/multiphase, surfacetension and heatconduction/phasechange over the half list
   with Newton-3 and reverse comm.  fix meso integrates with rmass. */
typedef struct {
  int rhosum_nstep;            /* sph/rhosum/multiphase N (0 = off); cut = h per pair */
  double rhosum_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  int cg_nstep;                /* sph/colorgradient N (0 = off): alpha, cut per pair */
  double cg_alpha[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  double cg_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  int tait_on;                 /* sph/taitwater/multiphase: per type rho0, c, gamma, rbg */
  double rho0[SPH_MAXTYPES + 1], soundspeed[SPH_MAXTYPES + 1], gamma[SPH_MAXTYPES + 1];
  double rbackground[SPH_MAXTYPES + 1];
  double tait_visc[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  double tait_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  int st_on;                   /* sph/surfacetension: cut per pair */
  double st_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  int heat_on;                 /* sph/heatconduction/phasechange: alpha, cut, fixflag, tc */
  double heat_alpha[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  double heat_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  double heat_tc[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  int heat_fixflag[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
} sph_engine_mp_config;

typedef struct {
  int dim;                     /* 2 or 3 */
  int ntypes;                  /* <= SPH_MAXTYPES */
  double boxlo[3], boxhi[3];   /* global box */
  int periodic[3];
  double skin;                 /* neighbor skin */
  int neigh_every;             /* rebuild every N steps (neigh_modify every N check no) */
  double dt;                   /* timestep (units lj: ftm2v = 1) */
  double ftm2v;                /* force->ftm2v */
  double mass[SPH_MAXTYPES + 1];
  /* integrator: 0 = fix meso for all types, 1 = fix meso/stationary for type 2.. (bc) */
  int stationary_mask;         /* bit t set: type t integrates with meso/stationary */
  /* sph/rhosum: enabled if rhosum_nstep > 0 */
  int rhosum_nstep;
  double rhosum_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  /* sph/taitwater[/morris]: enabled if tait_on */
  int tait_on;
  int tait_visc;               /* SPH_VISC_* */
  double rho0[SPH_MAXTYPES + 1], soundspeed[SPH_MAXTYPES + 1], B[SPH_MAXTYPES + 1];
  double tait_visc_coef[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  double tait_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  /* sph/heatconduction: enabled if heat_on */
  int heat_on;
  double heat_alpha[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  double heat_cut[(SPH_MAXTYPES + 1) * (SPH_MAXTYPES + 1)];
  /* body force per unit mass (fix gravity style), added in post_force: f += m*g, for the
     types in gravity_mask (bit t set: type t is in the fix's group; 0 = every type) */
  double gravity[3];
  int gravity_mask;
  /* brick decomposition (procgrid[0]*procgrid[1]*procgrid[2] bricks, uniform split; 1 1 1 or
     0 0 0 = one brick).  Bricks are numbered x fastest; each must be wider than the ghost
     cutoff (CommBrick maxneed = 1). */
  int procgrid[3];
  int rank;                    /* my rank in the brick, x fastest */
  /* spatially sort owned particles at every rebuild (atom->sort analogue) */
  int sort;
  /* pair-pass kernels (full lists, gather only, no atomics):
     0 = block-staged (production): blocks of consecutive owned rows stage the union of
         their neighbours in LDS, rows walk 16-bit slot lists built from the bins at every
         rebuild (falls back to 1 for a build whose blocks overflow the LDS image);
     1 = row path: rows gather neighbour records from HBM through a strided global-index
         list (the round-1 production path) */
  int kernel_path;
  /* multiphase stack (NULL: the single-phase styles above); copied at create */
  const sph_engine_mp_config *mp;
} sph_engine_config;

typedef struct {
  int64_t step;
  int nlocal, nghost;
  int64_t nbr_full;            /* entries in the device full list (owned rows) */
  int nbr_builds;
  int nbr_maxrow;              /* longest full-list row of the last CSR build */
  int staged;                  /* 1 if the last build produced block-staged lists */
  int stage_max;               /* block path: largest block union (LDS records) */
  double ms_rhosum, ms_tait, ms_heat, ms_integrate, ms_comm, ms_neigh; /* event-timed */
  int64_t n_rhosum, n_tait, n_heat, n_neigh;  /* launches timed */
  int blk_nbig;                /* block path: blocks of the last build whose union exceeds the
                                  force pass's LDS image (walked by the second launch) */
  int inner_rows;              /* block path: inner rows were built at the last rebuild */
  int inner_live;              /* ... and the last step's passes walked them (no atom had moved
                                  past their margin since they were written) */
  int flags;                   /* bit 0: the last rhosum/multiphase was summed inside the
                                  list fill (C5: its time is in ms_neigh, not ms_rhosum) */
  int64_t inner_refresh;       /* refresh launches since create (inner rows derived again
                                  between rebuilds when an atom passed their margin) */
} sph_engine_stats;

typedef struct sph_engine sph_engine;

int sph_engine_create(int device, const sph_engine_config *cfg, sph_engine **out);
int sph_engine_destroy(sph_engine *e);

/* Brick decomposition (cfg.procgrid, cfg.rank; CommBrick's swaps, comm_brick.cpp).  Every
   brick needs a communicator before sph_engine_setup:
   * RCCL, one process per GPU: uid = ncclUniqueId bytes (128) produced by
     sph_engine_comm_uid on rank 0 and distributed by the caller (MPI_Bcast / torch);
   * a local world: several bricks in one process (one host thread per brick, any devices),
     halo exchange by device copies -- for tests and bricks that share a GPU.
   Owned atoms migrate between bricks at rebuilds; sph_engine_get_atoms then returns them in
   local order with their tags (sph_engine_set_tags sets global tags; default = index). */
int sph_engine_comm_uid(void *uid128);
int sph_engine_comm_init(sph_engine *e, const void *uid128, int nranks, int rank);
/* One-brick engine with a communicator attached: on != 0 routes its periodic self swaps
   (borders, forward, rho, reverse) through the communicator -- RCCL send/recv to itself --
   instead of device copies, so the multi-brick data path runs on one GPU.  Before setup. */
int sph_engine_comm_loopback(sph_engine *e, int on);
typedef struct sph_local_world sph_local_world;
int sph_local_world_create(int nranks, sph_local_world **out);
int sph_local_world_destroy(sph_local_world *w);
int sph_engine_comm_local(sph_engine *e, sph_local_world *w, int rank);
/* Node-local world of PROCESSES without RCCL (one process per brick, any devices of the
   node, incl. several processes on one GPU, which RCCL refuses): `name` ("/word", chosen by
   rank 0 and distributed by the caller like the RCCL uid) names a POSIX shared-memory
   control segment; mode 0 moves halos device-to-device through hipIpc-exported outboxes,
   mode 1 stages them through host shared memory.  Same Transport calls, same order, as
   RCCL (comm_brick.cpp:444-506, 696-864, 999-1030).  Collective: every rank calls it. */
int sph_engine_comm_ipc(sph_engine *e, const char *name, int nranks, int rank, int mode);
/* Schedule choices that do not change results (parity-tested both ways), set explicitly
   rather than through the environment; before sph_engine_setup.
   SPH_TUNE_OVERLAP: bricks on the row path overlap interior rows' passes with the halo
   exchange (1) or not (0, default).  SPH_TUNE_BLKUMF: cap the block force pass's LDS image
   at `value` records, blocks with larger unions going to its second launch (0 = auto). */
#define SPH_TUNE_OVERLAP 1
#define SPH_TUNE_BLKUMF 2
int sph_engine_tune(sph_engine *e, int key, int value);
int sph_engine_set_tags(sph_engine *e, const int *tags);

/* Owned particles of this rank (tag order is the caller's order; results are returned in
   the same order).  v is the velocity; vest is set from v at setup (FixMeso::setup_pre_force). */
int sph_engine_set_atoms(sph_engine *e, int n, const double *x, const double *v,
                         const int *type, const double *rho, const double *en,
                         const double *cv);
/* Multiphase engines: per-atom rmass and cv (and the initial colorgradient, n*3, may be
   NULL = 0) of the set_atoms atoms, in the same order.  After set_atoms, before setup. */
int sph_engine_set_atoms_multiphase(sph_engine *e, const double *rmass, const double *cv,
                                    const double *cg);
/* fix phase_change on a one-brick multiphase engine (FixPhaseChange::pre_exchange at steps
   1, 1+nevery, ...; the rebuild follows): p's sublo/subhi/boxhi/top are filled by the
   engine, p->dt must be the engine's dt.  Candidates meet the Park-Miller stream (seed) in
   the reference's local atom order, which the engine tracks beside its own row order while
   the fix is armed: read order (ascending tag within the brick), CommBrick::exchange's hole
   fill (comm_brick.cpp:620-632; received atoms appended), Atom::sort at setup and every
   sortfreq steps (sph_engine_atom_sort), created atoms appended.  New atoms get tags n,
   n+1, ... in creation order (atom->tag_extend), type to_type.  Before setup. */
int sph_engine_phase_change(sph_engine *e, const sph_phasechange_params *p, int nevery,
                            int seed);
/* atom_modify sort sortfreq binsize (atom.cpp:540-551; replaces Atom::sortfreq/userbinsize):
   the spatial sort whose order fix phase_change meets its candidates in -- bins of binsize
   (0 = half the neighbor cutoff, Atom::setup_sort_bins) over the brick, at setup and every
   sortfreq steps (0 = never).  Default 1000 / 0, LAMMPS' own.  The engine's rows keep their
   own order; only the tracked LAMMPS order changes. */
int sph_engine_atom_sort(sph_engine *e, int sortfreq, double binsize);
/* Multiphase fields of the owned atoms in get_atoms order (any pointer may be NULL):
   rmass, cv, colorgradient (n*3), vest (n*3), type; *ninserted = atoms created so far. */
int sph_engine_get_atoms_multiphase(sph_engine *e, double *rmass, double *cv, double *cg,
                                    double *vest, int *type, int64_t *ninserted);

/* Restart records of the owned atoms (one brick), in get_atoms order, in the reference's
   per-atom restart layout: meso -- AtomVecMeso::pack_restart (atom_vec_meso.cpp:726-757),
   17 doubles {17, x[3], tag, type, mask, image (each an int64 bit pattern, LAMMPS ubuf),
   v[3], rho, e, cv, vest[3]}; multiphase -- AtomVecMesoMultiPhase::pack_restart
   (atom_vec_meso_multiphase.cpp:887-916), 21 doubles {21, x[3], tag, type, mask, image (as
   plain doubles, as that routine writes them), v[3], rho, colorgradient[3], rmass, e, cv,
   vest[3]}.  tag = 1 + the set_atoms index (LAMMPS tags start at 1), mask = 1 (group all),
   image = the packed imageint (lmptype.h, 10 bits per dimension, 512 = zero) counted by
   Domain::pbc.  buf == NULL: only *rec_size (17 or 21) is returned; else cap >= nlocal *
   rec_size doubles. */
int sph_engine_write_restart(sph_engine *e, double *buf, int64_t cap, int *rec_size);
/* Atoms from n restart records of the engine's layout (tags a permutation of 1..n; the
   atom with tag t becomes set_atoms index t-1): x, v, vest, rho, e, cv, type, image (and
   rmass, colorgradient for a multiphase engine).  Replaces set_atoms; before setup (whose
   FixMeso::setup_pre_force sets vest = v again, as a LAMMPS run after read_restart does). */
int sph_engine_read_restart(sph_engine *e, int n, const double *buf);

/* Verlet::setup: forced rebuild + forces at step 0. */
int sph_engine_setup(sph_engine *e);
/* Verlet::run(nsteps). */
int sph_engine_run(sph_engine *e, int nsteps);
/* Copy back owned particles in the set_atoms order (any pointer may be NULL). n is the
   current nlocal (sph_engine_nlocal). */
int sph_engine_nlocal(sph_engine *e);
int sph_engine_get_atoms(sph_engine *e, double *x, double *v, double *rho, double *en,
                         double *f, double *drho, double *de, int *tag);
/* per owned particle (set_atoms order): full-list count within cut+skin at last build */
int sph_engine_neighbor_counts(sph_engine *e, int *numneigh);
int sph_engine_stats_get(sph_engine *e, sph_engine_stats *s);
/* hipEvent timing of the kernel classes (adds an event pair per timed scope): on = 0 off,
   1 every class, (mask << 1) the classes in mask -- bit 0 rhosum, 1 taitwater (or the fused
   multiphase gather), 2 heat, 3 integrate, 4 comm, 5 neighbor build / phase change */
int sph_engine_set_timing(sph_engine *e, int on);
/* synchronise the engine's stream */
int sph_engine_sync(sph_engine *e);
/* run only the pair passes (rhosum + forward comm + taitwater [+heat]) n times on the
   current state, no integration or rebuild: the kernel-roofline workload */
int sph_engine_pair_passes(sph_engine *e, int n);
/* run only the neighbour rebuild (pbc, spatial sort, borders, bins, list) n times on the
   current positions: the list-build workload (timed under the neighbour class) */
int sph_engine_rebuild_passes(sph_engine *e, int n);

#ifdef __cplusplus
}
#endif
#endif /* SPH_HIP_H */
