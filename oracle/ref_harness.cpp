// ref_harness.cpp -- drives the REFERENCE's own USER-SPH compute code (compiled from
// /root/reference/src by oracle/build_ref.sh into oracle/_ref/libsph_ref.so).
// TEST INFRASTRUCTURE ONLY: used to pin the C restatement (sph_oracle.c) and to
// generate tests/golden fixtures.  Never part of the product.
//
// What runs is reference code, unmodified:
//   Neighbor::setup_bins/stencil_full_bin_{2d,3d}/bin_atoms/full_bin  (neighbor.cpp,
//     neigh_stencil.cpp, neigh_full.cpp)  and  Neighbor::half_from_full_newton
//     (neigh_derive.cpp:83-150)
//   PairSPH{RhoSum,Taitwater,TaitwaterMorris,HeatConduction,RhoSumMultiphase,
//     TaitwaterMultiphase,HeatConductionPhaseChange,ColorGradient}::compute, ::init_one
//     and Pair::init (pair.cpp:174-229)
//   AtomVecMeso{,Multiphase}::grow for the per-atom arrays.
// The LAMMPS top-level object, Atom, Domain, Force and Update are not constructed
// (their translation units need generated style_*.h headers, which we do not create);
// this harness zero-allocates those objects and fills only the fields the code above
// reads.  Coefficients are written straight into the pair's tables because
// Pair*::coeff() parses strings through Force (force.cpp), which is not built; the
// formulas applied are the coeff() ones (cited below).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <new>
#include <string>
#include <typeinfo>
#include <vector>

#include "mpi.h"
#include "lammps.h"
#include "memory.h"
#include "error.h"
#include "atom.h"
#include "atom_vec_meso.h"
#include "atom_vec_meso_multiphase.h"
#include "domain.h"
#include "force.h"
#include "update.h"
#include "comm_brick.h"
#include "neighbor.h"
#include "neigh_list.h"
#include "neigh_request.h"
#include "pair_sph_rhosum.h"
#include "pair_sph_taitwater.h"
#include "pair_sph_taitwater_morris.h"
#include "pair_sph_heatconduction.h"
#include "pair_sph_rhosum_multiphase.h"
#include "pair_sph_taitwater_multiphase.h"
#include "pair_sph_heatconduction_phasechange.h"
#include "pair_sph_colorgradient.h"
#include "pair_sph_surfacetension.h"
#include "group.h"
#include "universe.h"
#include "fix_meso.h"
#include "fix_meso_stationary.h"
#include "fix_phase_change.h"
#include "modify.h"
#include "region.h"
#include "region_block.h"

using namespace LAMMPS_NS;

// The same harness builds two test libraries (oracle/build_ref.sh): libsph_ref.so drives the
// reference's own styles and fix (entry points ref_*), and with -DSPH_SHIM libsph_shim.so
// drives the drop-in sph/<style>/hip classes and fix phase_change/hip
// (lammps-sph-multiphase_amd/lammps/), which call libsph_hip.so, on the same harness-filled
// universe (entry points shim_*).  SPH_INIT(p) is Pair::init's init_style() call
// (pair.cpp:211), which the /hip styles use to start a new run epoch.
#ifdef SPH_SHIM
#include "fix_phase_change_hip.h"
#include "pair_sph_hip.h"
#define SPH_H(base) base##HIP
#define REFNAME(n) shim_##n
#define SPH_INIT(p) (p)->init_style()
#else
#define SPH_H(base) base
#define REFNAME(n) ref_##n
#define SPH_INIT(p) ((void)0)
#endif

namespace {

template <class T> T *zalloc() { return static_cast<T *>(calloc(1, sizeof(T))); }

struct HNeighbor : public Neighbor {
  HNeighbor(LAMMPS *l) : Neighbor(l) {}
  using Neighbor::bboxlo;
  using Neighbor::bboxhi;
  using Neighbor::triclinic;
  using Neighbor::bin_atoms;
  using Neighbor::full_bin;
  using Neighbor::half_from_full_newton;
  using Neighbor::stencil_full_bin_2d;
  using Neighbor::stencil_full_bin_3d;
  using Neighbor::sx;
  using Neighbor::sy;
  using Neighbor::sz;
  using Neighbor::smax;
  using Neighbor::dimension;
  using Neighbor::exclude;
  using Neighbor::mbins;
  using Neighbor::maxbin;
  using Neighbor::cutneighsq;
  using Neighbor::bins;
  using Neighbor::cutneighmaxsq;
};

struct HComm : public CommBrick {
  HComm(LAMMPS *l) : CommBrick(l) { nswap = 0; }
  using CommBrick::grow_list;
  using CommBrick::grow_send;
  using CommBrick::maxsend;
  using CommBrick::maxsendlist;
  // self swaps as CommBrick::borders leaves them on one process (comm_brick.cpp:696-864):
  // swap s received ghosts [first[s], first[s+1]) (offsets past nlocal), each copied from
  // src[g] (its sendlist entry: an owned atom or a ghost of an earlier swap)
  void set_self_swaps(int nlocal, int ns, const int *first, const int *src) {
    if (ns > maxswap) grow_swap(ns);
    nswap = ns;
    int most = 0;
    for (int s = 0; s < ns; s++) {
      const int n = first[s + 1] - first[s];
      sendproc[s] = recvproc[s] = me;
      sendnum[s] = recvnum[s] = n;
      firstrecv[s] = nlocal + first[s];
      if (n > maxsendlist[s]) grow_list(s, n);
      for (int k = 0; k < n; k++) sendlist[s][k] = src[first[s] + k];
      if (n > most) most = n;
    }
    if (most > maxsend) grow_send(most, 0);
  }
};

template <class Base = PairSPHRhoSum>
struct HRhoSumT : public Base {
  HRhoSumT(LAMMPS *l) : Base(l) {}
  using PairSPHRhoSum::allocate;
  using PairSPHRhoSum::cut;
  using PairSPHRhoSum::nstep;
};
using HRhoSum = HRhoSumT<SPH_H(PairSPHRhoSum)>;
template <class Base = PairSPHTaitwater>
struct HTaitT : public Base {
  HTaitT(LAMMPS *l) : Base(l) {}
  using PairSPHTaitwater::allocate;
  using PairSPHTaitwater::cut;
  using PairSPHTaitwater::rho0;
  using PairSPHTaitwater::soundspeed;
  using PairSPHTaitwater::B;
  using PairSPHTaitwater::viscosity;
};
using HTait = HTaitT<SPH_H(PairSPHTaitwater)>;
template <class Base = PairSPHTaitwaterMorris>
struct HMorrisT : public Base {
  HMorrisT(LAMMPS *l) : Base(l) {}
  using PairSPHTaitwaterMorris::allocate;
  using PairSPHTaitwaterMorris::cut;
  using PairSPHTaitwaterMorris::rho0;
  using PairSPHTaitwaterMorris::soundspeed;
  using PairSPHTaitwaterMorris::B;
  using PairSPHTaitwaterMorris::viscosity;
};
using HMorris = HMorrisT<SPH_H(PairSPHTaitwaterMorris)>;
template <class Base = PairSPHHeatConduction>
struct HHeatT : public Base {
  HHeatT(LAMMPS *l) : Base(l) {}
  using PairSPHHeatConduction::allocate;
  using PairSPHHeatConduction::cut;
  using PairSPHHeatConduction::alpha;
};
using HHeat = HHeatT<SPH_H(PairSPHHeatConduction)>;
template <class Base = PairSPHRhoSumMultiphase>
struct HRhoMPT : public Base {
  HRhoMPT(LAMMPS *l) : Base(l) {}
  using PairSPHRhoSumMultiphase::allocate;
  using PairSPHRhoSumMultiphase::cut;
  using PairSPHRhoSumMultiphase::nstep;
};
using HRhoMP = HRhoMPT<SPH_H(PairSPHRhoSumMultiphase)>;
template <class Base = PairSPHTaitwaterMultiphase>
struct HTaitMPT : public Base {
  HTaitMPT(LAMMPS *l) : Base(l) {}
  using PairSPHTaitwaterMultiphase::allocate;
  using PairSPHTaitwaterMultiphase::cut;
  using PairSPHTaitwaterMultiphase::rho0;
  using PairSPHTaitwaterMultiphase::soundspeed;
  using PairSPHTaitwaterMultiphase::B;
  using PairSPHTaitwaterMultiphase::gamma;
  using PairSPHTaitwaterMultiphase::rbackground;
  using PairSPHTaitwaterMultiphase::viscosity;
};
using HTaitMP = HTaitMPT<SPH_H(PairSPHTaitwaterMultiphase)>;
template <class Base = PairSPHHeatConductionPhaseChange>
struct HHeatPCT : public Base {
  HHeatPCT(LAMMPS *l) : Base(l) {}
  using PairSPHHeatConductionPhaseChange::allocate;
  using PairSPHHeatConductionPhaseChange::cut;
  using PairSPHHeatConductionPhaseChange::alpha;
  using PairSPHHeatConductionPhaseChange::fixflag;
  using PairSPHHeatConductionPhaseChange::tc;
};
using HHeatPC = HHeatPCT<SPH_H(PairSPHHeatConductionPhaseChange)>;
template <class Base = PairSPHSurfaceTension>
struct HSTT : public Base {
  HSTT(LAMMPS *l) : Base(l) {}
  using PairSPHSurfaceTension::allocate;
  using PairSPHSurfaceTension::cut;
};
using HST = HSTT<SPH_H(PairSPHSurfaceTension)>;

template <class Base = PairSPHColorGradient>
struct HCGT : public Base {
  HCGT(LAMMPS *l) : Base(l) {}
  using PairSPHColorGradient::allocate;
  using PairSPHColorGradient::cut;
  using PairSPHColorGradient::alpha;
  using PairSPHColorGradient::nstep;
};
using HCG = HCGT<SPH_H(PairSPHColorGradient)>;

// One self-contained "LAMMPS" universe per call: owned atoms + ghosts supplied by the
// caller (positions already imaged), newton_pair as given.
struct World {
  LAMMPS *lmp;
  HComm *comm;
  HNeighbor *neigh;
  AtomVec *avec;
  int nall;

  World(int dim, int ntypes, int nlocal, int nghost, int newton, int multiphase) {
    lmp = zalloc<LAMMPS>();
    lmp->world = MPI_COMM_WORLD;
    lmp->screen = stdout;  // (Error::all / Error::one print there, error.cpp)
    lmp->logfile = NULL;
    lmp->universe = zalloc<Universe>();
    lmp->universe->nworlds = 1;
    lmp->memory = new Memory(lmp);
    lmp->error = new Error(lmp);
    lmp->atom = zalloc<Atom>();
    lmp->domain = zalloc<Domain>();
    lmp->force = zalloc<Force>();
    lmp->update = zalloc<Update>();
    lmp->domain->dimension = dim;
    lmp->domain->triclinic = 0;
    lmp->force->newton_pair = newton;
    lmp->force->newton = newton;
    lmp->update->ntimestep = 0;
    comm = new HComm(lmp);
    lmp->comm = comm;
    neigh = new HNeighbor(lmp);
    lmp->neighbor = neigh;
    Atom *atom = lmp->atom;
    atom->ntypes = ntypes;
    atom->nlocal = nlocal;
    atom->nghost = nghost;
    nall = nlocal + nghost;
    if (multiphase)
      avec = new AtomVecMesoMultiPhase(lmp);
    else
      avec = new AtomVecMeso(lmp);
    atom->avec = avec;
    avec->grow(nall > 0 ? nall : 1);
    atom->mass = (double *)calloc(ntypes + 1, sizeof(double));
    atom->rmass_flag = multiphase;
  }
};

void fill_atoms(World &w, const double *x, const double *vest, const double *rho,
                const double *e, const double *cv, const int *type, const double *rmass) {
  Atom *a = w.lmp->atom;
  for (int i = 0; i < w.nall; i++) {
    for (int k = 0; k < 3; k++) {
      a->x[i][k] = x[3 * i + k];
      a->f[i][k] = 0.0;
      if (a->vest) a->vest[i][k] = vest ? vest[3 * i + k] : 0.0;
      if (a->v) a->v[i][k] = vest ? vest[3 * i + k] : 0.0;
    }
    a->type[i] = type[i];
    a->mask[i] = 1;
    if (a->rho) a->rho[i] = rho ? rho[i] : 0.0;
    if (a->drho) a->drho[i] = 0.0;
    if (a->e) a->e[i] = e ? e[i] : 0.0;
    if (a->de) a->de[i] = 0.0;
    if (a->cv) a->cv[i] = cv ? cv[i] : 0.0;
    if (a->rmass && rmass) a->rmass[i] = rmass[i];
  }
}

// Build a NeighList from caller CSR (owned atoms, ilist = identity).
NeighList *make_list(World &w, int nlocal, const long *off, const int *neigh) {
  NeighList *l = new NeighList(w.lmp);
  l->inum = nlocal;
  l->gnum = 0;
  l->ilist = (int *)malloc(sizeof(int) * (nlocal > 0 ? nlocal : 1));
  l->numneigh = (int *)malloc(sizeof(int) * (nlocal > 0 ? nlocal : 1));
  l->firstneigh = (int **)malloc(sizeof(int *) * (nlocal > 0 ? nlocal : 1));
  for (int i = 0; i < nlocal; i++) {
    l->ilist[i] = i;
    l->numneigh[i] = (int)(off[i + 1] - off[i]);
    l->firstneigh[i] = const_cast<int *>(neigh) + off[i];
  }
  return l;
}

void free_list(NeighList *l) {
  free(l->ilist);
  free(l->numneigh);
  free(l->firstneigh);
  l->ilist = NULL;
  l->numneigh = NULL;
  l->firstneigh = NULL;
}

// Device-built lists through the /hip classes (sph_hip_build_list): while on, the pair
// drivers below make their style force->pair and set neighbor->skin for the duration of
// compute(), the shim's device-list path then builds the lists from cutsq + skin exactly
// as Neighbor::init sizes them; off (default), the caller's lists are staged.
int g_devlists = 0;
double g_devskin = 0.0;
#ifdef SPH_SHIM
extern "C" void sph_hip_shim_set_device_lists(int on);
#endif
struct DevListScope {
  World &w;
  DevListScope(World &w_, Pair *p) : w(w_) {
#ifdef SPH_SHIM
    sph_hip_shim_set_device_lists(g_devlists);
#endif
    if (g_devlists) {
      w.lmp->force->pair = p;
      w.neigh->skin = g_devskin;
    }
  }
  ~DevListScope() { w.lmp->force->pair = NULL; }
};

// Pair::init (pair.cpp:174-229) minus init_style (no neighbor request machinery here):
// cutsq[i][j] = cutsq[j][i] = cut*cut with cut = init_one(i,j).
void pair_init_cutsq(Pair *p, int ntypes) {
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      double cut = p->init_one(i, j);
      p->cutsq[i][j] = p->cutsq[j][i] = cut * cut;
    }
}

}  // namespace

extern "C" {

// Full list by the reference's own binned builder.  x holds nlocal owned + nghost ghost
// atoms.  cutneighsq is (nt+1)^2.  On return off[0..nlocal], neigh[] (cap entries).
long REFNAME(neigh_full)(int dim, int ntypes, int nlocal, int nghost, const double *x,
                    const int *type, const double *boxlo, const double *boxhi,
                    const double *sublo, const double *subhi, double cutghost,
                    const double *cutneighsq, long *off, int *neigh, long cap) {
  World w(dim, ntypes, nlocal, nghost, 1, 0);
  fill_atoms(w, x, NULL, NULL, NULL, NULL, type, NULL);
  Domain *d = w.lmp->domain;
  for (int k = 0; k < 3; k++) {
    d->boxlo[k] = boxlo[k];
    d->boxhi[k] = boxhi[k];
    d->sublo[k] = sublo[k];
    d->subhi[k] = subhi[k];
    d->prd[k] = boxhi[k] - boxlo[k];
    w.comm->cutghost[k] = cutghost;
  }
  HNeighbor *n = w.neigh;
  n->dimension = dim;
  n->triclinic = 0;
  n->exclude = 0;
  n->bboxlo = d->boxlo;
  n->bboxhi = d->boxhi;
  w.lmp->memory->create(n->cutneighsq, ntypes + 1, ntypes + 1, "neigh:cutneighsq");
  double cmax = 0.0;
  for (int i = 0; i <= ntypes; i++)
    for (int j = 0; j <= ntypes; j++) {
      n->cutneighsq[i][j] = cutneighsq[i * (ntypes + 1) + j];
      if (i && j) cmax = fmax(cmax, sqrt(cutneighsq[i * (ntypes + 1) + j]));
    }
  n->cutneighmax = cmax;
  n->cutneighmaxsq = cmax * cmax;  // Neighbor::init, neighbor.cpp:280
  n->setup_bins();
  // Neighbor::build, neighbor.cpp:1477-1481: bins sized to atom->nmax
  n->maxbin = w.lmp->atom->nmax;
  w.lmp->memory->create(n->bins, n->maxbin, "bins");
  NeighList *l = new NeighList(w.lmp);
  l->setup_pages(100000, 2000, 0);
  l->grow(nlocal + nghost + 1);
  l->stencil_allocate(n->smax, 1 /*BIN: enum{NSQ,BIN,MULTI}, neigh_list.cpp:28*/);
  if (dim == 3)
    n->stencil_full_bin_3d(l, n->sx, n->sy, n->sz);
  else
    n->stencil_full_bin_2d(l, n->sx, n->sy, n->sz);
  n->full_bin(l);  // bins atoms itself (binatomflag = 1)
  long tot = 0;
  for (int ii = 0; ii < l->inum; ii++) {
    int i = l->ilist[ii];
    off[i] = tot;
    tot += l->numneigh[i];
  }
  off[nlocal] = tot;
  if (neigh) {
    if (tot > cap) return -1;
    for (int ii = 0; ii < l->inum; ii++) {
      int i = l->ilist[ii];
      memcpy(neigh + off[i], l->firstneigh[i], sizeof(int) * l->numneigh[i]);
    }
  }
  return tot;
}

// Neighbor::half_from_full_newton on a caller full list.
long REFNAME(neigh_half_from_full)(int nlocal, int nghost, const double *x, const long *foff,
                              const int *fneigh, long *hoff, int *hneigh) {
  World w(3, 1, nlocal, nghost, 1, 0);
  int *type = (int *)calloc(nlocal + nghost + 1, sizeof(int));
  for (int i = 0; i < nlocal + nghost; i++) type[i] = 1;
  fill_atoms(w, x, NULL, NULL, NULL, NULL, type, NULL);
  free(type);
  NeighList *full = make_list(w, nlocal, foff, fneigh);
  NeighList *half = new NeighList(w.lmp);
  half->setup_pages(100000, 2000, 0);
  half->grow(nlocal + nghost + 1);
  half->listfull = full;
  w.neigh->half_from_full_newton(half);
  long tot = 0;
  for (int ii = 0; ii < half->inum; ii++) {
    int i = half->ilist[ii];
    hoff[i] = tot;
    if (hneigh) memcpy(hneigh + tot, half->firstneigh[i], sizeof(int) * half->numneigh[i]);
    tot += half->numneigh[i];
  }
  hoff[nlocal] = tot;
  free_list(full);
  return tot;
}

// PairSPHRhoSum: coeff semantics pair_sph_rhosum.cpp:239-263 (cut[i][j] = h, j>=i).
// rho is nall long; owned entries are written; ghosts untouched (forward comm is the
// caller's job -- nswap = 0 here).
int REFNAME(rhosum)(int dim, int ntypes, int nlocal, int nghost, const double *x,
               const int *type, const double *mass, const double *cut, const long *off,
               const int *neigh, double *rho) {
  World w(dim, ntypes, nlocal, nghost, 1, 0);
  fill_atoms(w, x, NULL, rho, NULL, NULL, type, NULL);
  for (int t = 0; t <= ntypes; t++) w.lmp->atom->mass[t] = mass[t];
  HRhoSum *p = new HRhoSum(w.lmp);
  p->nstep = 1;
  p->allocate();
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->setflag[i][j] = 1;
    }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  {
    DevListScope dl(w, p);
    p->compute(0, 0);
  }
  for (int i = 0; i < nlocal; i++) rho[i] = w.lmp->atom->rho[i];
  free_list(l);
  return 0;
}

// PairSPHRhoSum as a hybrid/overlay sub-style with a SKIP list (pair_hybrid.cpp:428-485):
// coefficients only where ijskip[i][j] == 0 (the others left as allocate() leaves them --
// poisoned with NaN here, so a path that reads them shows), the caller's list holds the rows
// of types with iskip == 0 (ilist) and only pairs with ijskip == 0, and carries the skip info
// as NeighList::copy_skip_info sets it (neigh_list.cpp:204-215).
int REFNAME(rhosum_skip)(int dim, int ntypes, int nlocal, int nghost, const double *x,
                    const int *type, const double *mass, const double *cut, int inum,
                    const int *ilist, const long *off, const int *neigh, const int *iskip,
                    const int *ijskip, double *rho) {
  World w(dim, ntypes, nlocal, nghost, 1, 0);
  fill_atoms(w, x, NULL, rho, NULL, NULL, type, NULL);
  for (int t = 0; t <= ntypes; t++) w.lmp->atom->mass[t] = mass[t];
  HRhoSum *p = new HRhoSum(w.lmp);
  p->nstep = 1;
  p->allocate();
  const double nan = std::nan("");
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      const bool on = ijskip[i * (ntypes + 1) + j] == 0;
      p->cut[i][j] = on ? cut[i * (ntypes + 1) + j] : nan;
      p->setflag[i][j] = on ? 1 : 0;
    }
  for (int i = 1; i <= ntypes; i++)  // (init_one of the assigned pairs only, as hybrid's)
    for (int j = i; j <= ntypes; j++)
      if (p->setflag[i][j]) {
        const double c = p->init_one(i, j);
        p->cutsq[i][j] = p->cutsq[j][i] = c * c;
      } else {
        p->cutsq[i][j] = p->cutsq[j][i] = nan;
      }
  NeighList *l = new NeighList(w.lmp);
  l->inum = inum;
  l->gnum = 0;
  l->ilist = (int *)malloc(sizeof(int) * (inum > 0 ? inum : 1));
  // (numneigh / firstneigh are indexed by the atom, not the list position)
  l->numneigh = (int *)calloc(nlocal > 0 ? nlocal : 1, sizeof(int));
  l->firstneigh = (int **)calloc(nlocal > 0 ? nlocal : 1, sizeof(int *));
  for (int k = 0; k < inum; k++) {
    const int i = ilist[k];
    l->ilist[k] = i;
    l->numneigh[i] = (int)(off[k + 1] - off[k]);
    l->firstneigh[i] = const_cast<int *>(neigh) + off[k];
  }
  {
    std::vector<int> is(iskip, iskip + ntypes + 1);
    int **ij;
    w.lmp->memory->create(ij, ntypes + 1, ntypes + 1, "harness:ijskip");
    for (int i = 0; i <= ntypes; i++)
      for (int j = 0; j <= ntypes; j++) ij[i][j] = ijskip[i * (ntypes + 1) + j];
    l->copy_skip_info(is.data(), ij);
    w.lmp->memory->destroy(ij);
  }
  p->list = l;
  SPH_INIT(p);
  {
    // (device lists on: the style is force->pair, whose cutsq the shim would size the
    // device list from -- a hybrid's covers every pair, here the assigned ones are NaN)
    DevListScope dl(w, p);
    p->compute(0, 0);
  }
  for (int i = 0; i < nlocal; i++) rho[i] = w.lmp->atom->rho[i];
  free_list(l);
  return 0;
}

// PairSPHTaitwater / Morris: coeff semantics pair_sph_taitwater.cpp:238-276 including the
// per-type "last write wins" of rho0/c0/B; here the caller passes per-type rho0/c0 and
// per-pair visc/cut (j>=i), and B = c0^2 rho0 / 7 as coeff() computes it.
static int run_tait(int morris, int dim, int ntypes, int nlocal, int nghost, int newton,
                    const double *x, const double *vest, const double *rho, const int *type,
                    const double *mass, const double *rho0, const double *c0,
                    const double *visc, const double *cut, const long *off,
                    const int *neigh, double *f, double *drho, double *de) {
  World w(dim, ntypes, nlocal, nghost, newton, 0);
  fill_atoms(w, x, vest, rho, NULL, NULL, type, NULL);
  for (int t = 0; t <= ntypes; t++) w.lmp->atom->mass[t] = mass[t];
  Pair *p;
  if (morris) {
    HMorris *q = new HMorris(w.lmp);
    q->allocate();
    for (int i = 1; i <= ntypes; i++) {
      q->rho0[i] = rho0[i];
      q->soundspeed[i] = c0[i];
      q->B[i] = c0[i] * c0[i] * rho0[i] / 7.0;
      for (int j = i; j <= ntypes; j++) {
        q->viscosity[i][j] = visc[i * (ntypes + 1) + j];
        q->cut[i][j] = cut[i * (ntypes + 1) + j];
        q->setflag[i][j] = 1;
      }
    }
    p = q;
  } else {
    HTait *q = new HTait(w.lmp);
    q->allocate();
    for (int i = 1; i <= ntypes; i++) {
      q->rho0[i] = rho0[i];
      q->soundspeed[i] = c0[i];
      q->B[i] = c0[i] * c0[i] * rho0[i] / 7.0;
      for (int j = i; j <= ntypes; j++) {
        q->viscosity[i][j] = visc[i * (ntypes + 1) + j];
        q->cut[i][j] = cut[i * (ntypes + 1) + j];
        q->setflag[i][j] = 1;
      }
    }
    p = q;
  }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  {
    DevListScope dl(w, p);
    p->compute(0, 0);
  }
  Atom *a = w.lmp->atom;
  for (int i = 0; i < nlocal + nghost; i++) {
    for (int k = 0; k < 3; k++) f[3 * i + k] = a->f[i][k];
    drho[i] = a->drho[i];
    de[i] = a->de[i];
  }
  free_list(l);
  return 0;
}

int REFNAME(taitwater)(int dim, int ntypes, int nlocal, int nghost, int newton, const double *x,
                  const double *vest, const double *rho, const int *type, const double *mass,
                  const double *rho0, const double *c0, const double *visc,
                  const double *cut, const long *off, const int *neigh, double *f,
                  double *drho, double *de) {
  return run_tait(0, dim, ntypes, nlocal, nghost, newton, x, vest, rho, type, mass, rho0, c0,
                  visc, cut, off, neigh, f, drho, de);
}

int REFNAME(taitwater_morris)(int dim, int ntypes, int nlocal, int nghost, int newton,
                         const double *x, const double *vest, const double *rho,
                         const int *type, const double *mass, const double *rho0,
                         const double *c0, const double *visc, const double *cut,
                         const long *off, const int *neigh, double *f, double *drho,
                         double *de) {
  return run_tait(1, dim, ntypes, nlocal, nghost, newton, x, vest, rho, type, mass, rho0, c0,
                  visc, cut, off, neigh, f, drho, de);
}

// PairSPHHeatConduction: coeff pair_sph_heatconduction.cpp:(alpha, cut) for j>=i.
int REFNAME(heatconduction)(int dim, int ntypes, int nlocal, int nghost, int newton,
                       const double *x, const double *e, const double *rho, const int *type,
                       const double *mass, const double *alpha, const double *cut,
                       const long *off, const int *neigh, double *de) {
  World w(dim, ntypes, nlocal, nghost, newton, 0);
  fill_atoms(w, x, NULL, rho, e, NULL, type, NULL);
  for (int t = 0; t <= ntypes; t++) w.lmp->atom->mass[t] = mass[t];
  HHeat *p = new HHeat(w.lmp);
  p->allocate();
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      p->alpha[i][j] = alpha[i * (ntypes + 1) + j];
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->setflag[i][j] = 1;
    }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  {
    DevListScope dl(w, p);
    p->compute(0, 0);
  }
  for (int i = 0; i < nlocal + nghost; i++) de[i] = w.lmp->atom->de[i];
  free_list(l);
  return 0;
}

// the device-list switch of the single-phase drivers above (DevListScope)
void REFNAME(set_device_lists)(int on, double skin) {
  g_devlists = on;
  g_devskin = skin;
}

// ---- multiphase styles (atom_style meso/multiphase: per-atom rmass) -------------------

int REFNAME(rhosum_multiphase)(int dim, int ntypes, int nlocal, int nghost, const double *x,
                          const int *type, const double *rmass, const double *cut,
                          const long *off, const int *neigh, double *rho) {
  World w(dim, ntypes, nlocal, nghost, 1, 1);
  fill_atoms(w, x, NULL, rho, NULL, NULL, type, rmass);
  HRhoMP *p = new HRhoMP(w.lmp);
  p->nstep = 1;
  p->allocate();
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->setflag[i][j] = 1;
    }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  p->compute(0, 0);
  for (int i = 0; i < nlocal; i++) rho[i] = w.lmp->atom->rho[i];
  free_list(l);
  return 0;
}

// coeff: pair_sph_taitwater_multiphase.cpp:225-262 (B = c^2 rho0 / gamma).
int REFNAME(taitwater_multiphase)(int dim, int ntypes, int nlocal, int nghost, int newton,
                             const double *x, const double *vest, const double *rho,
                             const int *type, const double *rmass, const double *rho0,
                             const double *c0, const double *gamma, const double *rbg,
                             const double *visc, const double *cut, const long *off,
                             const int *neigh, double *f) {
  World w(dim, ntypes, nlocal, nghost, newton, 1);
  fill_atoms(w, x, vest, rho, NULL, NULL, type, rmass);
  HTaitMP *p = new HTaitMP(w.lmp);
  p->allocate();
  for (int i = 1; i <= ntypes; i++) {
    p->rho0[i] = rho0[i];
    p->gamma[i] = gamma[i];
    p->soundspeed[i] = c0[i];
    p->B[i] = c0[i] * c0[i] * rho0[i] / gamma[i];
    p->rbackground[i] = rbg[i];
    for (int j = i; j <= ntypes; j++) {
      p->viscosity[i][j] = visc[i * (ntypes + 1) + j];
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->setflag[i][j] = 1;
    }
  }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  p->compute(0, 0);
  for (int i = 0; i < nlocal + nghost; i++)
    for (int k = 0; k < 3; k++) f[3 * i + k] = w.lmp->atom->f[i][k];
  free_list(l);
  return 0;
}

// coeff: pair_sph_heatconduction_phasechange.cpp:177-225.  fixflag/tc per pair (j>=i),
// 0 meaning "no clamp" (the 4-arg form leaves them uninitialised: quirk A.6-4).
int REFNAME(heatconduction_phasechange)(int dim, int ntypes, int nlocal, int nghost, int newton,
                                   const double *x, const double *e, const double *cv,
                                   const double *rho, const double *rmass, const int *type,
                                   const double *alpha, const int *fixflag,
                                   const double *tc, const double *cut, const long *off,
                                   const int *neigh, double *de) {
  World w(dim, ntypes, nlocal, nghost, newton, 1);
  fill_atoms(w, x, NULL, rho, e, cv, type, rmass);
  HHeatPC *p = new HHeatPC(w.lmp);
  p->allocate();
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      p->alpha[i][j] = alpha[i * (ntypes + 1) + j];
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->fixflag[i][j] = fixflag ? fixflag[i * (ntypes + 1) + j] : 0;
      p->tc[i][j] = tc ? tc[i * (ntypes + 1) + j] : 0.0;
      p->setflag[i][j] = 1;
    }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  p->compute(0, 0);
  for (int i = 0; i < nlocal + nghost; i++) de[i] = w.lmp->atom->de[i];
  free_list(l);
  return 0;
}

int REFNAME(colorgradient)(int dim, int ntypes, int nlocal, int nghost, const double *x,
                      const double *rho, const double *rmass, const int *type,
                      const double *alpha, const double *cut, const long *off,
                      const int *neigh, double *cg) {
  World w(dim, ntypes, nlocal, nghost, 1, 1);
  fill_atoms(w, x, NULL, rho, NULL, NULL, type, rmass);
  HCG *p = new HCG(w.lmp);
  p->nstep = 1;
  p->allocate();
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      p->alpha[i][j] = alpha[i * (ntypes + 1) + j];
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->setflag[i][j] = 1;
    }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  p->compute(0, 0);
  for (int i = 0; i < nlocal; i++)
    for (int k = 0; k < 3; k++) cg[3 * i + k] = w.lmp->atom->colorgradient[i][k];
  free_list(l);
  return 0;
}

// PairSPHSurfaceTension (coeff pair_sph_surfacetension.cpp:222-247: cut per pair).  cg is
// the caller's colorgradient for all nall atoms (atom->colorgradient); f (nall*3) out.
int REFNAME(surfacetension)(int dim, int ntypes, int nlocal, int nghost, int newton,
                       const double *x, const double *rho, const double *rmass,
                       const int *type, const double *cg, const double *cut, const long *off,
                       const int *neigh, double *f) {
  World w(dim, ntypes, nlocal, nghost, newton, 1);
  fill_atoms(w, x, NULL, rho, NULL, NULL, type, rmass);
  for (int i = 0; i < nlocal + nghost; i++)
    for (int k = 0; k < 3; k++) w.lmp->atom->colorgradient[i][k] = cg[3 * i + k];
  HST *p = new HST(w.lmp);
  p->allocate();
  for (int i = 1; i <= ntypes; i++)
    for (int j = i; j <= ntypes; j++) {
      p->cut[i][j] = cut[i * (ntypes + 1) + j];
      p->setflag[i][j] = 1;
    }
  pair_init_cutsq(p, ntypes);
  NeighList *l = make_list(w, nlocal, off, neigh);
  p->list = l;
  SPH_INIT(p);
  p->compute(0, 0);
  for (int i = 0; i < nlocal + nghost; i++)
    for (int k = 0; k < 3; k++) f[3 * i + k] = w.lmp->atom->f[i][k];
  free_list(l);
  return 0;
}

// FixMeso / FixMesoStationary (fix_meso.cpp, fix_meso_stationary.cpp), built by their own
// constructors ("ID group style", Fix::Fix -> Group::find) on the group "g" = the atoms whose
// type is in tmask (0: group "all"), then init() (dtv, dtf from update->dt, force->ftm2v) and
// one call: phase 0 = setup_pre_force (FixMeso), 1 = initial_integrate, 2 = final_integrate.
// Arrays are owned atoms, updated in place.
int REFNAME(fix_meso)(int stationary, int phase, int nlocal, int ntypes, double dt, const int *type,
                 int tmask, const double *mass, double *x, double *v, const double *f,
                 double *vest, double *rho, const double *drho, double *e, const double *de) {
  World w(3, ntypes, nlocal, 0, 1, 0);
  Atom *a = w.lmp->atom;
  a->firstgroup = -1;  // (Atom::Atom's default; the zero-allocated Atom has 0 = "all")
  w.lmp->update->dt = dt;
  w.lmp->force->ftm2v = 1.0;
  Group *grp = new Group(w.lmp);
  w.lmp->group = grp;
  grp->names[1] = new char[2];
  strcpy(grp->names[1], "g");
  grp->ngroup = 2;
  for (int t = 0; t <= ntypes; t++) a->mass[t] = mass[t];
  for (int i = 0; i < nlocal; i++) {
    for (int k = 0; k < 3; k++) {
      a->x[i][k] = x[3 * i + k];
      a->v[i][k] = v[3 * i + k];
      a->f[i][k] = f[3 * i + k];
      a->vest[i][k] = vest[3 * i + k];
    }
    a->type[i] = type[i];
    a->mask[i] = 1 | (((tmask >> type[i]) & 1) ? grp->bitmask[1] : 0);
    a->rho[i] = rho[i];
    a->drho[i] = drho[i];
    a->e[i] = e[i];
    a->de[i] = de[i];
  }
  char id[] = "f1", all[] = "all", g[] = "g", meso[] = "meso", stat[] = "meso/stationary";
  char *arg[3] = {id, tmask ? g : all, stationary ? stat : meso};
  Fix *fix;
  if (stationary)
    fix = new FixMesoStationary(w.lmp, 3, arg);
  else
    fix = new FixMeso(w.lmp, 3, arg);
  fix->init();
  if (phase == 0) {
    if (stationary) return -1;  // (meso/stationary has no setup_pre_force)
    fix->setup_pre_force(0);
  } else if (phase == 1) {
    fix->initial_integrate(0);
  } else {
    fix->final_integrate();
  }
  for (int i = 0; i < nlocal; i++) {
    for (int k = 0; k < 3; k++) {
      x[3 * i + k] = a->x[i][k];
      v[3 * i + k] = a->v[i][k];
      vest[3 * i + k] = a->vest[i][k];
    }
    rho[i] = a->rho[i];
    e[i] = a->e[i];
  }
  return 0;
}


// ---- FixPhaseChange (fix_phase_change.cpp), constructed from its own argument list -------
// A persistent one-process universe: the fix keeps its RanPark stream across
// ref_pc_pre_exchange calls exactly as it does across a LAMMPS run.  The fix's region is a
// real RegBlock ("block EDGE x6 units box" = the box, region_block.cpp:26-92), found through
// Domain::find_region (restated at the bottom of this file: domain.cpp needs the generated
// style_region.h).  Atom::tag_extend and Atom::map_* (atom.cpp, not built) are kept out of
// reach with tag_enable = map_style = 0: tags are the caller's bookkeeping.
struct PCWorld {
  World *w;
  Fix *fix;
  NeighList *list;
};

void *REFNAME(pc_new)(int dim, int ntypes, const double *boxlo, const double *boxhi, long step0,
                 double dt, int narg, const char **args) {
  PCWorld *pw = new PCWorld;
  pw->w = new World(dim, ntypes, 0, 0, 1, 1);
  World &w = *pw->w;
  LAMMPS *lmp = w.lmp;
  Domain *d = lmp->domain;
  d->box_exist = 1;
  for (int k = 0; k < 3; k++) {
    d->boxlo[k] = d->sublo[k] = boxlo[k];
    d->boxhi[k] = d->subhi[k] = boxhi[k];
    d->prd[k] = boxhi[k] - boxlo[k];
    w.comm->procgrid[k] = 1;
    w.comm->myloc[k] = 0;
  }
  lmp->update->ntimestep = step0;
  lmp->update->dt = dt;
  lmp->modify = zalloc<Modify>();
  lmp->group = new Group(lmp);
  lmp->atom->tag_enable = 0;
  lmp->atom->map_style = 0;
  char rid[] = "box", rst[] = "block", edge[] = "EDGE", un[] = "units", bx[] = "box";
  char *rarg[10] = {rid, rst, edge, edge, edge, edge, edge, edge, un, bx};
  d->maxregion = 1;
  d->nregion = 1;
  d->regions = (Region **)calloc(1, sizeof(Region *));
  d->regions[0] = new RegBlock(lmp, 10, rarg);
  pw->fix = new SPH_H(FixPhaseChange)(lmp, narg, const_cast<char **>(args));
  pw->fix->init();  // Fix::init (find_region, the full-list request)
  pw->list = NULL;
  return pw;
}

// One Modify::pre_exchange of the fix at `step` on nlocal owned + nghost ghost atoms (in
// LAMMPS' index order, ghosts right after the owned atoms) in arrays with room for nmax
// atoms; the FULL list rows cover the owned atoms.  Arrays are updated in place; returns
// atom->nlocal afterwards (created atoms sit at [nlocal, return)).
int REFNAME(pc_pre_exchange)(void *h, long step, int nlocal, int nghost, int nmax, double *x,
                        double *v, double *vest, double *cg, double *e, double *rmass,
                        double *rho, double *cv, int *type, const long *off, const int *neigh,
                        int nswap, const int *swap_first, const int *ghost_src,
                        long *next_reneighbor) {
  PCWorld *pw = static_cast<PCWorld *>(h);
  World &w = *pw->w;
  Atom *a = w.lmp->atom;
  a->nlocal = nlocal;
  a->nghost = nghost;
  w.nall = nlocal + nghost;
  w.avec->grow(nmax);
  for (int i = 0; i < w.nall; i++) {
    for (int k = 0; k < 3; k++) {
      a->x[i][k] = x[3 * i + k];
      a->v[i][k] = v[3 * i + k];
      a->vest[i][k] = vest[3 * i + k];
      a->colorgradient[i][k] = cg[3 * i + k];
      a->f[i][k] = 0.0;
    }
    a->e[i] = e[i];
    a->rmass[i] = rmass[i];
    a->rho[i] = rho[i];
    a->cv[i] = cv[i];
    a->type[i] = type[i];
    a->mask[i] = 1;
    a->tag[i] = 0;
    a->drho[i] = 0.0;
    a->de[i] = 0.0;
  }
  if (pw->list) free_list(pw->list);
  pw->list = make_list(w, nlocal, off, neigh);
  pw->fix->init_list(0, pw->list);
  w.comm->set_self_swaps(nlocal, nswap, swap_first, ghost_src);
  w.lmp->update->ntimestep = step;
  pw->fix->pre_exchange();
  const int n = a->nlocal;
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 3; k++) {
      x[3 * i + k] = a->x[i][k];
      v[3 * i + k] = a->v[i][k];
      vest[3 * i + k] = a->vest[i][k];
      cg[3 * i + k] = a->colorgradient[i][k];
    }
    e[i] = a->e[i];
    rmass[i] = a->rmass[i];
    rho[i] = a->rho[i];
    cv[i] = a->cv[i];
    type[i] = a->type[i];
  }
  if (next_reneighbor) *next_reneighbor = pw->fix->next_reneighbor;
  return n;
}

// ---- per-atom restart records: AtomVecMeso::pack_restart (atom_vec_meso.cpp:729-757) and
// AtomVecMesoMultiPhase::pack_restart (atom_vec_meso_multiphase.cpp:887-916), one call per
// atom into rec[i*stride...]; returns the record length the routine reported.
int REFNAME(pack_restart)(int multiphase, int n, const double *x, const int *tag, const int *type,
                     const int *mask, const int *image, const double *v, const double *rho,
                     const double *cg, const double *rmass, const double *e, const double *cv,
                     const double *vest, int stride, double *rec) {
  World w(3, 8, n, 0, 1, multiphase);
  Atom *a = w.lmp->atom;
  int len = 0;
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 3; k++) {
      a->x[i][k] = x[3 * i + k];
      a->v[i][k] = v[3 * i + k];
      a->vest[i][k] = vest[3 * i + k];
      if (multiphase) a->colorgradient[i][k] = cg[3 * i + k];
    }
    a->tag[i] = tag[i];
    a->type[i] = type[i];
    a->mask[i] = mask[i];
    a->image[i] = image[i];
    a->rho[i] = rho[i];
    a->e[i] = e[i];
    a->cv[i] = cv[i];
    if (multiphase) a->rmass[i] = rmass[i];
  }
  for (int i = 0; i < n; i++) len = w.avec->pack_restart(i, rec + (size_t)i * stride);
  return len;
}

double REFNAME(kernel_quintic3d)(double r);
double REFNAME(dw_quintic3d)(double r);
}

#include "sph_kernel_quintic.h"
extern "C" double REFNAME(kernel_quintic3d)(double r) { return sph_kernel_quintic3d(r); }
extern "C" double REFNAME(dw_quintic3d)(double r) { return sph_dw_quintic3d(r); }
extern "C" double REFNAME(kernel_quintic2d)(double r) { return sph_kernel_quintic2d(r); }
extern "C" double REFNAME(dw_quintic2d)(double r) { return sph_dw_quintic2d(r); }

// Domain::find_region (domain.cpp:1436-1441), restated: domain.cpp itself needs the
// generated style_region.h, so it is not part of the reference build here.
int LAMMPS_NS::Domain::find_region(char *name) {
  for (int iregion = 0; iregion < nregion; iregion++)
    if (strcmp(name, regions[iregion]->id) == 0) return iregion;
  return -1;
}

#ifdef SPH_SHIM
// Style registration as LAMMPS does it: force.cpp:81-88 turns every PairStyle(key, Class)
// line of the generated style_pair.h into a creator map entry, modify.cpp likewise for
// FixStyle; with "-sf hip" Force::new_pair / Modify::add_fix first try "style/hip"
// (force.cpp:148-166).  Here the /hip headers' own PairStyle/FixStyle lines are expanded
// the same way and `style` + "/" + suffix is looked up and constructed; cls gets the C++ type
// of the object created (empty: no such style).
extern "C" int shim_style_lookup(int is_fix, const char *style, const char *suffix, char *cls,
                                 int n) {
  World w(3, 2, 0, 0, 1, 1);
  const std::string want = std::string(style) + (suffix && *suffix ? "/" : "") +
                           (suffix ? suffix : "");
  Pair *p = NULL;
  const char *fixname = NULL;
  if (!is_fix) {
#define PAIR_CLASS
#define PairStyle(key, Class) \
  if (!p && want == #key) p = new Class(w.lmp);
#include "pair_sph_hip.h"
#undef PairStyle
#undef PAIR_CLASS
  } else {
#define FIX_CLASS
#define FixStyle(key, Class) \
  if (!fixname && want == #key) fixname = typeid(Class).name();
#include "fix_phase_change_hip.h"
#undef FixStyle
#undef FIX_CLASS
  }
  cls[0] = 0;
  if (p) snprintf(cls, n, "%s", typeid(*p).name());
  if (fixname) snprintf(cls, n, "%s", fixname);
  return cls[0] ? 1 : 0;
}
#endif
