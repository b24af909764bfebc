/*
 * sph_oracle.c -- CPU restatement of the USER-SPH hot path.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker; never linked into or called by the product library.  See sph_oracle.h for
 * the routine-by-routine map to the reference (paths relative to /root/reference).
 *
 * Arithmetic is kept in the reference's operation order so that, for identical inputs
 * and identical neighbor order, results are bit-identical to the reference loops.
 */
#include "sph_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define IDX2(nt, i, j) ((i) * ((nt) + 1) + (j))

/* ------------------------------------------------------------------------------------
   Domain::pbc, src/domain.cpp:478-560 (orthogonal box, image flags not tracked)
   ------------------------------------------------------------------------------------ */
void orc_pbc(const orc_domain *d, int nlocal, double *x) {
  for (int i = 0; i < nlocal; i++) {
    for (int k = 0; k < 3; k++) {
      if (!d->periodic[k]) continue;
      const double prd = d->boxhi[k] - d->boxlo[k];
      if (x[3 * i + k] < d->boxlo[k]) x[3 * i + k] += prd;
      if (x[3 * i + k] >= d->boxhi[k]) {
        x[3 * i + k] -= prd;
        x[3 * i + k] = fmax(x[3 * i + k], d->boxlo[k]);
      }
    }
  }
}

/* ------------------------------------------------------------------------------------
   CommBrick::setup (slablo/slabhi, src/comm_brick.cpp:330-380) + CommBrick::borders
   (src/comm_brick.cpp:696-864) for one process (procgrid 1x1x1, sublo/subhi = box).
   Per dim: swap 0 sends atoms with x[dim] in [-BIG, sublo+cutghost] and they arrive
   shifted by +prd (myloc==0 -> pbc=+1); swap 1 sends [subhi-cutghost, BIG] with -prd.
   Both swaps of a dim scan the atoms that existed before that dim (nfirst=0,
   nlast=nlocal+nghost at ineed==0).  Non-periodic dims send nothing (sendneed=0).
   Ghost coordinates are x + pbc*prd, one add per coordinate (atom_vec_meso.cpp:266-279).
   ------------------------------------------------------------------------------------ */
int orc_borders(const orc_domain *d, double cutghost, int nlocal, double *x, int *type,
                int nmax, int *ghost_owner, int *ghost_image) {
  return orc_borders_ex(d, cutghost, nlocal, x, type, nmax, ghost_owner, ghost_image, NULL,
                        NULL, NULL);
}

/* The same, also recording CommBrick's swap structure for a reverse comm done the
   reference's way (comm_brick.cpp:513-571, 999-1030): ghost_src[g] = the index the ghost
   was copied from (sendlist entry, owned or an earlier ghost), swap_first[s] = the first
   ghost of swap s (firstrecv - nlocal), swap_first[nswap] = nghost.  Non-periodic
   dimensions still count their two (empty) swaps, as CommBrick does. */
int orc_borders_ex(const orc_domain *d, double cutghost, int nlocal, double *x, int *type,
                   int nmax, int *ghost_owner, int *ghost_image, int *ghost_src,
                   int *swap_first, int *nswap) {
  int nall = nlocal, iswap = 0;
  const int ndim = (d->dim == 2) ? 2 : 3;
  for (int dim = 0; dim < ndim; dim++) {
    const double prd = d->boxhi[dim] - d->boxlo[dim];
    const int nlast = nall;
    for (int ineed = 0; ineed < 2; ineed++) {
      if (swap_first) swap_first[iswap] = nall - nlocal;
      iswap++;
      if (!d->periodic[dim]) continue;
      double lo, hi, shift;
      int pbc;
      if (ineed == 0) {
        lo = -1.0e20;
        hi = d->boxlo[dim] + cutghost;
        pbc = 1;
      } else {
        lo = d->boxhi[dim] - cutghost;
        hi = 1.0e20;
        pbc = -1;
      }
      shift = pbc * prd;
      for (int i = 0; i < nlast; i++) {
        const double c = x[3 * i + dim];
        if (c >= lo && c <= hi) {
          if (nall >= nmax) return -1;
          const int g = nall - nlocal;
          x[3 * nall + 0] = x[3 * i + 0];
          x[3 * nall + 1] = x[3 * i + 1];
          x[3 * nall + 2] = x[3 * i + 2];
          x[3 * nall + dim] = x[3 * i + dim] + shift;
          type[nall] = type[i];
          if (i < nlocal) {
            ghost_owner[g] = i;
            ghost_image[3 * g + 0] = ghost_image[3 * g + 1] = ghost_image[3 * g + 2] = 0;
          } else {
            const int gi = i - nlocal;
            ghost_owner[g] = ghost_owner[gi];
            ghost_image[3 * g + 0] = ghost_image[3 * gi + 0];
            ghost_image[3 * g + 1] = ghost_image[3 * gi + 1];
            ghost_image[3 * g + 2] = ghost_image[3 * gi + 2];
          }
          ghost_image[3 * g + dim] += pbc;
          if (ghost_src) ghost_src[g] = i;
          nall++;
        }
      }
    }
  }
  if (swap_first) swap_first[iswap] = nall - nlocal;
  if (nswap) *nswap = iswap;
  return nall - nlocal;
}

/* Fix::pack_reverse_comm / unpack_reverse_comm through CommBrick::reverse_comm_fix
   (comm_brick.cpp:999-1030) for self swaps: swaps in reverse order, each adding its
   ghosts' values onto the atoms they were copied from (an earlier ghost or the owner). */
void orc_reverse_swaps(int nlocal, int nswap, const int *swap_first, const int *ghost_src,
                       double *a) {
  for (int s = nswap - 1; s >= 0; s--)
    for (int g = swap_first[s]; g < swap_first[s + 1]; g++) a[ghost_src[g]] += a[nlocal + g];
}

/* AtomVecMeso::pack_comm/unpack_comm, src/USER-SPH/atom_vec_meso.cpp:246-360.
   Each coordinate of a ghost carries exactly one periodic add (its own dim's hop),
   so owner + image*prd reproduces the hop-by-hop value bit for bit. */
void orc_forward_comm(const orc_domain *d, int nlocal, int nghost, const int *ghost_owner,
                      const int *ghost_image, double *x, double *rho, double *e,
                      double *vest) {
  double prd[3];
  for (int k = 0; k < 3; k++) prd[k] = d->boxhi[k] - d->boxlo[k];
  for (int g = 0; g < nghost; g++) {
    const int i = nlocal + g, o = ghost_owner[g];
    for (int k = 0; k < 3; k++) {
      const int im = ghost_image[3 * g + k];
      x[3 * i + k] = im ? x[3 * o + k] + im * prd[k] : x[3 * o + k];
      if (vest) vest[3 * i + k] = vest[3 * o + k];
    }
    if (rho) rho[i] = rho[o];
    if (e) e[i] = e[o];
  }
}

/* AtomVecMeso::pack_reverse/unpack_reverse, src/USER-SPH/atom_vec_meso.cpp:387-418 */
void orc_reverse_comm(int nlocal, int nghost, const int *ghost_owner, double *f,
                      double *drho, double *de) {
  for (int g = nghost - 1; g >= 0; g--) {
    const int i = nlocal + g, o = ghost_owner[g];
    if (f) {
      f[3 * o + 0] += f[3 * i + 0];
      f[3 * o + 1] += f[3 * i + 1];
      f[3 * o + 2] += f[3 * i + 2];
    }
    if (drho) drho[o] += drho[i];
    if (de) de[o] += de[i];
  }
}

/* ------------------------------------------------------------------------------------
   Neighbor::init cutoffs, src/neighbor.cpp:251-268: cutoff = sqrt(pair->cutsq[i][j])
   where pair->cutsq = cut*cut (src/pair.cpp:221-229); cut = cutoff + skin; sq.
   ------------------------------------------------------------------------------------ */
void orc_cutneighsq(int ntypes, const double *cutmax, double skin, double *cutneighsq,
                    double *cutneighmax) {
  double cmax = 0.0;
  for (int i = 0; i <= ntypes; i++)
    for (int j = 0; j <= ntypes; j++) {
      double c = cutmax[IDX2(ntypes, i, j)];
      double cutoff = sqrt(c * c);
      double delta = cutoff > 0.0 ? skin : 0.0;
      double cut = cutoff + delta;
      cutneighsq[IDX2(ntypes, i, j)] = cut * cut;
      if (i >= 1 && j >= 1 && cut > cmax) cmax = cut;
    }
  if (cutneighmax) *cutneighmax = cmax;
}

/* ------------------------------------------------------------------------------------
   Neighbor::full_bin membership, src/neigh_full.cpp:241-344: for each owned i, every
   j != i (owned or ghost) with rsq <= cutneighsq[itype][jtype] (inclusive).  Binned
   here with cubic bins >= the largest cutoff; only the order of a row differs from
   the reference's stencil walk.
   ------------------------------------------------------------------------------------ */
long orc_neigh_full(int dim, int nlocal, int nall, const double *x, const int *type,
                    int ntypes, const double *cutneighsq, long *off, int *neigh, long cap) {
  double cmaxsq = 0.0;
  for (int i = 1; i <= ntypes; i++)
    for (int j = 1; j <= ntypes; j++)
      if (cutneighsq[IDX2(ntypes, i, j)] > cmaxsq) cmaxsq = cutneighsq[IDX2(ntypes, i, j)];
  /* bins a hair wider than the cutoff: a pair at exactly the cutoff (lattices) then never
     lands two bins apart through the rounding of (x - lo) / binsize, so the 27-bin walk
     finds every j the reference's stencil finds (neigh_full.cpp:312 keeps rsq <= cutneighsq) */
  double binsize = sqrt(cmaxsq) * (1.0 + 1e-9);
  if (binsize <= 0.0) binsize = 1.0;
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int i = 0; i < nall; i++)
    for (int k = 0; k < 3; k++) {
      if (x[3 * i + k] < lo[k]) lo[k] = x[3 * i + k];
      if (x[3 * i + k] > hi[k]) hi[k] = x[3 * i + k];
    }
  int nb[3];
  for (int k = 0; k < 3; k++) {
    nb[k] = (nall > 0) ? (int)((hi[k] - lo[k]) / binsize) + 1 : 1;
    if (nb[k] < 1) nb[k] = 1;
  }
  if (dim == 2) nb[2] = 1;
  const long nbins = (long)nb[0] * nb[1] * nb[2];
  int *head = (int *)malloc(sizeof(int) * (nbins > 0 ? nbins : 1));
  int *next = (int *)malloc(sizeof(int) * (nall > 0 ? nall : 1));
  int *bin = (int *)malloc(sizeof(int) * (nall > 0 ? nall : 1));
  for (long b = 0; b < nbins; b++) head[b] = -1;
  for (int i = nall - 1; i >= 0; i--) {
    int c[3];
    for (int k = 0; k < 3; k++) {
      c[k] = (int)((x[3 * i + k] - lo[k]) / binsize);
      if (c[k] >= nb[k]) c[k] = nb[k] - 1;
      if (c[k] < 0) c[k] = 0;
    }
    if (dim == 2) c[2] = 0;
    const int b = (c[2] * nb[1] + c[1]) * nb[0] + c[0];
    bin[i] = b;
    next[i] = head[b];
    head[b] = i;
  }
  long n = 0;
  const int dz = (dim == 2) ? 0 : 1;
  for (int i = 0; i < nlocal; i++) {
    off[i] = n;
    const int b = bin[i];
    const int cx = b % nb[0], cy = (b / nb[0]) % nb[1], cz = b / (nb[0] * nb[1]);
    const int itype = type[i];
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    for (int oz = -dz; oz <= dz; oz++) {
      const int bz = cz + oz;
      if (bz < 0 || bz >= nb[2]) continue;
      for (int oy = -1; oy <= 1; oy++) {
        const int by = cy + oy;
        if (by < 0 || by >= nb[1]) continue;
        for (int ox = -1; ox <= 1; ox++) {
          const int bx = cx + ox;
          if (bx < 0 || bx >= nb[0]) continue;
          for (int j = head[(bz * nb[1] + by) * nb[0] + bx]; j >= 0; j = next[j]) {
            if (j == i) continue;
            const int jtype = type[j];
            const double delx = xtmp - x[3 * j];
            const double dely = ytmp - x[3 * j + 1];
            const double delz = ztmp - x[3 * j + 2];
            const double rsq = delx * delx + dely * dely + delz * delz;
            if (rsq <= cutneighsq[IDX2(ntypes, itype, jtype)]) {
              if (neigh) {
                if (n >= cap) {
                  free(head);
                  free(next);
                  free(bin);
                  return -1;
                }
                neigh[n] = j;
              }
              n++;
            }
          }
        }
      }
    }
  }
  off[nlocal] = n;
  free(head);
  free(next);
  free(bin);
  return n;
}

/* Neighbor::half_from_full_newton, src/neigh_derive.cpp:83-150 */
long orc_neigh_half_from_full(int nlocal, const double *x, const long *foff,
                              const int *fneigh, long *hoff, int *hneigh) {
  long n = 0;
  for (int i = 0; i < nlocal; i++) {
    hoff[i] = n;
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    for (long jj = foff[i]; jj < foff[i + 1]; jj++) {
      const int j = fneigh[jj];
      if (j < nlocal) {
        if (i > j) continue;
      } else {
        if (x[3 * j + 2] < ztmp) continue;
        if (x[3 * j + 2] == ztmp) {
          if (x[3 * j + 1] < ytmp) continue;
          if (x[3 * j + 1] == ytmp && x[3 * j] < xtmp) continue;
        }
      }
      if (hneigh) hneigh[n] = j;
      n++;
    }
  }
  hoff[nlocal] = n;
  return n;
}

/* ------------------------------------------------------------------------------------
   PairSPHRhoSum::compute, src/USER-SPH/pair_sph_rhosum.cpp:116-195 (full list; the
   nstep gate at :112-113 and forward_comm_pair at :203 are the caller's business)
   ------------------------------------------------------------------------------------ */
void orc_rhosum(int dim, int nlocal, const double *x, const int *type, int ntypes,
                const double *mass, const double *cut, const double *cutsq,
                const long *off, const int *neigh, double *rho) {
  for (int i = 0; i < nlocal; i++) {
    const int itype = type[i];
    const double imass = mass[itype];
    const double h = cut[IDX2(ntypes, itype, itype)];
    double wf;
    if (dim == 3)
      wf = 2.1541870227086614782 / (h * h * h);
    else
      wf = 1.5915494309189533576e0 / (h * h);
    rho[i] = imass * wf;
  }
  for (int i = 0; i < nlocal; i++) {
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const int itype = type[i];
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const int jtype = type[j];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        const double ihsq = ih * ih;
        double wf;
        if (dim == 3) {
          wf = 1.0 - rsq * ihsq;
          wf = wf * wf;
          wf = wf * wf;
          wf = 2.1541870227086614782e0 * wf * ihsq * ih;
        } else {
          wf = 1.0 - rsq * ihsq;
          wf = wf * wf;
          wf = wf * wf;
          wf = 1.5915494309189533576e0 * wf * ihsq;
        }
        rho[i] += mass[jtype] * wf;
      }
    }
  }
}

/* ------------------------------------------------------------------------------------
   PairSPHTaitwater::compute, src/USER-SPH/pair_sph_taitwater.cpp:101-197 (half list,
   Newton-3 scatter onto j when newton_pair || j < nlocal).  virial (if non-NULL) is the
   pairwise ev_tally form v += del_a*del_b*fpair (src/pair.cpp:770-850).
   ------------------------------------------------------------------------------------ */
void orc_taitwater(int dim, int nlocal, int newton_pair, const double *x,
                   const double *vest, const double *rho, const int *type, int ntypes,
                   const double *mass, const double *rho0, const double *soundspeed,
                   const double *B, const double *viscosity, const double *cut,
                   const double *cutsq, const long *off, const int *neigh, double *f,
                   double *drho, double *de, double *virial) {
  const double *v = vest;
  for (int i = 0; i < nlocal; i++) {
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const double vxtmp = v[3 * i], vytmp = v[3 * i + 1], vztmp = v[3 * i + 2];
    const int itype = type[i];
    const double imass = mass[itype];
    double tmp = rho[i] / rho0[itype];
    double fi = tmp * tmp * tmp;
    fi = B[itype] * (fi * fi * tmp - 1.0) / (rho[i] * rho[i]);
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      const int jtype = type[j];
      const double jmass = mass[jtype];
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        const double ihsq = ih * ih;
        double wfd = h - sqrt(rsq);
        if (dim == 3)
          wfd = -25.066903536973515383e0 * wfd * wfd * ihsq * ihsq * ihsq * ih;
        else
          wfd = -19.098593171027440292e0 * wfd * wfd * ihsq * ihsq * ihsq;
        tmp = rho[j] / rho0[jtype];
        double fj = tmp * tmp * tmp;
        fj = B[jtype] * (fj * fj * tmp - 1.0) / (rho[j] * rho[j]);
        const double delVdotDelR = delx * (vxtmp - v[3 * j]) + dely * (vytmp - v[3 * j + 1]) +
                                   delz * (vztmp - v[3 * j + 2]);
        double fvisc;
        if (delVdotDelR < 0.) {
          const double mu = h * delVdotDelR / (rsq + 0.01 * h * h);
          fvisc = -viscosity[IDX2(ntypes, itype, jtype)] *
                  (soundspeed[itype] + soundspeed[jtype]) * mu / (rho[i] + rho[j]);
        } else {
          fvisc = 0.;
        }
        const double fpair = -imass * jmass * (fi + fj + fvisc) * wfd;
        const double deltaE = -0.5 * fpair * delVdotDelR;
        f[3 * i + 0] += delx * fpair;
        f[3 * i + 1] += dely * fpair;
        f[3 * i + 2] += delz * fpair;
        drho[i] += jmass * delVdotDelR * wfd;
        de[i] += deltaE;
        if (newton_pair || j < nlocal) {
          f[3 * j + 0] -= delx * fpair;
          f[3 * j + 1] -= dely * fpair;
          f[3 * j + 2] -= delz * fpair;
          de[j] += deltaE;
          drho[j] += imass * delVdotDelR * wfd;
        }
        if (virial) {
          const double s = (newton_pair || j < nlocal) ? 1.0 : 0.5;
          virial[0] += s * delx * delx * fpair;
          virial[1] += s * dely * dely * fpair;
          virial[2] += s * delz * delz * fpair;
          virial[3] += s * delx * dely * fpair;
          virial[4] += s * delx * delz * fpair;
          virial[5] += s * dely * delz * fpair;
        }
      }
    }
  }
}

/* PairSPHTaitwaterMorris::compute, src/USER-SPH/pair_sph_taitwater_morris.cpp:100-197 */
void orc_taitwater_morris(int dim, int nlocal, int newton_pair, const double *x,
                          const double *vest, const double *rho, const int *type,
                          int ntypes, const double *mass, const double *rho0,
                          const double *soundspeed, const double *B,
                          const double *viscosity, const double *cut, const double *cutsq,
                          const long *off, const int *neigh, double *f, double *drho,
                          double *de, double *virial) {
  (void)soundspeed;
  const double *v = vest;
  for (int i = 0; i < nlocal; i++) {
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const double vxtmp = v[3 * i], vytmp = v[3 * i + 1], vztmp = v[3 * i + 2];
    const int itype = type[i];
    const double imass = mass[itype];
    double tmp = rho[i] / rho0[itype];
    double fi = tmp * tmp * tmp;
    fi = B[itype] * (fi * fi * tmp - 1.0) / (rho[i] * rho[i]);
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      const int jtype = type[j];
      const double jmass = mass[jtype];
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        const double ihsq = ih * ih;
        double wfd = h - sqrt(rsq);
        if (dim == 3)
          wfd = -25.066903536973515383e0 * wfd * wfd * ihsq * ihsq * ihsq * ih;
        else
          wfd = -19.098593171027440292e0 * wfd * wfd * ihsq * ihsq * ihsq;
        tmp = rho[j] / rho0[jtype];
        double fj = tmp * tmp * tmp;
        fj = B[jtype] * (fj * fj * tmp - 1.0) / (rho[j] * rho[j]);
        const double velx = vxtmp - v[3 * j];
        const double vely = vytmp - v[3 * j + 1];
        const double velz = vztmp - v[3 * j + 2];
        const double delVdotDelR = delx * velx + dely * vely + delz * velz;
        double fvisc = 2 * viscosity[IDX2(ntypes, itype, jtype)] / (rho[i] * rho[j]);
        fvisc *= imass * jmass * wfd;
        const double fpair = -imass * jmass * (fi + fj) * wfd;
        const double deltaE =
            -0.5 * (fpair * delVdotDelR + fvisc * (velx * velx + vely * vely + velz * velz));
        f[3 * i + 0] += delx * fpair + velx * fvisc;
        f[3 * i + 1] += dely * fpair + vely * fvisc;
        f[3 * i + 2] += delz * fpair + velz * fvisc;
        drho[i] += jmass * delVdotDelR * wfd;
        de[i] += deltaE;
        if (newton_pair || j < nlocal) {
          f[3 * j + 0] -= delx * fpair + velx * fvisc;
          f[3 * j + 1] -= dely * fpair + vely * fvisc;
          f[3 * j + 2] -= delz * fpair + velz * fvisc;
          de[j] += deltaE;
          drho[j] += imass * delVdotDelR * wfd;
        }
        if (virial) {
          const double s = (newton_pair || j < nlocal) ? 1.0 : 0.5;
          virial[0] += s * delx * delx * fpair;
          virial[1] += s * dely * dely * fpair;
          virial[2] += s * delz * delz * fpair;
          virial[3] += s * delx * dely * fpair;
          virial[4] += s * delx * delz * fpair;
          virial[5] += s * dely * delz * fpair;
        }
      }
    }
  }
}

/* PairSPHHeatConduction::compute, src/USER-SPH/pair_sph_heatconduction.cpp:76-131 */
void orc_heatconduction(int dim, int nlocal, int newton_pair, const double *x,
                        const double *e, const double *rho, const int *type, int ntypes,
                        const double *mass, const double *alpha, const double *cut,
                        const double *cutsq, const long *off, const int *neigh,
                        double *de) {
  for (int i = 0; i < nlocal; i++) {
    const int itype = type[i];
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const double imass = mass[itype];
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      const int jtype = type[j];
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        const double ihsq = ih * ih;
        double wfd = h - sqrt(rsq);
        if (dim == 3)
          wfd = -25.066903536973515383e0 * wfd * wfd * ihsq * ihsq * ihsq * ih;
        else
          wfd = -19.098593171027440292e0 * wfd * wfd * ihsq * ihsq * ihsq;
        const double jmass = mass[jtype];
        const double D = alpha[IDX2(ntypes, itype, jtype)];
        double deltaE = 2.0 * imass * jmass / (imass + jmass);
        deltaE *= (rho[i] + rho[j]) / (rho[i] * rho[j]);
        deltaE *= D * (e[i] - e[j]) * wfd;
        de[i] += deltaE;
        if (newton_pair || j < nlocal) de[j] -= deltaE;
      }
    }
  }
}

/* ------------------------------------------------------------------------------------
   Quintic spline, src/USER-SPH/sph_kernel_quintic.cpp:17-73 (pow() semantics kept)
   ------------------------------------------------------------------------------------ */
/* qpow: the reference's pow(x, n) (glibc), or for test aids only (orc_set_pow_mode):
   1 = the correctly rounded power (double-double products, one rounding: what the engine
   evaluates, sph_mp_kernels.h qr_pow*; glibc's pow differs from it by 1 ulp in ~0.09 % of the
   calls, tools/quintic_pow_check.c), 2 = glibc's result moved one ulp up (how far the
   reference's own result moves under a last-bit change of its libm's pow -- the tests'
   spread shadow, pyoracle _Spread).  0 (default) is the reference. */
static int g_pow_mode = 0;
void orc_set_pow_mode(int m) { g_pow_mode = m; }
static double cr_pow(double x, int n) {
  const double h = x * x, l = fma(x, x, -h);
  if (n == 2) return h;
  if (n == 3) {
    const double p = x * h, e = fma(x, h, -p);
    return p + fma(x, l, e);
  }
  const double q = h * h, t = fma(2.0 * h, l, fma(h, h, -q));
  if (n == 4) return q + t;
  const double p = x * q, e = fma(x, q, -p);
  return p + fma(x, t, e);
}
static double qpow(double x, int n) {
  if (g_pow_mode == 1) return cr_pow(x, n);
  const double y = pow(x, n);
  if (g_pow_mode == 2 && n > 2 && y > 0.0) return nextafter(y, INFINITY);
  return y;
}

double orc_kernel_quintic3d(double r) {
  const double norm3d = 0.0716197243913529;
  const double s = 3.0 * r;
  if (s < 1.0) return norm3d * (qpow(3 - s, 5) - 6 * qpow(2 - s, 5) + 15 * qpow(1 - s, 5));
  if (s < 2.0) return norm3d * (qpow(3 - s, 5) - 6 * qpow(2 - s, 5));
  if (s < 3.0) return norm3d * qpow(3 - s, 5);
  return 0.0;
}

double orc_kernel_quintic2d(double r) {
  const double norm2d = 0.04195297663091802;
  const double s = 3.0 * r;
  if (s < 1.0) return norm2d * (qpow(3 - s, 5) - 6 * qpow(2 - s, 5) + 15 * qpow(1 - s, 5));
  if (s < 2.0) return norm2d * (qpow(3 - s, 5) - 6 * qpow(2 - s, 5));
  if (s < 3.0) return norm2d * qpow(3 - s, 5);
  return 0.0;
}

/* Test aid (never the reference's arithmetic): orc_set_quintic_factored(1) evaluates dW/ds
   in the factored form -5 (3-s)^4 + 30 (2-s)^4 - 75 (1-s)^4, which is the same polynomial
   without the expanded form's cancellation near the pieces' ends (s -> 3: terms ~400 summing
   to ~1e-4); tools/cg_probe.py compares the forms. */
static int g_quintic_factored = 0;
void orc_set_quintic_factored(int on) { g_quintic_factored = on; }

static double dw_quintic_poly(double s) {
  if (g_quintic_factored) {
    const double a = s < 3.0 ? 3.0 - s : 0.0, b = s < 2.0 ? 2.0 - s : 0.0,
                 c = s < 1.0 ? 1.0 - s : 0.0;
    return -5 * (a * a) * (a * a) + 30 * (b * b) * (b * b) - 75 * (c * c) * (c * c);
  }
  if (s < 1) return -50 * qpow(s, 4) + 120 * qpow(s, 3) - 120 * s;
  if (s < 2) return 25 * qpow(s, 4) - 180 * qpow(s, 3) + 450 * qpow(s, 2) - 420 * s + 75;
  if (s < 3.0) return -5 * qpow(s, 4) + 60 * qpow(s, 3) - 270 * qpow(s, 2) + 540 * s - 405;
  return 0.0;
}

double orc_dw_quintic3d(double r) { return 3.0 * 0.0716197243913529 * dw_quintic_poly(3.0 * r); }
double orc_dw_quintic2d(double r) { return 3.0 * 0.04195297663091802 * dw_quintic_poly(3.0 * r); }

/* PairSPHRhoSumMultiphase::compute, src/USER-SPH/pair_sph_rhosum_multiphase.cpp:112-167 */
void orc_rhosum_multiphase(int dim, int nlocal, const double *x, const int *type,
                           int ntypes, const double *rmass, const double *cut,
                           const double *cutsq, const long *off, const int *neigh,
                           double *rho) {
  for (int i = 0; i < nlocal; i++) {
    const int itype = type[i];
    const double h = cut[IDX2(ntypes, itype, itype)];
    rho[i] = (dim == 3) ? orc_kernel_quintic3d(0.0) / (h * h * h)
                        : orc_kernel_quintic2d(0.0) / (h * h);
  }
  for (int i = 0; i < nlocal; i++) {
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const int itype = type[i];
    const double imass = rmass[i];
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const int jtype = type[j];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        double wf;
        if (dim == 3) {
          const double r = sqrt(rsq) * ih;
          wf = orc_kernel_quintic3d(r) * ih * ih * ih;
        } else {
          const double r = sqrt(rsq) * ih;
          wf = orc_kernel_quintic2d(r) * ih * ih;
        }
        rho[i] += wf;
      }
    }
    rho[i] *= imass;
  }
}

/* sph_pressure, src/USER-SPH/pair_sph_taitwater_multiphase.cpp:289-292 */
static double sph_pressure(double B, double rho0, double gamma, double rbackground,
                           double rho) {
  return B * (pow(rho / rho0, gamma) - rbackground);
}

/* PairSPHTaitwaterMultiphase::compute, src/USER-SPH/pair_sph_taitwater_multiphase.cpp:
   95-183.  Reference quirk kept: p_j uses gamma[itype] (:148). */
void orc_taitwater_multiphase(int dim, int nlocal, int newton_pair, const double *x,
                              const double *vest, const double *rho, const int *type,
                              int ntypes, const double *rmass, const double *rho0,
                              const double *soundspeed, const double *B,
                              const double *gamma, const double *rbackground,
                              const double *viscosity, const double *cut,
                              const double *cutsq, const long *off, const int *neigh,
                              double *f) {
  (void)soundspeed;
  const double *v = vest;
  for (int i = 0; i < nlocal; i++) {
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const double vxtmp = v[3 * i], vytmp = v[3 * i + 1], vztmp = v[3 * i + 2];
    const int itype = type[i];
    const double imass = rmass[i];
    const double pi = sph_pressure(B[itype], rho0[itype], gamma[itype], rbackground[itype],
                                   rho[i]);
    const double Vi = imass / rho[i];
    const double Vi2 = Vi * Vi;
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      const int jtype = type[j];
      const double jmass = rmass[j];
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        double wfd;
        if (dim == 3) {
          wfd = orc_dw_quintic3d(sqrt(rsq) * ih);
          wfd = wfd * ih * ih * ih * ih / sqrt(rsq);
        } else {
          wfd = orc_dw_quintic2d(sqrt(rsq) * ih);
          wfd = wfd * ih * ih * ih / sqrt(rsq);
        }
        const double Vj = jmass / rho[j];
        const double Vj2 = Vj * Vj;
        const double pj = sph_pressure(B[jtype], rho0[jtype], gamma[itype],
                                       rbackground[jtype], rho[j]);
        const double pij_wave = (rho[j] * pi + rho[i] * pj) / (rho[i] + rho[j]);
        const double velx = vxtmp - v[3 * j];
        const double vely = vytmp - v[3 * j + 1];
        const double velz = vztmp - v[3 * j + 2];
        const double fvisc = (Vi2 + Vj2) * viscosity[IDX2(ntypes, itype, jtype)] * wfd;
        const double fpair = -(Vi2 + Vj2) * pij_wave * wfd;
        f[3 * i + 0] += delx * fpair + velx * fvisc;
        f[3 * i + 1] += dely * fpair + vely * fvisc;
        f[3 * i + 2] += delz * fpair + velz * fvisc;
        if (newton_pair || j < nlocal) {
          f[3 * j + 0] -= delx * fpair + velx * fvisc;
          f[3 * j + 1] -= dely * fpair + vely * fvisc;
          f[3 * j + 2] -= delz * fpair + velz * fvisc;
        }
      }
    }
  }
}

/* PairSPHHeatConductionPhaseChange::compute,
   src/USER-SPH/pair_sph_heatconduction_phasechange.cpp:81-138.  fixflag/tc are taken
   as given (callers pass 0 where coeff() had 4 args: reference quirk A.6-4). */
void orc_heatconduction_phasechange(int dim, int nlocal, int newton_pair, const double *x,
                                    const double *e, const double *cv, const double *rho,
                                    const double *rmass, const int *type, int ntypes,
                                    const double *alpha, const int *fixflag,
                                    const double *tc, const double *cut,
                                    const double *cutsq, const long *off,
                                    const int *neigh, double *de) {
  for (int i = 0; i < nlocal; i++) {
    const int itype = type[i];
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const double imass = rmass[i];
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      const int jtype = type[j];
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        double wfd;
        if (dim == 3) {
          wfd = orc_dw_quintic3d(sqrt(rsq) * ih);
          wfd = wfd * ih * ih * ih * ih / sqrt(rsq);
        } else {
          wfd = orc_dw_quintic2d(sqrt(rsq) * ih);
          wfd = wfd * ih * ih * ih / sqrt(rsq);
        }
        const double jmass = rmass[j];
        const double D = alpha[IDX2(ntypes, itype, jtype)];
        double Ti = e[i] / cv[i];
        double Tj = e[j] / cv[j];
        const int ff = fixflag ? fixflag[IDX2(ntypes, itype, jtype)] : 0;
        if ((ff == itype) && (Ti < Tj)) Ti = tc[IDX2(ntypes, itype, jtype)];
        if ((ff == jtype) && (Tj < Ti)) Tj = tc[IDX2(ntypes, itype, jtype)];
        const double deltaE = 2.0 * D * (Ti - Tj) * wfd / (rho[i] * rho[j]);
        de[i] += deltaE * jmass;
        if (newton_pair || j < nlocal) de[j] -= deltaE * imass;
      }
    }
  }
}

/* PairSPHColorGradient::compute, src/USER-SPH/pair_sph_colorgradient.cpp:118-187 */
void orc_colorgradient(int dim, int nlocal, const double *x, const double *rho,
                       const double *rmass, const int *type, int ntypes,
                       const double *alpha, const double *cut, const double *cutsq,
                       const long *off, const int *neigh, double *cg) {
  for (int i = 0; i < nlocal; i++) cg[3 * i] = cg[3 * i + 1] = cg[3 * i + 2] = 0.0;
  for (int i = 0; i < nlocal; i++) {
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const int itype = type[i];
    const double sigmai = rho[i] / rmass[i];
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const int jtype = type[j];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double r = sqrt(rsq);
        const double e0 = delx / r, e1 = dely / r, e2 = delz / r;
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        double wfd;
        if (dim == 3) {
          wfd = orc_dw_quintic3d(r * ih);
          wfd = wfd * ih * ih * ih * ih;
        } else {
          wfd = orc_dw_quintic2d(r * ih);
          wfd = wfd * ih * ih * ih;
        }
        const double sigmaj = rho[j] / rmass[j];
        const double sigmaj2 = sigmaj * sigmaj;
        const double dphi = -wfd * alpha[IDX2(ntypes, itype, jtype)] / sigmaj2 * sigmai;
        cg[3 * i + 0] += dphi * e0;
        cg[3 * i + 1] += dphi * e1;
        if (dim == 3) cg[3 * i + 2] += dphi * e2;
      }
    }
  }
}

/* PairSPHSurfaceTension::compute, src/USER-SPH/pair_sph_surfacetension.cpp:50-192.
   S = (|c|^2/ndim I - c c^T) e / |c| for c = the atom's colorgradient (zero when
   |c| <= EPSILON = 1e-12, :29), F = (S_i V_i^2 + S_j V_j^2) dW, V = rmass/rho; the
   reference's expressions and operation order are kept term by term.  cg is nall*3. */
static void st_vector(int dim, const double *c, double absc, const double *e, double *S) {
  S[0] = S[1] = S[2] = 0.0;
  if (!(absc > 1.0e-12)) return;
  if (dim == 2) {
    S[0] = (e[0] * ((c[1] * c[1] + c[0] * c[0]) / 2 - c[0] * c[0]) - c[0] * e[1] * c[1]) / absc;
    S[1] = (e[1] * ((c[1] * c[1] + c[0] * c[0]) / 2 - c[1] * c[1]) - e[0] * c[0] * c[1]) / absc;
  } else {
    S[0] = (e[0] * (0.3333333333333333 * c[2] * c[2] + 0.3333333333333333 * c[1] * c[1] -
                    0.6666666666666666 * c[0] * c[0]) -
            1.0 * c[0] * e[2] * c[2] - 1.0 * c[0] * e[1] * c[1]) / absc;
    S[1] = (e[1] * (0.3333333333333333 * c[2] * c[2] - 0.6666666666666666 * c[1] * c[1] +
                    0.3333333333333333 * c[0] * c[0]) -
            1.0 * c[1] * e[2] * c[2] - 1.0 * e[0] * c[0] * c[1]) / absc;
    S[2] = (e[2] * (-0.6666666666666666 * c[2] * c[2] + 0.3333333333333333 * c[1] * c[1] +
                    0.3333333333333333 * c[0] * c[0]) -
            1.0 * e[1] * c[1] * c[2] - 1.0 * e[0] * c[0] * c[2]) / absc;
  }
}
static double st_abs(int dim, const double *c) {
  return dim == 3 ? sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2])
                  : sqrt(c[0] * c[0] + c[1] * c[1]);
}
void orc_surfacetension(int dim, int nlocal, int newton_pair, const double *x,
                        const double *rho, const double *rmass, const int *type, int ntypes,
                        const double *cg, const double *cut, const double *cutsq,
                        const long *off, const int *neigh, double *f) {
  for (int i = 0; i < nlocal; i++) {
    const int itype = type[i];
    const double xtmp = x[3 * i], ytmp = x[3 * i + 1], ztmp = x[3 * i + 2];
    const double imass = rmass[i];
    const double abscgi = st_abs(dim, cg + 3 * i);
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      const double delx = xtmp - x[3 * j];
      const double dely = ytmp - x[3 * j + 1];
      const double delz = ztmp - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      const int jtype = type[j];
      const double jmass = rmass[j];
      if (rsq < cutsq[IDX2(ntypes, itype, jtype)]) {
        const double h = cut[IDX2(ntypes, itype, jtype)];
        const double ih = 1.0 / h;
        double wfd;
        if (dim == 3) {
          wfd = orc_dw_quintic3d(sqrt(rsq) * ih);
          wfd = wfd * ih * ih * ih * ih;
        } else {
          wfd = orc_dw_quintic2d(sqrt(rsq) * ih);
          wfd = wfd * ih * ih * ih;
        }
        double eij[3] = {delx / sqrt(rsq), dely / sqrt(rsq), 0.0};
        if (dim == 3) eij[2] = delz / sqrt(rsq);
        double Si[3], Sj[3];
        st_vector(dim, cg + 3 * i, abscgi, eij, Si);
        st_vector(dim, cg + 3 * j, st_abs(dim, cg + 3 * j), eij, Sj);
        const double Vi = imass / rho[i];
        const double Vj = jmass / rho[j];
        for (int k = 0; k < dim; k++) {
          const double fk = (Si[k] * Vi * Vi + Sj[k] * Vj * Vj) * wfd;
          f[3 * i + k] += fk;
          if (newton_pair || j < nlocal) f[3 * j + k] -= fk;
        }
      }
    }
  }
}

/* ------------------------------------------------------------------------------------
   FixMeso, src/USER-SPH/fix_meso.cpp:68-85 (setup_pre_force), :91-140, :144-180
   ------------------------------------------------------------------------------------ */
void orc_meso_setup(int nlocal, const double *v, double *vest) {
  memcpy(vest, v, sizeof(double) * 3 * (size_t)nlocal);
}

static int in_group(const int *type, int tmask, int i) {
  return tmask == 0 || ((tmask >> type[i]) & 1);
}

/* FixMeso::setup_pre_force (fix_meso.cpp:68-85): vest = v for the group's atoms */
void orc_meso_setup_g(int nlocal, const int *type, int tmask, const double *v, double *vest) {
  for (int i = 0; i < nlocal; i++)
    if (in_group(type, tmask, i))
      for (int k = 0; k < 3; k++) vest[3 * i + k] = v[3 * i + k];
}

/* FixMeso::initial_integrate (fix_meso.cpp:91-140) over the group's atoms */
void orc_meso_initial_g(int nlocal, double dtv, double dtf, const int *type, int tmask,
                        const double *mass, const double *rmass, double *x, double *v,
                        const double *f, double *vest, double *rho, const double *drho,
                        double *e, const double *de) {
  for (int i = 0; i < nlocal; i++) {
    if (!in_group(type, tmask, i)) continue;
    const double dtfm = rmass ? dtf / rmass[i] : dtf / mass[type[i]];
    e[i] += dtf * de[i];
    rho[i] += dtf * drho[i];
    for (int k = 0; k < 3; k++) {
      vest[3 * i + k] = v[3 * i + k] + 2.0 * dtfm * f[3 * i + k];
      v[3 * i + k] += dtfm * f[3 * i + k];
      x[3 * i + k] += dtv * v[3 * i + k];
    }
  }
}

/* FixMeso::final_integrate (fix_meso.cpp:144-180) over the group's atoms */
void orc_meso_final_g(int nlocal, double dtf, const int *type, int tmask, const double *mass,
                      const double *rmass, double *v, const double *f, double *rho,
                      const double *drho, double *e, const double *de) {
  for (int i = 0; i < nlocal; i++) {
    if (!in_group(type, tmask, i)) continue;
    const double dtfm = rmass ? dtf / rmass[i] : dtf / mass[type[i]];
    for (int k = 0; k < 3; k++) v[3 * i + k] += dtfm * f[3 * i + k];
    e[i] += dtf * de[i];
    rho[i] += dtf * drho[i];
  }
}

/* FixMesoStationary::initial_integrate / final_integrate (fix_meso_stationary.cpp:71-112):
   the group's atoms integrate only e and rho; x, v and vest stay */
void orc_meso_stationary(int nlocal, double dtf, const int *type, int tmask, double *rho,
                         const double *drho, double *e, const double *de) {
  for (int i = 0; i < nlocal; i++) {
    if (!in_group(type, tmask, i)) continue;
    e[i] += dtf * de[i];
    rho[i] += dtf * drho[i];
  }
}

/* FixGravity::post_force (fix_gravity.cpp:244-295), style vector: acc = magnitude * unit
   direction (set_acceleration, :320-336); f += massone * acc for the group's owned atoms */
void orc_gravity(int nlocal, const int *type, int tmask, const double *mass,
                 const double *rmass, const double *acc, double *f) {
  for (int i = 0; i < nlocal; i++) {
    if (!in_group(type, tmask, i)) continue;
    const double m = rmass ? rmass[i] : mass[type[i]];
    for (int k = 0; k < 3; k++) f[3 * i + k] += m * acc[k];
  }
}

void orc_meso_initial(int nlocal, double dtv, double dtf, const int *type,
                      const double *mass, const double *rmass, double *x, double *v,
                      const double *f, double *vest, double *rho, const double *drho,
                      double *e, const double *de) {
  for (int i = 0; i < nlocal; i++) {
    const double dtfm = rmass ? dtf / rmass[i] : dtf / mass[type[i]];
    e[i] += dtf * de[i];
    rho[i] += dtf * drho[i];
    vest[3 * i + 0] = v[3 * i + 0] + 2.0 * dtfm * f[3 * i + 0];
    vest[3 * i + 1] = v[3 * i + 1] + 2.0 * dtfm * f[3 * i + 1];
    vest[3 * i + 2] = v[3 * i + 2] + 2.0 * dtfm * f[3 * i + 2];
    v[3 * i + 0] += dtfm * f[3 * i + 0];
    v[3 * i + 1] += dtfm * f[3 * i + 1];
    v[3 * i + 2] += dtfm * f[3 * i + 2];
    x[3 * i + 0] += dtv * v[3 * i + 0];
    x[3 * i + 1] += dtv * v[3 * i + 1];
    x[3 * i + 2] += dtv * v[3 * i + 2];
  }
}

void orc_meso_final(int nlocal, double dtf, const int *type, const double *mass,
                    const double *rmass, double *v, const double *f, double *rho,
                    const double *drho, double *e, const double *de) {
  for (int i = 0; i < nlocal; i++) {
    const double dtfm = rmass ? dtf / rmass[i] : dtf / mass[type[i]];
    v[3 * i + 0] += dtfm * f[3 * i + 0];
    v[3 * i + 1] += dtfm * f[3 * i + 1];
    v[3 * i + 2] += dtfm * f[3 * i + 2];
    e[i] += dtf * de[i];
    rho[i] += dtf * drho[i];
  }
}

/* ------------------------------------------------------------------------------------
   FixPhaseChange, src/USER-SPH/fix_phase_change.cpp
   ------------------------------------------------------------------------------------ */
/* RanPark::uniform, src/random_park.cpp:42-49 */
double orc_park_uniform(int *seed) {
  const int IA = 16807, IM = 2147483647, IQ = 127773, IR = 2836;
  const double AM = 1.0 / IM;
  int k = *seed / IQ;
  *seed = IA * (*seed - k * IQ) - IR * k;
  if (*seed < 0) *seed += IM;
  return AM * *seed;
}

/* isfromphasearound, fix_phase_change.cpp:538-563 */
static int pc_around(const orc_pc_params *p, int i, const double *x, const int *type,
                     const long *off, const int *neigh) {
  const double cutoff2 = p->cutoff * p->cutoff;
  for (long jj = off[i]; jj < off[i + 1]; jj++) {
    const int j = neigh[jj];
    if (type[j] == p->from_type) {
      const double delx = x[3 * i] - x[3 * j];
      const double dely = x[3 * i + 1] - x[3 * j + 1];
      const double delz = x[3 * i + 2] - x[3 * j + 2];
      const double rsq = delx * delx + dely * dely + delz * delz;
      if (rsq <= cutoff2) return 1;
    }
  }
  return 0;
}

/* insert_one_atom's ownership test, fix_phase_change.cpp:425-456 (orthogonal box) */
static int pc_mine(const orc_pc_params *p, const double *c) {
  if (c[0] >= p->sublo[0] && c[0] < p->subhi[0] && c[1] >= p->sublo[1] &&
      c[1] < p->subhi[1] && c[2] >= p->sublo[2] && c[2] < p->subhi[2])
    return 1;
  if (p->dim == 3 && c[2] >= p->boxhi[2] && p->top[2] && c[0] >= p->sublo[0] &&
      c[0] < p->subhi[0] && c[1] >= p->sublo[1] && c[1] < p->subhi[1])
    return 1;
  if (p->dim == 2 && c[1] >= p->boxhi[1] && p->top[1] && c[0] >= p->sublo[0] &&
      c[0] < p->subhi[0])
    return 1;
  return 0;
}

/* create_newpos_simple / create_newpos, fix_phase_change.cpp:466-520 */
static void pc_newpos_simple(int *seed, const double *xone, double delta, double *coord) {
  coord[0] = xone[0] + (orc_park_uniform(seed) - 0.5) * delta;
  coord[1] = xone[1] + (orc_park_uniform(seed) - 0.5) * delta;
  coord[2] = xone[2] + (orc_park_uniform(seed) - 0.5) * delta;
}

static void pc_newpos(int dim, int *seed, const double *xone, const double *cg, double delta,
                      double *coord) {
  const double CG_SMALL = 1.0e-20;
  double eij[3];
  if (dim == 3) {
    double b1[3] = {-cg[1], cg[0], 0};
    const double b1abs = sqrt(b1[0] * b1[0] + b1[1] * b1[1] + b1[2] * b1[2]);
    if (b1abs > CG_SMALL) {
      b1[0] = b1[0] / b1abs;
      b1[1] = b1[1] / b1abs;
      b1[2] = b1[2] / b1abs;
    }
    double b2[3];
    b2[0] = -cg[0] * cg[1] * cg[2] / (pow(cg[1], 2) + pow(cg[0], 2));
    b2[1] = -cg[2] * pow(cg[1], 2) / (pow(cg[1], 2) + pow(cg[0], 2));
    b2[2] = cg[1];
    const double b2abs = sqrt(b2[0] * b2[0] + b2[1] * b2[1] + b2[2] * b2[2]);
    if (b1abs > CG_SMALL) { /* the reference tests b1abs here (:494) */
      b2[0] = b2[0] / b2abs;
      b2[1] = b2[1] / b2abs;
      b2[2] = b2[2] / b2abs;
    }
    const double atmp = orc_park_uniform(seed) - 0.5;
    const double btmp = orc_park_uniform(seed) - 0.5;
    eij[0] = atmp * b1[0] + btmp * b2[0];
    eij[1] = atmp * b1[1] + btmp * b2[1];
    eij[2] = atmp * b1[2] + btmp * b2[2];
  } else {
    double atmp = orc_park_uniform(seed);
    if (atmp > 0.5) atmp = 1;
    else atmp = -1;
    eij[0] = -atmp * cg[1];
    eij[1] = atmp * cg[0];
    eij[2] = 0.0;
  }
  const double eijabs = sqrt(eij[0] * eij[0] + eij[1] * eij[1] + eij[2] * eij[2]);
  coord[0] = xone[0] + eij[0] * delta / eijabs;
  coord[1] = xone[1] + eij[1] * delta / eijabs;
  coord[2] = xone[2] + eij[2] * delta / eijabs;
}

/* FixPhaseChange::pre_exchange, fix_phase_change.cpp:167-321 (up to reverse comm) */
int orc_phasechange(const orc_pc_params *p, int *seed, int nlocal, int nall, const double *x,
                    const double *v, const double *vest, const double *cg, double *e,
                    const double *rmass, const double *rho, const double *cv,
                    const int *type, const long *off, const int *neigh, double *dmass,
                    int cap, double *new_atoms, int *parent) {
  int nins = 0;
  for (int i = 0; i < nall; i++) dmass[i] = 0.0;
  for (int i = 0; i < nlocal; i++) {
    const double Ti = e[i] / cv[i];
    int isphasechange;
    if ((Ti < p->Tc) || (type[i] != p->to_type)) {
      isphasechange = 0;
    } else if (p->energy_chance) {
      const double threshold = (e[i] - p->Tc * cv[i]) / p->Hwv * p->dt * p->rate;
      isphasechange = (orc_park_uniform(seed) < threshold) && pc_around(p, i, x, type, off, neigh);
    } else {
      isphasechange = (orc_park_uniform(seed) < p->change_chance) && (Ti > p->Tt) &&
                      pc_around(p, i, x, type, off, neigh);
    }
    if (!isphasechange) continue;
    double coord[3];
    int ok = 0, natempt = 0;
    double delta = p->dr;
    do {
      pc_newpos(p->dim, seed, x + 3 * i, cg + 3 * i, delta, coord);
      ok = pc_mine(p, coord);
      delta = 0.75 * delta;
      natempt++;
    } while (!ok && natempt < p->maxattempt);
    if (!ok) {
      delta = p->dr;
      natempt = 0;
      do {
        pc_newpos_simple(seed, x + 3 * i, delta, coord);
        ok = pc_mine(p, coord);
        delta = 0.75 * delta;
        natempt++;
      } while (!ok && natempt < p->maxattempt);
    }
    if (!ok) continue;
    /* weights over from_type neighbours heavier than half a new particle (:236-256) */
    double wtotal = 0.0;
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      if (type[j] == p->from_type && rmass[j] > 0.5 * p->to_mass) {
        const double delx = x[3 * i] - x[3 * j];
        const double dely = x[3 * i + 1] - x[3 * j + 1];
        const double delz = x[3 * i + 2] - x[3 * j + 2];
        const double rsq = delx * delx + dely * dely + delz * delz;
        wtotal += (p->dim == 3) ? orc_kernel_quintic3d(sqrt(rsq) * p->cutoff)
                                : orc_kernel_quintic2d(sqrt(rsq) * p->cutoff);
      }
    }
    double dmom[3] = {0, 0, 0}, dmomest[3] = {0, 0, 0};
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      if (type[j] == p->from_type && rmass[j] > 0.5 * p->to_mass) {
        const double delx = x[3 * i] - x[3 * j];
        const double dely = x[3 * i + 1] - x[3 * j + 1];
        const double delz = x[3 * i + 2] - x[3 * j + 2];
        const double rsq = delx * delx + dely * dely + delz * delz;
        const double wfd = (p->dim == 3) ? orc_kernel_quintic3d(sqrt(rsq) * p->cutoff)
                                         : orc_kernel_quintic2d(sqrt(rsq) * p->cutoff);
        const double dmass_aux = p->to_mass * wfd / wtotal;
        dmass[j] += dmass_aux;
        dmom[0] += v[3 * j] * dmass_aux;
        dmom[1] += v[3 * j + 1] * dmass_aux;
        dmom[2] += v[3 * j + 2] * dmass_aux;
        dmomest[0] += vest[3 * j] * dmass_aux;
        dmomest[1] += vest[3 * j + 1] * dmass_aux;
        dmomest[2] += vest[3 * j + 2] * dmass_aux;
      }
    }
    const double energy_aux = 0.5 * (e[i] - p->Hwv);
    if (nins < cap) {
      double *r = new_atoms + 13 * (size_t)nins;
      r[0] = coord[0];
      r[1] = coord[1];
      r[2] = coord[2];
      r[3] = dmom[0] / p->to_mass;
      r[4] = dmom[1] / p->to_mass;
      r[5] = dmom[2] / p->to_mass;
      r[6] = dmomest[0] / p->to_mass;
      r[7] = dmomest[1] / p->to_mass;
      r[8] = dmomest[2] / p->to_mass;
      r[9] = energy_aux;
      r[10] = p->to_mass;
      r[11] = rho[i];
      r[12] = cv[i];
      parent[nins] = i;
    }
    e[i] = energy_aux;
    nins++;
  }
  return nins;
}

void orc_phasechange_finish(int nlocal, const double *dmass, double *rmass, double *e) {
  for (int i = 0; i < nlocal; i++) {
    const double mold = rmass[i];
    rmass[i] -= dmass[i];
    e[i] = e[i] * mold / rmass[i];
  }
}

/* FixPhaseChange::pre_exchange, fix_phase_change.cpp:167-352, restated WITH the reference's
   memory behaviour on one process (the port's orc_phasechange above evaluates every
   candidate on the atoms as found instead).  The arrays have room for nmax atoms: owned
   [0, nlocal), ghosts [nlocal, nlocal+nghost).  The k-th atom created by this call goes to
   index nlocal + k through AtomVecMesoMultiPhase::create_atom
   (atom_vec_meso_multiphase.cpp:968-997) -- over a ghost slot that later candidates' full
   lists may still name, and with drho (= the fix's dmass, :193) of that slot zeroed.  Then
   the ghosts' dmass goes back along CommBrick's swaps (reverse_comm_fix), the donors lose
   mass and have their energy renormalised (:325-332).  dmass is scratch of nmax.  Returns
   the new nlocal (owned + created), or -1 when nmax is too small for the created atoms
   (the reference would grow the arrays there). */
int orc_pre_exchange_ref(const orc_pc_params *p, int *seed, int nlocal, int nghost, int nmax,
                         double *x, double *v, double *vest, double *cg, double *e,
                         double *rmass, double *rho, double *cv, int *type, const long *off,
                         const int *neigh, int nswap, const int *swap_first,
                         const int *ghost_src, double *dmass) {
  const int nall = nlocal + nghost;
  int ncur = nlocal;
  for (int i = 0; i < nall; i++) dmass[i] = 0.0;   /* force->newton on (:196-201) */
  for (int i = 0; i < nlocal; i++) {
    const double Ti = e[i] / cv[i];
    int isphasechange;
    if ((Ti < p->Tc) || (type[i] != p->to_type)) {
      isphasechange = 0;
    } else if (p->energy_chance) {
      const double threshold = (e[i] - p->Tc * cv[i]) / p->Hwv * p->dt * p->rate;
      isphasechange = (orc_park_uniform(seed) < threshold) && pc_around(p, i, x, type, off, neigh);
    } else {
      isphasechange = (orc_park_uniform(seed) < p->change_chance) && (Ti > p->Tt) &&
                      pc_around(p, i, x, type, off, neigh);
    }
    if (!isphasechange) continue;
    double coord[3];
    int ok = 0, natempt = 0;
    double delta = p->dr;
    do {
      pc_newpos(p->dim, seed, x + 3 * i, cg + 3 * i, delta, coord);
      ok = pc_mine(p, coord);
      delta = 0.75 * delta;
      natempt++;
    } while (!ok && natempt < p->maxattempt);
    if (!ok) {
      delta = p->dr;
      natempt = 0;
      do {
        pc_newpos_simple(seed, x + 3 * i, delta, coord);
        ok = pc_mine(p, coord);
        delta = 0.75 * delta;
        natempt++;
      } while (!ok && natempt < p->maxattempt);
    }
    if (!ok) continue;
    /* insert_one_atom -> create_atom(to_type, coord) at m = ncur (:455-462) */
    if (ncur >= nmax) return -1;
    const int m = ncur++;
    type[m] = p->to_type;
    for (int k = 0; k < 3; k++) {
      x[3 * m + k] = coord[k];
      v[3 * m + k] = 0.0;
      cg[3 * m + k] = 0.0;
      vest[3 * m + k] = 0.0;
    }
    rho[m] = 0.0;
    rmass[m] = 0.0;
    e[m] = 0.0;
    cv[m] = 1.0;
    dmass[m] = 0.0;
    /* weights and mass taken, over the atoms now in the list's slots (:242-300) */
    double wtotal = 0.0;
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      if (type[j] == p->from_type && rmass[j] > 0.5 * p->to_mass) {
        const double delx = x[3 * i] - x[3 * j];
        const double dely = x[3 * i + 1] - x[3 * j + 1];
        const double delz = x[3 * i + 2] - x[3 * j + 2];
        const double rsq = delx * delx + dely * dely + delz * delz;
        wtotal += (p->dim == 3) ? orc_kernel_quintic3d(sqrt(rsq) * p->cutoff)
                                : orc_kernel_quintic2d(sqrt(rsq) * p->cutoff);
      }
    }
    double dmom[3] = {0, 0, 0}, dmomest[3] = {0, 0, 0};
    for (long jj = off[i]; jj < off[i + 1]; jj++) {
      const int j = neigh[jj];
      if (type[j] == p->from_type && rmass[j] > 0.5 * p->to_mass) {
        const double delx = x[3 * i] - x[3 * j];
        const double dely = x[3 * i + 1] - x[3 * j + 1];
        const double delz = x[3 * i + 2] - x[3 * j + 2];
        const double rsq = delx * delx + dely * dely + delz * delz;
        const double wfd = (p->dim == 3) ? orc_kernel_quintic3d(sqrt(rsq) * p->cutoff)
                                         : orc_kernel_quintic2d(sqrt(rsq) * p->cutoff);
        const double dmass_aux = p->to_mass * wfd / wtotal;
        dmass[j] += dmass_aux;
        dmom[0] += v[3 * j] * dmass_aux;
        dmom[1] += v[3 * j + 1] * dmass_aux;
        dmom[2] += v[3 * j + 2] * dmass_aux;
        dmomest[0] += vest[3 * j] * dmass_aux;
        dmomest[1] += vest[3 * j + 1] * dmass_aux;
        dmomest[2] += vest[3 * j + 2] * dmass_aux;
      }
    }
    /* the new atom (:302-318): m = atom->nlocal - 1 */
    rmass[m] = p->to_mass;
    rho[m] = rho[i];
    cv[m] = cv[i];
    for (int k = 0; k < 3; k++) {
      v[3 * m + k] = dmom[k] / p->to_mass;
      vest[3 * m + k] = dmomest[k] / p->to_mass;
    }
    const double energy_aux = 0.5 * (e[i] - p->Hwv);
    e[i] = energy_aux;
    e[m] = energy_aux;
  }
  /* nswap < 0: one rank of several -- stop here with the ghosts' dmass in place; the
     caller runs reverse_comm_fix across the ranks' swaps and the finish loop */
  if (nswap < 0) return ncur;
  orc_reverse_swaps(nlocal, nswap, swap_first, ghost_src, dmass);   /* :324 */
  for (int i = 0; i < nlocal; i++) {
    const double mold = rmass[i];
    rmass[i] -= dmass[i];
    e[i] = e[i] * mold / rmass[i];
    dmass[i] = 0;
  }
  return ncur;
}
