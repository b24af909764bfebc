// sph_engine_mp.h -- streaming kernels of the multiphase engine (atom_style meso/multiphase,
// bubble_growth/bubble.lmp): the extra per-atom fields through sort/exchange/borders/
// forward, the hand-off between the multiphase pair passes, the one-field reverse comm of
// fix phase_change, and its device-side bookkeeping (finish, new atoms).
#pragma once
#include <hip/hip_runtime.h>

#include "sph_engine_kernels.h"

namespace sph {

// extra per-atom fields, packed MPX doubles per atom: v[3], rmass, cv, colorgradient[3]
// (atom_vec_meso_multiphase.cpp pack_border_vel / pack_comm_vel carry v, rmass, cv and the
// colorgradient next to the x, vest, rho, e of the single-phase records)
constexpr int MPX = 8;

// buf[k] <- fields of atom src[k] (src == nullptr: atom k)
static __global__ void k_mpx_pack(int n, const int *__restrict__ src,
                                  const double4 *__restrict__ vel, const double *__restrict__ rm,
                                  const double *__restrict__ cv, const double4 *__restrict__ cg,
                                  double *__restrict__ buf) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = src ? src[k] : k;
  const double4 v = vel[i], c = cg[i];
  double *const o = buf + (size_t)MPX * k;
  o[0] = v.x;
  o[1] = v.y;
  o[2] = v.z;
  o[3] = rm[i];
  o[4] = cv[i];
  o[5] = c.x;
  o[6] = c.y;
  o[7] = c.z;
}

// atom first + k <- buf[sel[k]] (sel == nullptr: buf[k])
static __global__ void k_mpx_unpack(int n, const int *__restrict__ sel, int first,
                                    const double *__restrict__ buf, double4 *__restrict__ vel,
                                    double *__restrict__ rm, double *__restrict__ cv,
                                    double4 *__restrict__ cg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double *const o = buf + (size_t)MPX * (sel ? sel[k] : k);
  const int i = first + k;
  vel[i] = make_double4(o[0], o[1], o[2], vel[i].w);  // (w: the owned atoms' image flags)
  rm[i] = o[3];
  cv[i] = o[4];
  cg[i] = make_double4(o[5], o[6], o[7], 0.0);
}

// rhosum/multiphase result into the owned rows' rho (vr.w); ghosts keep theirs (A.6-1)
static __global__ void k_mp_rho_store(int n, const double *__restrict__ rho,
                                      double4 *__restrict__ vr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) vr[i].w = rho[i];
}

// rho and colorgradient of atoms [0, n) as they are now (k_mp_gather's S or F version)
static __global__ void k_mp_snap(int n, const double4 *__restrict__ vr,
                                 const double4 *__restrict__ cg, double *__restrict__ rho,
                                 double4 *__restrict__ cgo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  rho[i] = vr[i].w;
  cgo[i] = cg[i];
}
// k_mp_gather's per-atom records, so a neighbour costs four loads instead of ten scattered
// ones: A = (x, y, z, rmass), K = (v, T = e/cv [heat]), F / S = (colorgradient, rho) in the
// fresh / stale version (the gather picks one per pair, see k_mp_gather)
static __global__ void k_mp_pack_rec(int nall, const double4 *__restrict__ xf,
                                     const double4 *__restrict__ vel, const double *__restrict__ rm,
                                     const double *__restrict__ en, const double *__restrict__ cv,
                                     const double *__restrict__ rhoF, const double *__restrict__ rhoS,
                                     const double4 *__restrict__ cgF, const double4 *__restrict__ cgS,
                                     int heat, double4 *__restrict__ A, double4 *__restrict__ K,
                                     double4 *__restrict__ F, double4 *__restrict__ S) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nall) return;
  const double4 x = xf[i], v = vel[i], cf = cgF[i], cs = cgS[i];
  A[i] = make_double4(x.x, x.y, x.z, rm[i]);
  K[i] = make_double4(v.x, v.y, v.z, heat ? en[i] / cv[i] : 0.0);  // (sph_energy2t)
  F[i] = make_double4(cf.x, cf.y, cf.z, rhoF[i]);
  S[i] = make_double4(cs.x, cs.y, cs.z, rhoS[i]);
}

// colorgradient's records: (x, y, z, sigma = rho / rmass), pair_sph_colorgradient.cpp:139, 173
static __global__ void k_mp_pack_sigma(int nall, const double4 *__restrict__ xf,
                                       const double4 *__restrict__ vr,
                                       const double *__restrict__ rm, double4 *__restrict__ xs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nall) return;
  const double4 x = xf[i];
  xs[i] = make_double4(x.x, x.y, x.z, vr[i].w / rm[i]);
}

// the fresh version of the ghosts from their owners (one brick)
static __global__ void k_mp_fwd_fresh(int nghost, int nlocal, const int *__restrict__ gowner,
                                      double *__restrict__ rho, double4 *__restrict__ cg) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nghost) return;
  const int o = gowner[g];
  rho[nlocal + g] = rho[o];
  cg[nlocal + g] = cg[o];
}
static __global__ void k_mp_pack_fresh(int n, const int *__restrict__ list,
                                       const double *__restrict__ rho,
                                       const double4 *__restrict__ cg, double *__restrict__ buf) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];
  const double4 c = cg[i];
  double *const o = buf + 4 * (size_t)k;
  o[0] = rho[i];
  o[1] = c.x;
  o[2] = c.y;
  o[3] = c.z;
}
static __global__ void k_mp_unpack_fresh(int n, int first, const double *__restrict__ buf,
                                         double *__restrict__ rho, double4 *__restrict__ cg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double *const o = buf + 4 * (size_t)k;
  rho[first + k] = o[0];
  cg[first + k] = make_double4(o[1], o[2], o[3], 0.0);
}

// comm->reverse_comm_fix of one per-atom double (one brick): owner += ghost
static __global__ void k_reverse1(int nghost, int nlocal, const int *__restrict__ gowner,
                                  double *__restrict__ a) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nghost) return;
  atomicAdd(&a[gowner[g]], a[nlocal + g]);
}
static __global__ void k_pack_rev1(int n, int first, const double *__restrict__ a,
                                   double *__restrict__ buf) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) buf[k] = a[first + k];
}
static __global__ void k_unpack_rev1(int n, const int *__restrict__ list,
                                     const double *__restrict__ buf, double *__restrict__ a) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) atomicAdd(&a[list[k]], buf[k]);
}

// ---- fix phase_change bookkeeping -------------------------------------------------------
// what the stream replay needs of candidate atom cand[k]: x[3], cg[3], e, cv, rho (9
// doubles) and its order key (the LAMMPS local index)
static __global__ void k_pc_gather(int n, const int *__restrict__ cand,
                                   const double4 *__restrict__ xf,
                                   const double4 *__restrict__ vr, const double *__restrict__ en,
                                   const double *__restrict__ cv, const double4 *__restrict__ cg,
                                   const int *__restrict__ key, double *__restrict__ out,
                                   int *__restrict__ okey) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = cand[k];
  const double4 x = xf[i], c = cg[i];
  double *const o = out + 9 * (size_t)k;
  o[0] = x.x;
  o[1] = x.y;
  o[2] = x.z;
  o[3] = c.x;
  o[4] = c.y;
  o[5] = c.z;
  o[6] = en[i];
  o[7] = cv[i];
  o[8] = vr[i].w;
  okey[k] = key[i];
}
// e of the atoms that changed phase (:317-320)
static __global__ void k_pc_set_e(int n, const int *__restrict__ idx,
                                  const double *__restrict__ val, double *__restrict__ en) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) en[idx[k]] = val[k];
}
// rmass -= dmass, e renormalised (:325-334), over the atoms owned when pre_exchange began
static __global__ void k_pc_finish(int n, const double *__restrict__ dmass,
                                   double *__restrict__ rm, double *__restrict__ en) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double mold = rm[i];
  const double m = mold - dmass[i];
  rm[i] = m;
  en[i] = en[i] * mold / m;
}
// the new atoms at first + k: AtomVecMesoMultiPhase::create_atom defaults (colorgradient 0,
// de = drho = 0) and the fix's fields from the 13-double records {x[3], v[3], vest[3], e,
// rmass, rho, cv} (:291-320)
static __global__ void k_pc_append(int n, const double *__restrict__ rec, int first,
                                   int to_type, int tag0, double4 *__restrict__ xf,
                                   double4 *__restrict__ vr, double4 *__restrict__ vel,
                                   double *__restrict__ en, double *__restrict__ rm,
                                   double *__restrict__ cv, double4 *__restrict__ cg,
                                   int *__restrict__ ty, int *__restrict__ tag,
                                   double4 *__restrict__ fo, double *__restrict__ de) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double *const o = rec + 13 * (size_t)k;
  const int i = first + k;
  xf[i] = make_double4(o[0], o[1], o[2], 0.0);
  vel[i] = make_double4(o[3], o[4], o[5], (double)IMG_ZERO);  // create_atom: zero image
  vr[i] = make_double4(o[6], o[7], o[8], o[11]);
  en[i] = o[9];
  rm[i] = o[10];
  cv[i] = o[12];
  cg[i] = make_double4(0.0, 0.0, 0.0, 0.0);
  ty[i] = to_type;
  tag[i] = tag0 + k;
  fo[i] = make_double4(0.0, 0.0, 0.0, 0.0);
  de[i] = 0.0;
}

}  // namespace sph
