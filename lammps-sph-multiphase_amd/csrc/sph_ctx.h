// sph_ctx.h -- the pair-style layer's context (include/sph_hip.h section 1), shared by
// the translation units that implement its entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdlib>
#include <utility>
#include <vector>

#include "sph_kernels.h"
#include "sph_mp_kernels.h"
#include "sph_util.h"

using namespace sph;

// half-list styles gather the j share through the reverse half list; study builds only
// (SPH_MPREV=0) scatter it with fp64 atomics instead
inline bool sph_rev_on() {
#ifdef SPH_STUDY
  static const bool v = [] {
    const char *e = getenv("SPH_MPREV");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
#else
  return true;
#endif
}

// a neighbor list parked in the context while another kind is active (sph_hip_list_keyed)
struct StagedList {
  int kind = -1, inum = 0;
  int64_t key = -1;
  DBuf<int> ilist, off, nbr, rkey, rnbr, rown, roff;
  std::vector<int> hoff, hilist;
  std::vector<double> cns;  // (a device-built list: the cutneighsq it was built with)
  bool rev_ok = false, devbuilt = false;
};

struct sph_hip_ctx {
  int device = 0, dim = 3, ntypes = 1, newton = 1;
  hipStream_t stream = nullptr;
  Coefs hc{};
  Coefs *dc = nullptr;
  bool have_rho = false, have_tait = false, have_heat = false;
  int tait_visc = SPH_VISC_MONAGHAN;
  int nlocal = 0, nghost = 0;
  bool have_atoms = false;
  int list_kind = -1, inum = 0;
  DBuf<double4> xf, vr, fo;
  DBuf<double> en, de, rho_out, virial, raw;  // (raw: LAMMPS arrays as uploaded)
  DBuf<int> ty, ilist, off, nbr, lbad;
  // multiphase styles (atom_style meso/multiphase): per-atom rmass and cv, own coefficients
  DBuf<double> rm, cv;
  DBuf<double4> cg, cgin;
  bool have_mp_atoms = false;
  bool have_mp_rho = false, have_mp_tait = false, have_mp_heat = false, have_mp_cg = false;
  bool have_mp_st = false;
  // reverse of the staged half list (k_mp_half REV), built on first use after a list upload
  DBuf<int> rkey, rnbr, rown, roff;
  DBuf<unsigned char> tmp;
  bool rev_ok = false;
  std::vector<double4> h4in;
  MpCoefs hm{};
  MpCoefs *dm = nullptr;
  bool mp_dirty = true;
  std::vector<double4> h4;
  std::vector<double> h1;
  std::vector<int> hoff, hnbr, hilist;
  bool coef_dirty = true;
  // the caller's host arrays registered as mapped host memory (sph_hip_host_arrays): the
  // kernels read inputs from and add results into them directly over PCIe
  struct HostMap {
    void *host = nullptr;
    size_t bytes = 0;
    void *dev = nullptr;
  };
  std::vector<HostMap> hmaps;
  // device address of [p, p + bytes) if a registered range holds it, else nullptr
  void *mapped(const void *p, size_t bytes) const {
    if (!p) return nullptr;
    const char *q = static_cast<const char *>(p);
    for (const auto &m : hmaps) {
      const char *h = static_cast<const char *>(m.host);
      if (q >= h && q + bytes <= h + m.bytes)
        return static_cast<char *>(m.dev) + (q - h);
    }
    return nullptr;
  }
  void unmap_all() {
    for (auto &m : hmaps) (void)hipHostUnregister(m.host);
    hmaps.clear();
  }
  // device-built lists (sph_hip_build_list, sph_pair_lists.hip): the active list was built
  // on the device; bins, bin-ordered copy, counts and the full list behind a half one
  bool list_devbuilt = false;
  std::vector<double> list_cns;
  DBuf<double> lbox;
  DBuf<unsigned> bkey, bkey2;
  DBuf<int> bidx, bidx2, qbeg, tb, lcnt, loff, lnbr;
  DBuf<double4> xb;
  // the active list's build key (-1: not reusable) and the parked lists, one per kind
  int64_t list_key = -1;
  StagedList parked[2];
  void swap_active(StagedList &p) {
    std::swap(list_kind, p.kind);
    std::swap(inum, p.inum);
    std::swap(list_key, p.key);
    std::swap(ilist, p.ilist);
    std::swap(off, p.off);
    std::swap(nbr, p.nbr);
    std::swap(rkey, p.rkey);
    std::swap(rnbr, p.rnbr);
    std::swap(rown, p.rown);
    std::swap(roff, p.roff);
    std::swap(hoff, p.hoff);
    std::swap(hilist, p.hilist);
    std::swap(rev_ok, p.rev_ok);
    std::swap(list_devbuilt, p.devbuilt);
    std::swap(list_cns, p.cns);
  }
  // make the kind-k list the active one: the active list is parked under its own kind,
  // the kind-k slot's list (if any) becomes active; a slot's stale buffers are kept for reuse
  void select_list(int k) {
    if (list_kind == k) return;
    if (list_kind >= 0) swap_active(parked[list_kind]);
    swap_active(parked[k]);
    if (parked[k].kind != k) {  // (what came back is not a kind-k list: an empty slot)
      parked[k].kind = -1;
      parked[k].key = -1;
      parked[k].rev_ok = false;
    }
    if (list_kind != k) {
      list_kind = k;
      list_key = -1;
      inum = 0;
      rev_ok = false;
    }
  }
  // every staged list stale (the atom set changed): restage before the next style call
  void drop_lists() {
    list_kind = -1;
    list_key = -1;
    rev_ok = false;
    for (auto &p : parked) {
      p.kind = -1;
      p.key = -1;
      p.rev_ok = false;
    }
  }
  void release_lists() {
    for (auto &p : parked)
      for (DBuf<int> *b : {&p.ilist, &p.off, &p.nbr, &p.rkey, &p.rnbr, &p.rown, &p.roff})
        b->release();
    for (DBuf<int> *b : {&bidx, &bidx2, &qbeg, &tb, &lcnt, &loff, &lnbr}) b->release();
    bkey.release();
    bkey2.release();
    xb.release();
    lbox.release();
  }
  // optional device timing of each style call's kernels (sph_hip_set_timing)
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double kernel_ms = 0.0;
  void tstart() {
    if (timing) SPH_HIP_TRY(hipEventRecord(ev0, stream));
  }
  void tstop() {
    if (timing) SPH_HIP_TRY(hipEventRecord(ev1, stream));
  }
  // after the stream synchronised
  void tread() {
    if (!timing) return;
    float ms = 0.f;
    SPH_HIP_TRY(hipEventElapsedTime(&ms, ev0, ev1));
    kernel_ms = ms;
  }

  // Reverse of the staged half list: entries sorted by j (stable radix sort of (j, row
  // atom) pairs), CSR offsets over the reverse rows (nall with newton_pair, else nlocal:
  // without newton the reference gives ghosts no share).  Built once per list upload.
  int rev_rows() const { return newton ? nlocal + nghost : nlocal; }
  void build_rev() {
    if (rev_ok) return;
    const int nall = nlocal + nghost;
    const int tot = hoff[inum];
    const int nrows = rev_rows();
    rkey.reserve(tot > 0 ? tot : 1);
    rnbr.reserve(tot > 0 ? tot : 1);
    rown.reserve(tot > 0 ? tot : 1);
    roff.reserve((size_t)nrows + 1);
    if (inum)
      hipLaunchKernelGGL(k_entry_owner, dim3((inum + 255) / 256), dim3(256), 0, stream, inum,
                         off.p, ilist.p, rown.p);
    int endbit = 1;
    while ((1u << endbit) < (unsigned)(nall + 1) && endbit < 31) endbit++;
    if (tot) {
      size_t tb = 0;
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, nbr.p, rkey.p, rown.p, rnbr.p,
                                                     tot, 0, endbit, stream));
      tmp.reserve(tb);
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, nbr.p, rkey.p, rown.p, rnbr.p,
                                                     tot, 0, endbit, stream));
    }
    hipLaunchKernelGGL(k_rev_offsets, dim3((nrows + 1 + 255) / 256), dim3(256), 0, stream,
                       nrows, tot, rkey.p, roff.p);
    SPH_HIP_TRY(hipGetLastError());
    rev_ok = true;
  }
  void upload_mp() {
    if (!mp_dirty) return;
    mp_inverses(hm);
    SPH_HIP_TRY(hipMemcpyAsync(dm, &hm, sizeof(MpCoefs), hipMemcpyHostToDevice, stream));
    mp_dirty = false;
  }
  void upload_coefs() {
    if (!coef_dirty) return;
    SPH_HIP_TRY(hipMemcpyAsync(dc, &hc, sizeof(Coefs), hipMemcpyHostToDevice, stream));
    coef_dirty = false;
  }
};

