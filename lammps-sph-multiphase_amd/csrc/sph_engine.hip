// sph_engine.hip -- device-resident engine of the C ABI (include/sph_hip.h, section 2).
//
// One engine = one rank's share of an SPH run, resident in HBM.  A step is Verlet::run's
// sequence (src/verlet.cpp:222-308) specialised to the USER-SPH hot path:
//   initial_integrate -> [rebuild: pbc, spatial sort, borders, bins, full list]
//   | forward comm -> rhosum (+EOS) -> forward rho -> taitwater[/morris][+heat] ->
//   final_integrate
// Full lists are walked gather-only, so the reverse communication of the reference
// (comm->reverse_comm, verlet.cpp:290-293) has nothing to carry and is skipped.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cmath>
#include <vector>

#include "sph_coef.h"
#include "sph_comm.h"
#include "sph_dispatch.h"
#include "sph_blk_kernels.h"
#ifdef SPH_STUDY  // (k_blk_build2: measured slower, study builds only)
#include "sph_blk_build2.h"
#endif
#include "sph_engine_kernels.h"
#include "sph_engine_mp.h"
#include "sph_ipc.h"
#include "sph_mp2_kernels.h"
#include "sph_pc.h"
#include "sph_row2_kernels.h"
#include "sph_util.h"

using namespace sph;

namespace sph {
#ifndef SPH_INNER_FRAC
#define SPH_INNER_FRAC 0.0625
#endif
int g_alloc_log = 0;
static int env_int(const char *name, int dflt) {
  const char *s = getenv(name);
  return s ? atoi(s) : dflt;
}
// Study knobs (tools/kernel_sweep.py, tools/build_sweep.py) exist only in study builds
// (make STUDY=1 -> -DSPH_STUDY); the production library ignores the variables, so no
// environment setting can change its results or run a variant whose outputs are
// meaningless.
#ifdef SPH_STUDY
static int study_int(const char *name, int dflt) { return env_int(name, dflt); }
#else
static int study_int(const char *, int dflt) { return dflt; }
#endif
// SPH_ROW2TILE: shape index of SPH_ROW2_TILES (default 3 = 8 lanes x 4 pairs, the fastest
// with lane-pair gathers on C2 1M: profiles/r01/sweep_row2.log)
int row2_tile() {
  static int t = study_int("SPH_ROW2TILE", 3);
  return t;
}
}  // namespace sph
// SPH_MORTON_DIV (default 4, the fastest of 1/2/4/8 on C2 1M for the row path): cells per
// bin edge of the owned atoms' sort key (Morton for the row path, Hilbert for the block path)
static int morton_div() {
  static int v = std::max(1, study_int("SPH_MORTON_DIV", 4));
  return v;
}
// Row path (kernel_path 1) knobs.  SPH_LP (default 1): lane-pair gathers in the row2
// kernels; SPH_IV (default 1): the strided list is stored chunk-transposed so each lane's
// four indices of a chunk are one 16-B load (sph_row2_kernels.h).
static bool row2_lp() {
  static bool v = study_int("SPH_LP", 1) != 0;
  return v;
}
// SPH_TIGHT (default 0): with a strided list, the rhosum pass writes this step's in-cut
// list (k_row2_rhosum TIGHT) and the force pass walks it instead of the full list.
// Measured on C2 1M: taitwater 0.57 -> 0.46 ms but rhosum 0.31 -> 0.48 ms (the stores
// count in vmcnt, so the loop waits for them with the prefetched indices) -> off.
static bool tight_on() {
  static bool v = study_int("SPH_TIGHT", 0) != 0;
  return v;
}
// SPH_PI (default 0): pair-interleaved entry slots with lane-pair gathers (entry_slot).
// Measured on C2 1M: taitwater 0.562 (off) vs 0.567 ms (on), rhosum equal -> off.
static bool row2_pi() {
  static bool v = study_int("SPH_PI", 0) != 0 && row2_lp();
  return v;
}
static bool row2_iv() {
  static bool v = study_int("SPH_IV", 1) != 0;
  return v;
}
// SPH_EXP: study variants of the pair passes (tools/kernel_sweep.py sets it for the timed
// passes only, so it is read per launch); 0 in production
static int row2_exp() { return study_int("SPH_EXP", 0); }
// SPH_OVERLAP (default 0): with a brick decomposition, run the pair passes of interior
// rows (no ghost in the list) on a second stream while the forward / rho halos are in
// flight, then the boundary rows after them (sph_engine::pair_compute_overlap).  Parity
// holds (tests/test_gpu_bricks.py with SPH_OVERLAP=1), but on one GPU through the RCCL
// loopback it measured 1.29 (serial) -> 1.35 ms per step at C2 1M: the split launches
// cost more than the loopback halo they hide.  Whether xGMI transfers (~17 MB per step
// per rank at C4) change that is unmeasured here (no multi-GPU box) -> off by default.
// SPH_TBITS (default 1): with several types, strided list entries carry the neighbour's
// type in their top bits, so the row2 passes skip the per-neighbour type gather
static bool tbits_env() {
  static bool v = study_int("SPH_TBITS", 1) != 0;
  return v;
}
// SPH_BLK (default 0 = 64-row blocks, 8 lanes x 4 slots; the fastest pair passes on C2 1M):
// block shape of the block-staged path (SPH_BLK_SHAPES)
static int blk_shape_env() {
  static int v = study_int("SPH_BLK", 0);
  return v;
}
// SPH_DIRECT (study builds; default 1): bricks forward the per-step halos owner -> ghost in
// one exchange
static bool direct_env() {
  static bool v = study_int("SPH_DIRECT", 1) != 0;
  return v;
}
// SPH_HIL_POW2 (default 1): power-of-two Hilbert cells per axis of the owned sub-box
static bool hil_pow2() {
  static bool v = study_int("SPH_HIL_POW2", 1) != 0;
  return v;
}
// SPH_SORT_EVERY (default 10): steps between spatial sorts of the owned atoms at rebuilds
// (row path and the multiphase stack)
static int sort_every() {
  static int v = study_int("SPH_SORT_EVERY", 10);
  return v;
}

// SPH_MP_TYPED (default 1): the multiphase passes take the neighbour's type from the entry
static bool mp_typed_env() {
  static bool v = study_int("SPH_MP_TYPED", 1) != 0;
  return v;
}
// one brick's borders: a dimension's two swaps in three launches (k_brd_*), or the
// per-swap flags + select + append of earlier rounds (SPH_BRD_FUSED=0, builds)
#ifndef SPH_BRD_FUSED
#define SPH_BRD_FUSED 1
#endif
// SPH_ROWSORT (study builds; default 0): the pair passes walk each block's rows longest
// first (k_blk_build's per-block order), so that a wave's rows have similar lengths
static bool rowsort() {
#ifndef SPH_ROWSORT_DEFAULT
#define SPH_ROWSORT_DEFAULT 0  // (on: force 0.291 vs 0.287 ms, rhosum 0.123 vs 0.111, profiles/r04/rowsort)
#endif
  static bool v = study_int("SPH_ROWSORT", SPH_ROWSORT_DEFAULT) != 0;
  return v;
}
// SPH_N3 (study builds only; default 0): the block build keeps each pair of rows of one
// block once (Newton-3 inside the blocks, k_blk_build N3) -- measured slower, DESIGN.md 5.2
// SPH_INNER_REFRESH (study builds; default 1): derive the inner rows again between rebuilds
// once an atom has moved past their margin (refresh_inner)
static bool inner_inline() {
  static bool v = study_int("SPH_INNER_INLINE", 1) != 0;
  return v;
}
static bool refresh_env() {
  static bool v = study_int("SPH_INNER_REFRESH", 1) != 0;
  return v;
}
static bool n3_env() {
  static bool v = BLK_N3_BUILT && study_int("SPH_N3", 0) != 0;
  return v;
}
// SPH_MP_RHOFUSE (default 1): the multiphase engine's list fill sums rhosum/multiphase over
// the hits it finds when the list is built in the step whose forces follow (k_neigh3 RHO)
static bool rhofuse_env() {
  static bool v = study_int("SPH_MP_RHOFUSE", 1) != 0;
  return v;
}

namespace {

constexpr int BLK = 256;
inline unsigned blocks(long n) { return (unsigned)((n + BLK - 1) / BLK); }

enum TimerClass { T_RHO, T_TAIT, T_HEAT, T_INT, T_COMM, T_NEIGH, T_NCLASS };

}  // namespace

struct sph_engine {
  int device = 0;
  hipStream_t s = nullptr;
  sph_engine_config cfg{};
  Coefs hc{};
  Coefs *dc = nullptr;
  Box box{};
  double sublo[3], subhi[3];
  double cutneighmax = 0.0, cutghost = 0.0;
  StepConst sc{};
  int force_mode = 0;  // M_TAIT | M_HEAT

  // multiphase stack (cfg.mp, sph_engine_mp.h): per-atom rmass, cv, colorgradient of owned
  // atoms and ghosts, and the ghosts' v (comm vel yes)
  bool mp = false;
  sph_engine_mp_config mpc{};
  MpCoefs hm{};
  MpCoefs *dm = nullptr;
  DBuf<double> rm, cvv, rho_tmp, dmass, xbuf, xbuf2, rhoS, rhoF;
  DBuf<double4> cg, cgS, cgF;
  DBuf<double4> recA, recK, recF, recS;  // k_mp_gather's packed records (k_mp_pack_rec)
  // fix phase_change scratch, kept across calls (no allocation per step)
  DBuf<int> pc_flag, pc_cand, pc_otag, pc_idx, pc_minr, pc_one, pc_grank, pc_key, pc_val, gsrc;
  std::vector<int> gswap_first;  // one brick: first ghost of each swap (+ nghost at the end)
  int gcap_hint = 0;              // one brick: ghost room of the next borders
  DBuf<int> gnall;                // one brick: nall before each swap (+ the overflow word)
  DBuf<int> bcnt;                 // one brick: the swaps' per-block counts (k_brd_*)
  DBuf<double> pc_rec, pc_gat, pc_Wd, pc_vals, pc_nrec, pc_v0, pc_v1;
  DBuf<unsigned long long> pc_k0, pc_k1;  // the donations' (donor, candidate) sort keys
  DBuf<int> pc_cnt;
  int64_t migrations = 0;  // atoms that left this brick at exchanges so far
  // LAMMPS' local order of the owned atoms, tracked while fix phase_change is armed (its
  // candidates meet the random stream in that order): lidx[row] = the atom's index in the
  // reference's arrays -- read order, CommBrick::exchange's hole fill, Atom::sort at setup and
  // every sortfreq steps (atom_modify sort, default 1000 at half the neighbour cutoff)
  DBuf<int> lidx, lidx2, lidx_tab;
  DBuf<unsigned long long> skey, skey2;
  DBuf<int> srow, srow2;
  std::vector<char> h_leave;
  bool lidx_valid = false;
  int sortfreq = 1000;
  double sort_binsize = 0.0;
  int64_t nextsort = 0;
  // fix phase_change (one brick): parameters, stream state, next call, atoms created
  bool pc = false;
  sph_phasechange_params pcp{};
  int pc_nevery = 1, pc_seed = 0;
  int64_t pc_next = 1, pc_inserted = 0;
  int tag_next = 0;  // tag of the next created atom (atom->tag_extend)
  bool pc_tags_agreed = false;  // bricks: tag_next agreed over the ranks (first call)
  std::vector<double> cv_by_tag;  // single-phase engines: the constant cv, for restarts

  int nlocal = 0, nghost = 0;
  // brick decomposition (CommBrick): this brick's grid location, face neighbours, swaps
  int pg[3] = {1, 1, 1}, myloc[3] = {0, 0, 0}, procneigh[3][2] = {{0, 0}, {0, 0}, {0, 0}};
  int me = 0, nprocs = 1;
  Transport *tr = nullptr;
  struct Swap {
    int dim = 0, dir = 0, sendproc = 0, recvproc = 0, nsend = 0, nrecv = 0, firstrecv = 0;
    int pbc = 0;
    double lo = 0.0, hi = 0.0, shift = 0.0;
    double lo_sel = 0.0, hi_sel = 0.0;  // (the selection's slab: empty without a send)
    bool remote = false;
    DBuf<int> list;
  };
  Swap swaps[6];
  int nswap = 0;
  DBuf<unsigned char> cbs, cbr, flag2;
  DBuf<int> sel2;
  // loopback: a one-brick run whose periodic self swaps go through the attached
  // communicator (RCCL send/recv to itself) instead of device copies -- the multi-brick
  // data path (slab selection, packing, RCCL groups, unpacking) on one GPU
  bool loopback = false;
  bool multi() const { return pg[0] * pg[1] * pg[2] > 1 || loopback; }
  // halo/compute overlap (multi only): interior and boundary rows of the current list
  hipStream_t s2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  DBuf<int> rows_in, rows_bd;
  DBuf<unsigned char> fl_in, fl_bd;
  int n_in = 0, n_bd = 0;
  bool ov_ready = false;  // rows_in / rows_bd describe the current list
  bool overlap = false;   // halo/compute overlap (sph_engine_tune SPH_TUNE_OVERLAP)
  int blkumf = 0;         // force pass LDS image cap in records (SPH_TUNE_BLKUMF; 0 = auto)
  int64_t step = 0;
  int64_t rho_fused_step = -1;  // step whose rhosum/multiphase the list fill summed (k_neigh3 RHO)
  int64_t last_sort = 0;        // step of the last spatial sort of the owned atoms
  bool force_sort = false;  // the next rebuild sorts (sph_engine_rebuild_passes)
  bool setup_done = false;
  bool global_tags = false;
  int last_build = 0;

  // atoms (owned first, then ghosts): layout of sph_kernels.h
  DBuf<double4> xf, vr;
  DBuf<double> en;
  DBuf<int> ty;
  // owned only
  DBuf<double4> vel, fo;
  DBuf<double> de;
  DBuf<int> tag;
  // sort scratch
  DBuf<double4> xf2, vr2, vel2;
  DBuf<double> en2;
  DBuf<int> ty2, tag2;
  // ghosts
  DBuf<int> gowner, gimg;
  DBuf<int> gorank, goidx;  // bricks: each ghost's origin rank and owned index (gimg: image)
  // direct forward comm (build_direct): peers, per-peer record offsets (sends / receives),
  // send lists (owned indices), receiving ghost slots, ghosts imaging own atoms
  bool dr_ok = false;
  std::vector<int> dr_peer;
  std::vector<size_t> dr_soff, dr_roff;
  DBuf<int> dr_sidx, dr_rslot, dr_self, dr_req;
  DBuf<int> dr_byq, dr_byg, dr_hist;  // ghosts grouped by origin rank: owned index, slot
  int dr_nself = 0;
  std::vector<const void *> dr_sb;
  std::vector<void *> dr_rb;
  std::vector<size_t> dr_sbytes, dr_rbytes;
  // borders scratch
  DBuf<unsigned char> flags;
  DBuf<int> sel, nsel;
  // bins
  Bins bn{};
  int nbins = 0;
  QBins qb{};
  int nqbins = 0;
  DBuf<int> qbeg, tb, xpos;
  DBuf<double4> xb;
  DBuf<unsigned> bkey, bkey2;
  DBuf<int> bidx, bidx2;
  // neighbor list
  DBuf<int> cnt, off, nbr;
  int64_t nbr_total = 0;   // list entries (-1: strided list, counted on demand)
  int nbr_builds = 0, nbr_maxrow = 0;
  int64_t inner_refreshes = 0;  // refresh_inner launches
  bool strided = false;    // list in fixed-stride rows (row i at i*list_stride, ccnt[i])
  int list_stride = 0;
  int list_perm_g = 0;     // strided rows stored chunk-transposed for G-lane rows (tpos)
  int list_perm_pi = 0;    // ... with pair-interleaved entry slots
  bool list_tbits = false; // strided entries carry the neighbour's type (SPH_TBIT_SHIFT)
  // this step's in-cut ("tight") list, written by the rhosum pass for the force pass
  DBuf<int> tnbr, tcnt;
  // block-staged path (production, sph_blk_kernels.h): per block of consecutive rows its
  // union of neighbour atoms (ulist, ucnt) and the rows' 16-bit slot rows (snbr)
  bool blk = false;
  int blk_sh = 0, blk_um = 0, blk_umf = 0, blk_sstride = 0, blk_rowcap = 0;
  DBuf<int> ulist, ucnt, kcnt;  // (kcnt: the build's candidates per block, statistics)
  DBuf<unsigned short> snbr;
  // the inner rows' own union (k_blk_build / k_blk_inner): a smaller LDS image for the passes
  DBuf<int> uilist, uicnt;
  bool blk_ksmall = false;  // k_blk_build with the small candidate image (BLK_SCAP_S)
  int blk_kover = 0;        // ... builds it overflowed
  bool blk_iu = false;  // (the inner rows index uilist; else the full union)
  // ... and the inner rows of the build (k_blk_inner: pairs within cut + inner_margin), the
  // owned positions they were written at and the flag that retires them (sc.x0 / sc.moved)
  DBuf<unsigned short> snbi;
  DBuf<int> icnt, moved;
  // the pair passes' row order inside each block (longest row first, k_blk_build)
  DBuf<unsigned char> bperm;
  bool blk_perm = false;
  unsigned char *bperm_buf(int nb, int R) {
    bperm.reserve((size_t)nb * R);
    return bperm.p;
  }
  DBuf<double4> x0;
  double inner_margin = 0.0;
  bool inner = false, inner_written = false;  // (written: by k_blk_build, with the full rows)
  DBuf<int> nbs;  // fixed-stride scratch rows of a CSR build (list_q)
  DBuf<int> mx, ccnt;  // scratch scalars; full-list row counts of the current build
  DBuf<int> pcnt;      // block path with Newton-3 (blk_n3): the rows' stored counts
  bool blk_n3 = false;
  DBuf<long long> blen;
  // cub scratch
  DBuf<unsigned char> tmp;
  // pinned host scalar
  int *h_scalar = nullptr;
  int *h_small = nullptr;  // pinned: a few device words read back together (borders)

  // timing
  bool timing = false;
  int timing_mask = 0;  // classes timed (bit k = TimerClass k)
  struct EvPair {
    hipEvent_t a, b;
    int cls;
  };
  std::vector<EvPair> pending;
  std::vector<hipEvent_t> evpool;
  double ms[T_NCLASS] = {0, 0, 0, 0, 0, 0};
  int64_t nlaunch[T_NCLASS] = {0, 0, 0, 0, 0, 0};

  hipEvent_t get_ev() {
    if (!evpool.empty()) {
      hipEvent_t e = evpool.back();
      evpool.pop_back();
      return e;
    }
    hipEvent_t e;
    SPH_HIP_TRY(hipEventCreate(&e));
    return e;
  }
  // A timed class of the step: a roctx range named after LAMMPS' Timer bucket it stands
  // for (timer.h:19-20: Pair, Neigh, Comm, Modify; seen by rocprofv3 --marker-trace; a few
  // tens of ns without a tool), and where timing asks for it a hipEvent pair
  struct Scope {
    sph_engine *e;
    EvPair p;
    bool on;
    Scope(sph_engine *eng, int cls) : e(eng), on(((eng->timing_mask >> cls) & 1) != 0) {
      static const char *const bucket[T_NCLASS] = {"Pair:rhosum", "Pair:taitwater",
                                                   "Pair:heatconduction", "Modify:integrate",
                                                   "Comm", "Neigh"};
      roctxRangePushA(bucket[cls]);
      if (!on) return;
      p.a = e->get_ev();
      p.b = e->get_ev();
      p.cls = cls;
      SPH_HIP_TRY(hipEventRecord(p.a, e->s));
    }
    ~Scope() {
      roctxRangePop();
      if (!on) return;
      (void)hipEventRecord(p.b, e->s);
      e->pending.push_back(p);
    }
  };
  void harvest() {
    if (pending.empty()) return;
    SPH_HIP_TRY(hipStreamSynchronize(s));
    for (auto &p : pending) {
      float t = 0.f;
      SPH_HIP_TRY(hipEventElapsedTime(&t, p.a, p.b));
      ms[p.cls] += t;
      nlaunch[p.cls] += 1;
      evpool.push_back(p.a);
      evpool.push_back(p.b);
    }
    pending.clear();
  }

  void tmp_reserve(size_t b) { tmp.reserve(b); }

  void ensure_atoms(size_t nall, bool keep) {
    xf.reserve(nall, keep, s);
    vr.reserve(nall, keep, s);
    en.reserve(nall, keep, s);
    ty.reserve(nall, keep, s);
    if (mp) {
      vel.reserve(nall, keep, s);
      rm.reserve(nall, keep, s);
      cvv.reserve(nall, keep, s);
      cg.reserve(nall, keep, s);
    }
  }
  // extra multiphase fields: atoms src[0..n) (nullptr: 0..n) -> xbuf -> atoms first..
  void mpx_copy(int n, const int *src, int first, DBuf<double> &buf) {
    if (!mp || n <= 0) return;
    buf.reserve((size_t)MPX * n, false, s);
    hipLaunchKernelGGL(k_mpx_pack, dim3(blocks(n)), dim3(BLK), 0, s, n, src, vel.p, rm.p, cvv.p,
                       cg.p, buf.p);
    hipLaunchKernelGGL(k_mpx_unpack, dim3(blocks(n)), dim3(BLK), 0, s, n, (const int *)nullptr,
                       first, buf.p, vel.p, rm.p, cvv.p, cg.p);
  }
  bool nt1() const { return cfg.ntypes == 1; }
  // the block force pass's viscosity variant: one type with Monaghan viscosity and viscC = 0
  // (nu = 0 or c0 = 0) has no viscosity term at all (BLK_VISC_NONE)
  int blk_visc() const {
    if (nt1() && cfg.tait_visc == SPH_VISC_MONAGHAN && hc.tait[3].viscC == 0.0)
      return BLK_VISC_NONE;
    return cfg.tait_visc;
  }

  // ------------------------------------------------------------------------------------
  void sort_owned() {
    if (nlocal < 1) return;
    const int n = nlocal;
    bkey.reserve(n);
    bkey2.reserve(n);
    bidx.reserve(n);
    bidx2.reserve(n);
    // Space-filling-curve order over cells of 1/div of a bin per axis (bins fit 10 bits per
    // axis; else linear bins): consecutive rows are a compact region, so a block's union
    // (block path) or a wave's gathers (row path) stay small and within one XCD's L2
    const int div = morton_div();
    Bins kbn = bn;
    for (int k = 0; k < 3; k++)
      if (bn.nb[k] > 1) {
        kbn.nb[k] = bn.nb[k] * div;
        kbn.inv[k] = bn.inv[k] * div;
      }
    if (want_blk()) {
      // block path: cells of ~1/div of a bin over the OWNED sub-box only, so the Hilbert
      // curve (over the next power of two of cells) leaves the rows' region as rarely as
      // possible -- a block of consecutive rows stays one compact piece of space
      for (int k = 0; k < 3; k++) {
        const double ext = subhi[k] - sublo[k];
        if (k >= cfg.dim || ext <= 0.0) {
          kbn.lo[k] = sublo[k];
          kbn.nb[k] = 1;
          kbn.inv[k] = 0.0;
          continue;
        }
        // a power of two per axis: a cubic sub-box (and the 2x1x1 / 2x2x1 / 2x2x2 bricks
        // of a cubic box) is then whole octants of the curve's cube, which the curve leaves
        // only between octants -- with any other count it exits and re-enters the
        // rows' region, and a block of consecutive rows spanning such a jump outgrows the
        // build's candidate image (seen at 125k particles per brick: the whole build fell
        // back to 32-row blocks)
        const int nc0 = std::max(1, (int)std::ceil(ext / (cutneighmax / div)));
        int nc = 1;
        while (nc < nc0 && nc < 1024) nc *= 2;
        if (!hil_pow2()) nc = std::min(nc0, 1024);
        kbn.lo[k] = sublo[k];
        kbn.nb[k] = nc;
        kbn.inv[k] = nc / ext;
      }
    }
    const bool mort = kbn.nb[0] <= 1024 && kbn.nb[1] <= 1024 && kbn.nb[2] <= 1024;
    if (!mort) kbn = bn;
    // the block path orders rows along a Hilbert curve (its blocks of consecutive rows stay
    // compact), the row path along a Morton curve
    int cb = 1;
    const int mx3 = std::max(kbn.nb[0], std::max(kbn.nb[1], kbn.nb[2]));
    while ((1 << cb) < mx3) cb++;
    const bool hil = mort && want_blk() && cb >= 2;
    hipLaunchKernelGGL(k_bin_keys, dim3(blocks(n)), dim3(BLK), 0, s, n, 0, kbn, xf.p, bkey.p,
                       bidx.p, hil ? cb + 1 : (mort ? 1 : 0), cfg.dim);
    // key bits: dim (Hilbert) or 3 (Morton) x bits of the largest cell dimension, else
    // bits(nbins)
    int kb = 1;
    if (mort) {
      kb = cb * (hil ? cfg.dim : 3);
    } else {
      while ((1u << kb) < (unsigned)nbins && kb < 32) kb++;
    }
    size_t tb = 0;
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, bkey.p, bkey2.p, bidx.p, bidx2.p, n, 0, kb, s));
    tmp_reserve(tb);
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, bkey.p, bkey2.p, bidx.p, bidx2.p, n, 0, kb, s));
    // twins of equal capacity: the swaps below then never reallocate (a growing twin would
    // cost a hipMalloc + a synchronising hipFree at every rebuild)
    if (mp) {  // the extra fields in the new order, packed before the permutation
      xbuf.reserve((size_t)MPX * n, false, s);
      hipLaunchKernelGGL(k_mpx_pack, dim3(blocks(n)), dim3(BLK), 0, s, n, bidx2.p, vel.p, rm.p,
                         cvv.p, cg.p, xbuf.p);
    }
    grow_twins();
    hipLaunchKernelGGL(k_permute, dim3(blocks(n)), dim3(BLK), 0, s, n, bidx2.p, xf.p, vr.p,
                       en.p, ty.p, vel.p, tag.p, xf2.p, vr2.p, en2.p, ty2.p, vel2.p, tag2.p);
    std::swap(xf, xf2);
    std::swap(vr, vr2);
    std::swap(en, en2);
    std::swap(ty, ty2);
    std::swap(vel, vel2);
    std::swap(tag, tag2);
    if (pc) {  // (the LAMMPS index rides along)
      lidx2.reserve_exact(lidx.cap);
      hipLaunchKernelGGL(k_lidx_take, dim3(blocks(n)), dim3(BLK), 0, s, n, bidx2.p, lidx.p, 0,
                         (const int *)nullptr, lidx2.p);
      std::swap(lidx, lidx2);
    }
    if (mp)
      hipLaunchKernelGGL(k_mpx_unpack, dim3(blocks(n)), dim3(BLK), 0, s, n, (const int *)nullptr,
                         0, xbuf.p, vel.p, rm.p, cvv.p, cg.p);
  }

  // the sort's twins at the capacity of the arrays they swap with; called again at the end
  // of every build, so that the growth borders caused (ghosts) is matched in the same build
  // -- at setup -- and not by a hipMalloc + synchronising hipFree in the next one (~1 ms of
  // host time in the first rebuild after setup, profiles/r04/first_rebuild)
  void grow_twins() {
    xf2.reserve_exact(xf.cap);
    vr2.reserve_exact(vr.cap);
    en2.reserve_exact(en.cap);
    ty2.reserve_exact(ty.cap);
    vel2.reserve_exact(vel.cap);
    tag2.reserve_exact(tag.cap);
  }

  // kernel_path 0: block-staged passes (production; the row path takes over for a build
  // whose blocks overflow); 1: the row path (row2 gathers over the strided global list)
  bool want_blk() const { return cfg.kernel_path == 0; }

  int read_scalar(const int *dptr) {
    SPH_HIP_TRY(hipMemcpyAsync(h_scalar, dptr, sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    return *h_scalar;
  }

  // CommBrick::setup slabs (comm_brick.cpp:330-380) + borders (:696-864) on one process

  // ordered indices i in [0, n) with flag[i] != 0 -> out (returns the count; host sync)
  int select_flagged(const unsigned char *flag, int n, DBuf<int> &out) {
    out.reserve(n > 0 ? n : 1);
    nsel.reserve(1);
    if (n == 0) return 0;
    hipcub::CountingInputIterator<int> it(0);
    size_t tb = 0;
    SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, flag, out.p, nsel.p, n, s));
    tmp_reserve(tb);
    SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, it, flag, out.p, nsel.p, n, s));
    return read_scalar(nsel.p);
  }

  // move the packed send buffer (cbs, sbytes) of swap-like traffic to cbr (rbytes)
  void swap_move(bool remote, size_t sbytes, int dest, size_t rbytes, int src) {
    if (remote) {
      tr->exchange(cbs.p, sbytes, dest, cbr.p, rbytes, src, s);
    } else if (rbytes) {
      SPH_HIP_TRY(hipMemcpyAsync(cbr.p, cbs.p, rbytes, hipMemcpyDeviceToDevice, s));
    }
  }

  // CommBrick::borders over a procgrid (comm_brick.cpp:690-880, maxneed = 1).  Both swaps
  // of a dimension select from the same atoms (owned + earlier dimensions' ghosts), so
  // their counts travel in one exchange and their records in another; the ghosts of the
  // lower swap are appended before those of the upper one, as in CommBrick.
  void borders_multi() {
    nghost = 0;
    int nall = nlocal;
    nswap = 0;
    for (int d = 0; d < cfg.dim; d++) {
      const int nlast = nall;
      Swap *pair[2] = {&swaps[nswap], &swaps[nswap + 1]};
      nswap += 2;
      for (int dir = 0; dir < 2; dir++) {
        Swap &sw = *pair[dir];
        sw.dim = d;
        sw.dir = dir;
        sw.sendproc = procneigh[d][dir];
        sw.recvproc = procneigh[d][1 - dir];
        sw.remote = pg[d] > 1 || loopback;
        bool sendflag = true;  // sendneed/recvneed across a non-periodic boundary (:226-274)
        if (!box.periodic[d]) sendflag = dir == 0 ? myloc[d] > 0 : myloc[d] < pg[d] - 1;
        sw.lo = dir == 0 ? -1.0e20 : subhi[d] - cutghost;
        sw.hi = dir == 0 ? sublo[d] + cutghost : 1.0e20;
        int pbc = 0;
        if (dir == 0 && myloc[d] == 0) pbc = 1;
        if (dir == 1 && myloc[d] == pg[d] - 1) pbc = -1;
        sw.shift = pbc * box.prd[d];
        sw.pbc = pbc;
        // the selection's count stays on the device (nsel[dir]); both swaps' counts and the
        // peers' are read back together below: one host sync per dimension
        nsel.reserve(2);
        sw.list.reserve(nlast > 0 ? nlast : 1);
        if (SPH_BRD_FUSED) {
          sw.lo_sel = sendflag ? sw.lo : 1.0;  // (no send: an empty slab)
          sw.hi_sel = sendflag ? sw.hi : 0.0;
        } else if (sendflag && nlast > 0) {
          flags.reserve(nlast);
          hipLaunchKernelGGL(k_slab_flags, dim3(blocks(nlast)), dim3(BLK), 0, s, nlast, d,
                             sw.lo, sw.hi, xf.p, flags.p);
          hipcub::CountingInputIterator<int> it(0);
          size_t tb = 0;
          SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, flags.p, sw.list.p,
                                                    nsel.p + dir, nlast, s));
          tmp_reserve(tb);
          SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, it, flags.p, sw.list.p,
                                                    nsel.p + dir, nlast, s));
        } else {
          SPH_HIP_TRY(hipMemsetAsync(nsel.p + dir, 0, sizeof(int), s));
        }
      }
      Swap &a = *pair[0], &b = *pair[1];
      if (SPH_BRD_FUSED) {  // both swaps' selections in three launches
        const int nb = (nlast + BRD_CH - 1) / BRD_CH;
        if (nb == 0) {
          SPH_HIP_TRY(hipMemsetAsync(nsel.p, 0, 2 * sizeof(int), s));
        } else {
          bcnt.reserve(2 * (size_t)nb);
          hipLaunchKernelGGL(k_brd_count, dim3(nb), dim3(BRD_T), 0, s, (const int *)nullptr, d,
                             a.lo_sel, a.hi_sel, b.lo_sel, b.hi_sel, xf.p, bcnt.p, nlast);
          hipLaunchKernelGGL(k_brd_scan, dim3(1), dim3(1024), 0, s, nb, bcnt.p, (int *)nullptr,
                             0, (int *)nullptr, nsel.p);
          hipLaunchKernelGGL(k_brd_lists, dim3(nb), dim3(BRD_T), 0, s, nlast, bcnt.p, d,
                             a.lo_sel, a.hi_sel, b.lo_sel, b.hi_sel, xf.p, a.list.p, b.list.p);
        }
      }
      if (a.remote) {
        int h[4];
        tr->exchange_count2_dev(nsel.p, a.sendproc, a.recvproc, b.sendproc, b.recvproc, s, h);
        a.nsend = h[0];
        b.nsend = h[1];
        a.nrecv = h[2];
        b.nrecv = h[3];
      } else {
        int *const h = h_small;  // (pinned)
        SPH_HIP_TRY(hipMemcpyAsync(h, nsel.p, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
        SPH_HIP_TRY(hipStreamSynchronize(s));
        a.nsend = a.nrecv = h[0];
        b.nsend = b.nrecv = h[1];
      }
      a.firstrecv = nall;
      b.firstrecv = nall + a.nrecv;
      const size_t rec = sizeof(BorderRec);
      const size_t sa = (size_t)a.nsend * rec, sb = (size_t)b.nsend * rec;
      const size_t ra = (size_t)a.nrecv * rec, rb = (size_t)b.nrecv * rec;
      const size_t so = (sa + 255) & ~(size_t)255, ro = (ra + 255) & ~(size_t)255;
      cbs.reserve(std::max<size_t>(so + sb, 1), true, s);
      cbr.reserve(std::max<size_t>(ro + rb, 1), true, s);
      for (int dir = 0; dir < 2; dir++) {
        Swap &sw = *pair[dir];
        if (sw.nsend)
          hipLaunchKernelGGL(k_pack_border, dim3(blocks(sw.nsend)), dim3(BLK), 0, s, sw.nsend,
                             sw.list.p, d, sw.shift, sw.pbc, tr->rank(), nlocal, xf.p, vr.p,
                             en.p, ty.p, gorank.p, goidx.p, gimg.p,
                             (BorderRec *)(cbs.p + (dir ? so : 0)));
      }
      if (a.remote) {
        tr->exchange2(cbs.p, sa, a.sendproc, cbr.p, ra, a.recvproc, cbs.p + so, sb, b.sendproc,
                      cbr.p + ro, rb, b.recvproc, s);
      } else {
        if (ra) SPH_HIP_TRY(hipMemcpyAsync(cbr.p, cbs.p, ra, hipMemcpyDeviceToDevice, s));
        if (rb) SPH_HIP_TRY(hipMemcpyAsync(cbr.p + ro, cbs.p + so, rb, hipMemcpyDeviceToDevice, s));
      }
      const int nr = a.nrecv + b.nrecv;
      if (nr) {
        ensure_atoms((size_t)nall + nr, true);
        const size_t ngn = (size_t)nall + nr - nlocal;
        gorank.reserve(ngn, true, s);
        goidx.reserve(ngn, true, s);
        gimg.reserve(ngn, true, s);
      }
      for (int dir = 0; dir < 2; dir++) {
        Swap &sw = *pair[dir];
        if (sw.nrecv)
          hipLaunchKernelGGL(k_unpack_border, dim3(blocks(sw.nrecv)), dim3(BLK), 0, s,
                             sw.nrecv, sw.firstrecv, nlocal,
                             (const BorderRec *)(cbr.p + (dir ? ro : 0)), xf.p, vr.p, en.p,
                             ty.p, gorank.p, goidx.p, gimg.p);
      }
      if (mp) mpx_swap_pair(a, b);
      nall += nr;
    }
    nghost = nall - nlocal;
    build_direct();
  }

  // Direct forward comm: the per-step halo goes straight from each ghost's owner (its
  // origin, carried through the border records) in ONE exchange, instead of one exchange
  // per dimension with earlier dimensions' ghosts forwarded again (CommBrick's
  // dimension-ordered swaps, comm_brick.cpp:475-530).  Built at every borders: the ghosts
  // are grouped by origin rank (ghost order kept), every rank sends its peers the owned
  // indices it needs from them (counts first), and what it receives becomes its send lists.
  // Ghosts imaging this rank's own atoms are device copies (through the communicator in
  // loopback mode).  The swaps stay for the reverse comm of the setup step and of fix
  // phase_change.  SPH_DIRECT=0 keeps the dimension-ordered forward.
  void build_direct() {
    dr_ok = false;
    if (!direct_env() || mp || !tr) return;
    const int P = tr->size(), me = tr->rank(), ng = nghost;
    // the ghosts grouped by origin rank on the device (a stable radix sort of (rank, ghost)
    // keeps the ghost order within a rank), the per-rank counts the only read-back
    std::vector<int> beg(P + 2, 0);
    dr_byq.reserve(ng > 0 ? ng : 1);
    dr_byg.reserve(ng > 0 ? ng : 1);
    dr_hist.reserve(P + 2);
    if (ng) {
      bkey.reserve(ng);
      bkey2.reserve(ng);
      bidx.reserve(ng);
      bidx2.reserve(ng);
      hipLaunchKernelGGL(k_dr_keys, dim3(blocks(ng)), dim3(BLK), 0, s, ng, P, gorank.p, bkey.p,
                         bidx.p);
      int eb = 1;
      while ((1 << eb) <= P) eb++;
      size_t tb = 0;
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, bkey.p, bkey2.p, bidx.p, bidx2.p, ng, 0, eb, s));
      tmp_reserve(tb);
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, bkey.p, bkey2.p, bidx.p, bidx2.p, ng, 0, eb, s));
      hipLaunchKernelGGL(k_dr_group, dim3(blocks(ng)), dim3(BLK), 0, s, ng, bidx2.p, goidx.p,
                         dr_byq.p, dr_byg.p);
      // beg[r]: the first ghost of rank r (r = 0 .. P + 1; ranks out of range sort as P)
      hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(64 * ((P + 2 + 63) / 64)), 0, s, P + 1,
                         ng, 0, bkey2.p, dr_hist.p);
      SPH_HIP_TRY(hipMemcpyAsync(beg.data(), dr_hist.p, (P + 2) * sizeof(int), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipStreamSynchronize(s));
    }
    SPH_REQUIRE(beg[P + 1] == beg[P], SPH_HIP_ERUNTIME,
                "%d ghosts with an origin rank outside [0,%d)", beg[P + 1] - beg[P], P);
    std::vector<int> scnt(P, 0), rcnt(P, 0);
    for (int r = 0; r < P; r++)
      if (r != me) scnt[r] = beg[r + 1] - beg[r];
    tr->exchange_counts_all(scnt.data(), rcnt.data(), s);  // rcnt[r]: what r needs from me
    dr_peer.clear();
    dr_soff.assign(1, 0);
    dr_roff.assign(1, 0);
    for (int r = 0; r < P; r++) {
      if (r == me && !loopback) continue;
      const size_t nin = beg[r + 1] - beg[r], nout = (r == me) ? nin : (size_t)rcnt[r];
      if (nin == 0 && nout == 0) continue;
      dr_peer.push_back(r);
      dr_roff.push_back(dr_roff.back() + nin);
      dr_soff.push_back(dr_soff.back() + nout);
    }
    const int np = (int)dr_peer.size();
    const size_t S = dr_soff.back(), R = dr_roff.back();
    // the peers' groups are the rank-ordered groups without this rank's own (unless the
    // loopback sends those through the communicator): two device copies
    DBuf<int> &req = dr_req;  // (persistent: no hipMalloc / synchronising hipFree per rebuild)
    req.reserve(R > 0 ? R : 1);
    dr_sidx.reserve(S > 0 ? S : 1);
    dr_rslot.reserve(R > 0 ? R : 1);
    {
      const size_t a = loopback ? (size_t)ng : (size_t)beg[me];
      const size_t b0 = loopback ? (size_t)ng : (size_t)beg[me + 1];
      SPH_REQUIRE(a + (ng - b0) == R, SPH_HIP_ERUNTIME, "direct forward: %zu != %zu", a + (ng - b0), R);
      if (a) {
        SPH_HIP_TRY(hipMemcpyAsync(req.p, dr_byq.p, a * sizeof(int), hipMemcpyDeviceToDevice, s));
        SPH_HIP_TRY(hipMemcpyAsync(dr_rslot.p, dr_byg.p, a * sizeof(int), hipMemcpyDeviceToDevice, s));
      }
      if (ng > (int)b0) {
        SPH_HIP_TRY(hipMemcpyAsync(req.p + a, dr_byq.p + b0, (ng - b0) * sizeof(int), hipMemcpyDeviceToDevice, s));
        SPH_HIP_TRY(hipMemcpyAsync(dr_rslot.p + a, dr_byg.p + b0, (ng - b0) * sizeof(int), hipMemcpyDeviceToDevice, s));
      }
    }
    dr_sb.resize(np);
    dr_rb.resize(np);
    dr_sbytes.resize(np);
    dr_rbytes.resize(np);
    for (int k = 0; k < np; k++) {  // requests out, the peers' requests in (= my send lists)
      dr_sb[k] = req.p + dr_roff[k];
      dr_sbytes[k] = (dr_roff[k + 1] - dr_roff[k]) * sizeof(int);
      dr_rb[k] = dr_sidx.p + dr_soff[k];
      dr_rbytes[k] = (dr_soff[k + 1] - dr_soff[k]) * sizeof(int);
    }
    tr->exchange_multi(np, dr_peer.data(), dr_sb.data(), dr_sbytes.data(), dr_rb.data(),
                       dr_rbytes.data(), s);
    dr_nself = loopback ? 0 : beg[me + 1] - beg[me];
    dr_self.reserve(dr_nself > 0 ? dr_nself : 1);
    if (dr_nself)
      SPH_HIP_TRY(hipMemcpyAsync(dr_self.p, dr_byg.p + beg[me], dr_nself * sizeof(int), hipMemcpyDeviceToDevice, s));
    dr_ok = true;
  }
  // one direct forward of rec-byte records: pack the send lists, one exchange, unpack
  template <class Pack, class Unpack, class Self>
  void forward_direct(size_t rec, Pack pack, Unpack unpack, Self self) {
    const int np = (int)dr_peer.size();
    const size_t S = dr_soff.back(), R = dr_roff.back();
    cbs.reserve(std::max<size_t>(S * rec, 1));
    cbr.reserve(std::max<size_t>(R * rec, 1));
    if (S) pack((int)S, cbs.p);
    for (int k = 0; k < np; k++) {
      dr_sb[k] = cbs.p + dr_soff[k] * rec;
      dr_sbytes[k] = (dr_soff[k + 1] - dr_soff[k]) * rec;
      dr_rb[k] = cbr.p + dr_roff[k] * rec;
      dr_rbytes[k] = (dr_roff[k + 1] - dr_roff[k]) * rec;
    }
    tr->exchange_multi(np, dr_peer.data(), dr_sb.data(), dr_sbytes.data(), dr_rb.data(),
                       dr_rbytes.data(), s);
    if (R) unpack((int)R, cbr.p);
    if (dr_nself) self();
  }

  // the extra multiphase fields of a dimension's two swaps (pack_border_vel / pack_comm_vel
  // of atom_vec_meso_multiphase.cpp): lists -> the peers -> firstrecv..
  void mpx_swap_pair(Swap &a, Swap &b) {
    const size_t rec = MPX * sizeof(double);
    const size_t sa = (size_t)a.nsend * rec, sb = (size_t)b.nsend * rec;
    const size_t ra = (size_t)a.nrecv * rec, rb = (size_t)b.nrecv * rec;
    const size_t so = (sa + 255) & ~(size_t)255, ro = (ra + 255) & ~(size_t)255;
    cbs.reserve(std::max<size_t>(so + sb, 1), true, s);
    cbr.reserve(std::max<size_t>(ro + rb, 1), true, s);
    if (a.nsend)
      hipLaunchKernelGGL(k_mpx_pack, dim3(blocks(a.nsend)), dim3(BLK), 0, s, a.nsend, a.list.p,
                         vel.p, rm.p, cvv.p, cg.p, (double *)cbs.p);
    if (b.nsend)
      hipLaunchKernelGGL(k_mpx_pack, dim3(blocks(b.nsend)), dim3(BLK), 0, s, b.nsend, b.list.p,
                         vel.p, rm.p, cvv.p, cg.p, (double *)(cbs.p + so));
    if (a.remote) {
      tr->exchange2(cbs.p, sa, a.sendproc, cbr.p, ra, a.recvproc, cbs.p + so, sb, b.sendproc,
                    cbr.p + ro, rb, b.recvproc, s);
    } else {
      if (ra) SPH_HIP_TRY(hipMemcpyAsync(cbr.p, cbs.p, ra, hipMemcpyDeviceToDevice, s));
      if (rb) SPH_HIP_TRY(hipMemcpyAsync(cbr.p + ro, cbs.p + so, rb, hipMemcpyDeviceToDevice, s));
    }
    if (a.nrecv)
      hipLaunchKernelGGL(k_mpx_unpack, dim3(blocks(a.nrecv)), dim3(BLK), 0, s, a.nrecv,
                         (const int *)nullptr, a.firstrecv, (const double *)cbr.p, vel.p, rm.p,
                         cvv.p, cg.p);
    if (b.nrecv)
      hipLaunchKernelGGL(k_mpx_unpack, dim3(blocks(b.nrecv)), dim3(BLK), 0, s, b.nrecv,
                         (const int *)nullptr, b.firstrecv, (const double *)(cbr.p + ro), vel.p,
                         rm.p, cvv.p, cg.p);
  }

  // Per-step forward traffic, one dimension at a time: the two swaps of a dimension send
  // from the same atoms (owned + earlier dimensions' ghosts, see borders_multi) and
  // receive into disjoint ghost ranges, so both are packed into one buffer and moved as
  // ONE exchange (one RCCL group over xGMI per dimension instead of one per swap).
  template <class Pack, class Unpack>
  void forward_dims(size_t rec, Pack pack, Unpack unpack) {
    for (int k = 0; k + 1 < nswap; k += 2) {
      Swap &a = swaps[k], &b = swaps[k + 1];
      const size_t sa = (size_t)a.nsend * rec, sb = (size_t)b.nsend * rec;
      const size_t ra = (size_t)a.nrecv * rec, rb = (size_t)b.nrecv * rec;
      const size_t so = (sa + 255) & ~(size_t)255, ro = (ra + 255) & ~(size_t)255;
      cbs.reserve(std::max<size_t>(so + sb, 1), true, s);
      cbr.reserve(std::max<size_t>(ro + rb, 1), true, s);
      if (a.nsend) pack(a, cbs.p);
      if (b.nsend) pack(b, cbs.p + so);
      if (a.remote) {
        tr->exchange2(cbs.p, sa, a.sendproc, cbr.p, ra, a.recvproc, cbs.p + so, sb, b.sendproc,
                      cbr.p + ro, rb, b.recvproc, s);
      } else {  // this brick is its own neighbour along this dimension (periodic self swap)
        if (ra) SPH_HIP_TRY(hipMemcpyAsync(cbr.p, cbs.p, ra, hipMemcpyDeviceToDevice, s));
        if (rb) SPH_HIP_TRY(hipMemcpyAsync(cbr.p + ro, cbs.p + so, rb, hipMemcpyDeviceToDevice, s));
      }
      if (a.nrecv) unpack(a, cbr.p);
      if (b.nrecv) unpack(b, cbr.p + ro);
    }
  }

  // Comm::forward_comm (x, vest, rho, e)
  void forward_multi() {
    if (dr_ok) {
      forward_direct(
          9 * sizeof(double),
          [&](int n, unsigned char *buf) {
            hipLaunchKernelGGL(k_pack_direct, dim3(blocks(n)), dim3(BLK), 0, s, n, dr_sidx.p,
                               xf.p, vr.p, en.p, (double *)buf);
          },
          [&](int n, unsigned char *buf) {
            hipLaunchKernelGGL(k_unpack_direct, dim3(blocks(n)), dim3(BLK), 0, s, n,
                               dr_rslot.p, nlocal, box, gimg.p, (const double *)buf, xf.p, vr.p,
                               en.p);
          },
          [&] {
            hipLaunchKernelGGL(k_forward_self, dim3(blocks(dr_nself)), dim3(BLK), 0, s,
                               dr_nself, dr_self.p, nlocal, box, goidx.p, gimg.p, xf.p, vr.p,
                               en.p);
          });
      return;
    }
    forward_dims(
        9 * sizeof(double),
        [&](Swap &sw, unsigned char *buf) {
          hipLaunchKernelGGL(k_pack_forward, dim3(blocks(sw.nsend)), dim3(BLK), 0, s, sw.nsend,
                             sw.list.p, sw.dim, sw.shift, xf.p, vr.p, en.p, (double *)buf);
        },
        [&](Swap &sw, unsigned char *buf) {
          hipLaunchKernelGGL(k_unpack_forward, dim3(blocks(sw.nrecv)), dim3(BLK), 0, s,
                             sw.nrecv, sw.firstrecv, (const double *)buf, xf.p, vr.p, en.p);
        });
    if (mp)
      for (int k = 0; k + 1 < nswap; k += 2) mpx_swap_pair(swaps[k], swaps[k + 1]);
  }

  // comm->reverse_comm_fix of one per-atom double (fix phase_change's dmass)
  void reverse1(double *a) {
    if (!multi()) {
      if (nghost)
        hipLaunchKernelGGL(k_reverse1, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost, nlocal,
                           gowner.p, a);
      return;
    }
    for (int k = nswap - 1; k >= 0; k--) {
      Swap &sw = swaps[k];
      cbs.reserve((size_t)(sw.nrecv > 0 ? sw.nrecv : 1) * sizeof(double), true, s);
      cbr.reserve((size_t)(sw.nsend > 0 ? sw.nsend : 1) * sizeof(double), true, s);
      if (sw.nrecv)
        hipLaunchKernelGGL(k_pack_rev1, dim3(blocks(sw.nrecv)), dim3(BLK), 0, s, sw.nrecv,
                           sw.firstrecv, a, (double *)cbs.p);
      swap_move(sw.remote, (size_t)sw.nrecv * sizeof(double), sw.recvproc,
                (size_t)sw.nsend * sizeof(double), sw.sendproc);
      if (sw.nsend)
        hipLaunchKernelGGL(k_unpack_rev1, dim3(blocks(sw.nsend)), dim3(BLK), 0, s, sw.nsend,
                           sw.list.p, (const double *)cbr.p, a);
    }
  }

  // comm->forward_comm_pair of sph/rhosum: rho (+ the EOS term)
  void forward_rho_multi() {
    if (dr_ok) {
      forward_direct(
          sizeof(double2),
          [&](int n, unsigned char *buf) {
            hipLaunchKernelGGL(k_pack_rho, dim3(blocks(n)), dim3(BLK), 0, s, n, dr_sidx.p, xf.p,
                               vr.p, (double2 *)buf);
          },
          [&](int n, unsigned char *buf) {
            hipLaunchKernelGGL(k_unpack_rho_direct, dim3(blocks(n)), dim3(BLK), 0, s, n,
                               dr_rslot.p, nlocal, (const double2 *)buf, xf.p, vr.p);
          },
          [&] {
            hipLaunchKernelGGL(k_forward_rho_self, dim3(blocks(dr_nself)), dim3(BLK), 0, s,
                               dr_nself, dr_self.p, nlocal, goidx.p, xf.p, vr.p);
          });
      return;
    }
    forward_dims(
        sizeof(double2),
        [&](Swap &sw, unsigned char *buf) {
          hipLaunchKernelGGL(k_pack_rho, dim3(blocks(sw.nsend)), dim3(BLK), 0, s, sw.nsend,
                             sw.list.p, xf.p, vr.p, (double2 *)buf);
        },
        [&](Swap &sw, unsigned char *buf) {
          hipLaunchKernelGGL(k_unpack_rho, dim3(blocks(sw.nrecv)), dim3(BLK), 0, s, sw.nrecv,
                             sw.firstrecv, (const double2 *)buf, xf.p, vr.p);
        });
  }

  // Comm::reverse_comm (f, drho, de): swaps in reverse order, ghosts back to senders
  void reverse_multi() {
    for (int k = nswap - 1; k >= 0; k--) {
      Swap &sw = swaps[k];
      cbs.reserve((size_t)(sw.nrecv > 0 ? sw.nrecv : 1) * 5 * sizeof(double), true, s);
      cbr.reserve((size_t)(sw.nsend > 0 ? sw.nsend : 1) * 5 * sizeof(double), true, s);
      if (sw.nrecv)
        hipLaunchKernelGGL(k_pack_reverse, dim3(blocks(sw.nrecv)), dim3(BLK), 0, s, sw.nrecv,
                           sw.firstrecv, fo.p, de.p, (double *)cbs.p);
      swap_move(sw.remote, (size_t)sw.nrecv * 5 * sizeof(double), sw.recvproc,
                (size_t)sw.nsend * 5 * sizeof(double), sw.sendproc);
      if (sw.nsend)
        hipLaunchKernelGGL(k_unpack_reverse, dim3(blocks(sw.nsend)), dim3(BLK), 0, s, sw.nsend,
                           sw.list.p, (const double *)cbr.p, fo.p, de.p);
    }
  }

  // CommBrick::exchange (comm_brick.cpp:573-680): atoms that left the brick along each
  // split dimension go to the face neighbours, which keep the ones inside their slab
  void exchange_multi() {
    for (int d = 0; d < cfg.dim; d++) {
      if (pg[d] == 1) continue;
      const int n = nlocal;
      flags.reserve(n > 0 ? n : 1);
      flag2.reserve(n > 0 ? n : 1);
      if (n)
        hipLaunchKernelGGL(k_flag_leave, dim3(blocks(n)), dim3(BLK), 0, s, n, d, sublo[d],
                           subhi[d], xf.p, flags.p, flag2.p);
      const int nl = select_flagged(flags.p, n, sel);
      migrations += nl;
      const int nst = select_flagged(flag2.p, n, sel2);
      if (pc && nl) hole_fill(n, nl, nst);  // (leavers put in send order, lidx renumbered)
      cbs.reserve((size_t)(nl > 0 ? nl : 1) * sizeof(MigRec));
      if (nl)
        hipLaunchKernelGGL(k_pack_mig, dim3(blocks(nl)), dim3(BLK), 0, s, nl, sel.p, xf.p,
                           vr.p, vel.p, en.p, ty.p, tag.p, (MigRec *)cbs.p);
      if (mp && nl) {  // the leavers' extra fields
        xbuf.reserve((size_t)MPX * nl, false, s);
        hipLaunchKernelGGL(k_mpx_pack, dim3(blocks(nl)), dim3(BLK), 0, s, nl, sel.p, vel.p,
                           rm.p, cvv.p, cg.p, xbuf.p);
      }
      if (nl) {  // compact the staying atoms to the front (order kept)
        DBuf<unsigned char> keep;
        keep.reserve((size_t)(nst > 0 ? nst : 1) * sizeof(MigRec));
        // (every record is packed from the old rows before any row is rewritten: the extra
        // fields' copy rewrites vel, which the records carry whole)
        if (nst)
          hipLaunchKernelGGL(k_pack_mig, dim3(blocks(nst)), dim3(BLK), 0, s, nst, sel2.p, xf.p,
                             vr.p, vel.p, en.p, ty.p, tag.p, (MigRec *)keep.p);
        mpx_copy(nst, sel2.p, 0, xbuf2);
        if (nst)
          hipLaunchKernelGGL(k_gather_mig, dim3(blocks(nst)), dim3(BLK), 0, s, nst,
                             (const int *)nullptr, (const MigRec *)keep.p, 0, xf.p, vr.p,
                             vel.p, en.p, ty.p, tag.p);
        SPH_HIP_TRY(hipStreamSynchronize(s));
        keep.release();
      }
      nlocal = nst;
      // pg == 2: both neighbours are the same brick, one exchange; otherwise send the
      // leavers to both and let each keep its own
      const int nex = (pg[d] == 2) ? 1 : 2;
      for (int x = 0; x < nex; x++) {
        const int dest = procneigh[d][x], src = procneigh[d][1 - x];
        const int nr = tr->exchange_count(nl, dest, src, s);
        cbr.reserve((size_t)(nr > 0 ? nr : 1) * sizeof(MigRec));
        tr->exchange(cbs.p, (size_t)nl * sizeof(MigRec), dest, cbr.p, (size_t)nr * sizeof(MigRec),
                     src, s);
        if (mp) {
          xbuf2.reserve((size_t)MPX * (nr > 0 ? nr : 1), false, s);
          tr->exchange((unsigned char *)xbuf.p, (size_t)nl * MPX * sizeof(double), dest,
                       (unsigned char *)xbuf2.p, (size_t)nr * MPX * sizeof(double), src, s);
        }
        if (nr == 0) continue;
        flags.reserve(nr);
        hipLaunchKernelGGL(k_flag_mine, dim3(blocks(nr)), dim3(BLK), 0, s, nr, d, sublo[d],
                           subhi[d], (const MigRec *)cbr.p, flags.p);
        const int nm = select_flagged(flags.p, nr, sel2);
        if (nm == 0) continue;
        ensure_atoms((size_t)nlocal + nm, true);
        vel.reserve((size_t)nlocal + nm, true, s);
        tag.reserve((size_t)nlocal + nm, true, s);
        hipLaunchKernelGGL(k_gather_mig, dim3(blocks(nm)), dim3(BLK), 0, s, nm, sel2.p,
                           (const MigRec *)cbr.p, nlocal, xf.p, vr.p, vel.p, en.p, ty.p, tag.p);
        if (pc) {  // unpack_exchange appends in buffer order
          lidx.reserve((size_t)nlocal + nm, true, s);
          hipLaunchKernelGGL(k_lidx_iota, dim3(blocks(nm)), dim3(BLK), 0, s, nm, nlocal,
                             lidx.p + nlocal);
        }
        if (mp)
          hipLaunchKernelGGL(k_mpx_unpack, dim3(blocks(nm)), dim3(BLK), 0, s, nm, sel2.p,
                             nlocal, (const double *)xbuf2.p, vel.p, rm.p, cvv.p, cg.p);
        nlocal += nm;
      }
    }
    fo.reserve(nlocal > 0 ? nlocal : 1, true, s);
    de.reserve(nlocal > 0 ? nlocal : 1, true, s);
  }

  // CommBrick::exchange's scan of one dimension (comm_brick.cpp:620-632) on the LAMMPS
  // indices: a departing atom's slot takes the last atom, which is examined next.  The n - nst
  // leavers (sel) go into the buffer in that order -- the receivers append them as LAMMPS
  // does -- and the stayers' indices are compacted along sel2, the tail atoms that moved
  // into holes renumbered.  Host work over the leavers only (the tail atom at LAMMPS index
  // m is always the one that started there: moves only go from the tail into lower holes).
  void hole_fill(int n, int nl, int nst) {
    std::vector<int> hl(nl), hr(nl);
    lidx_tab.reserve(nl);
    hipLaunchKernelGGL(k_lidx_take, dim3(blocks(nl)), dim3(BLK), 0, s, nl, sel.p, lidx.p, 0,
                       (const int *)nullptr, lidx_tab.p);
    SPH_HIP_TRY(hipMemcpyAsync(hl.data(), lidx_tab.p, nl * sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipMemcpyAsync(hr.data(), sel.p, nl * sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    std::vector<int> ord(nl);
    for (int k = 0; k < nl; k++) ord[k] = k;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return hl[a] < hl[b]; });
    if ((int)h_leave.size() < n) h_leave.resize(n, 0);
    for (int k = 0; k < nl; k++) h_leave[hl[k]] = 1;
    std::vector<int> sent, tab(nl, -1);
    sent.reserve(nl);
    int m = n;
    for (int q = 0; q < nl; q++) {
      const int p = hl[ord[q]];  // the leavers in ascending LAMMPS index
      if (p >= m) break;         // (already sent from the tail)
      sent.push_back(p);
      for (;;) {
        m--;
        if (m == p) break;  // the hole was the last slot
        if (h_leave[m]) {   // the tail atom leaves too: examined in the hole, sent
          sent.push_back(m);
          continue;
        }
        tab[m - nst] = p;
        break;
      }
    }
    for (int k = 0; k < nl; k++) h_leave[hl[k]] = 0;
    SPH_REQUIRE((int)sent.size() == nl && m == nst, SPH_HIP_ERUNTIME,
                "exchange: hole fill sent %zu of %d atoms", sent.size(), nl);
    std::vector<int> rows(nl);  // sel in send order
    for (int k = 0; k < nl; k++) {
      const int v = sent[k];
      const auto it = std::lower_bound(ord.begin(), ord.end(), v,
                                       [&](int a, int val) { return hl[a] < val; });
      rows[k] = hr[*it];
    }
    SPH_HIP_TRY(hipMemcpyAsync(sel.p, rows.data(), nl * sizeof(int), hipMemcpyHostToDevice, s));
    SPH_HIP_TRY(hipMemcpyAsync(lidx_tab.p, tab.data(), nl * sizeof(int), hipMemcpyHostToDevice, s));
    if (nst) {
      lidx2.reserve_exact(lidx.cap);
      hipLaunchKernelGGL(k_lidx_take, dim3(blocks(nst)), dim3(BLK), 0, s, nst, sel2.p, lidx.p,
                         nst, lidx_tab.p, lidx2.p);
      SPH_HIP_TRY(hipMemcpyAsync(lidx.p, lidx2.p, nst * sizeof(int), hipMemcpyDeviceToDevice, s));
    }
    SPH_HIP_TRY(hipStreamSynchronize(s));  // (host vectors)
  }

  // Atom::sort (atom.cpp:1555-1654) on the LAMMPS indices: the bins of setup_sort_bins
  // (:1660-1726) over this brick's sub-box, atoms listed bin by bin and in their current order
  // within a bin; one bin = no sort.  nextsort as atom.cpp:1561.
  void atom_sort() {
    nextsort = (step / sortfreq) * sortfreq + sortfreq;
    const double bs = sort_binsize > 0.0 ? sort_binsize : 0.5 * cutneighmax;
    const double bininv = 1.0 / bs;
    SortBins b{};
    double nbins = 1.0;
    for (int d = 0; d < 3; d++) {
      const double ext = subhi[d] - sublo[d];
      int m = (int)(ext * bininv);
      if (d == 2 && cfg.dim == 2) m = 1;
      if (m == 0) m = 1;
      b.lo[d] = sublo[d];
      b.nb[d] = m;
      b.inv[d] = m / ext;
      nbins *= m;
    }
    SPH_REQUIRE(nbins <= 2147483647.0, SPH_HIP_EINVAL, "Too many atom sorting bins");
    const int n = nlocal;
    if (nbins == 1.0 || n == 0) return;
    skey.reserve(n);
    skey2.reserve(n);
    srow.reserve(n);
    srow2.reserve(n);
    hipLaunchKernelGGL(k_lidx_sortkeys, dim3(blocks(n)), dim3(BLK), 0, s, n, b, xf.p, lidx.p,
                       skey.p, srow.p);
    int hb = 32;
    while ((double)(1ll << (hb - 32)) < nbins) hb++;
    size_t tb = 0;
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, skey.p, skey2.p, srow.p, srow2.p,
                                                   n, 0, hb, s));
    tmp_reserve(tb);
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, skey.p, skey2.p, srow.p, srow2.p,
                                                   n, 0, hb, s));
    hipLaunchKernelGGL(k_lidx_rank, dim3(blocks(n)), dim3(BLK), 0, s, n, srow2.p, lidx.p);
  }

  // the LAMMPS indices from the tags: read order (tag order) -- set_atoms, read_restart
  void lidx_from_tags() {
    const int n = nlocal;
    lidx.reserve(n > 0 ? n : 1);
    lidx_valid = true;
    if (n == 0) return;
    skey.reserve(n);
    skey2.reserve(n);
    srow.reserve(n);
    srow2.reserve(n);
    hipLaunchKernelGGL(k_lidx_tagkeys, dim3(blocks(n)), dim3(BLK), 0, s, n, tag.p, skey.p,
                       srow.p);
    size_t tb = 0;
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, skey.p, skey2.p, srow.p, srow2.p,
                                                   n, 0, 32, s));
    tmp_reserve(tb);
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, skey.p, skey2.p, srow.p, srow2.p,
                                                   n, 0, 32, s));
    hipLaunchKernelGGL(k_lidx_rank, dim3(blocks(n)), dim3(BLK), 0, s, n, srow2.p, lidx.p);
  }

  // One brick: CommBrick::borders' self swaps (comm_brick.cpp:696-864) with every count kept
  // on the device -- each swap's selection size, and where its ghosts go, is read by the next
  // kernels from device words (gnall), so the swaps run back to back with ONE host read at
  // the end.  The ghost arrays are sized ahead from the last borders' ghost count (or the
  // box geometry); a borders that would outgrow them is redone with twice the room.
  void borders() {
    if (multi()) {
      borders_multi();
      return;
    }
    const int ndim = cfg.dim;
    int nsw = 0;
    for (int d = 0; d < ndim; d++)
      if (cfg.periodic[d]) nsw += 2;
    if (gcap_hint <= 0) {  // the ghost shell's share of the sub-box, with room
      double in = 1.0, out = 1.0;
      for (int d = 0; d < ndim; d++) {
        const double ext = std::max(subhi[d] - sublo[d], 1e-300);
        in *= ext;
        out *= ext + (cfg.periodic[d] ? 2.0 * cutghost : 0.0);
      }
      gcap_hint = (int)std::min(1.5 * (out / in - 1.0) * nlocal + 4096.0, 2.0e9 - nlocal);
    }
    gnall.reserve(nsw + 2);
    nsel.reserve(nsw + 1);
    for (;;) {
      const int gcap = gcap_hint, cap = nlocal + gcap;
      ensure_atoms((size_t)cap, true);
      gowner.reserve(gcap, true, s);
      gimg.reserve(gcap, true, s);
      if (pc) gsrc.reserve(gcap, true, s);
      flags.reserve(cap);
      sel.reserve(cap);
      h_small[14] = nlocal;  // (pinned; the read-back below lands in words 0 .. nsw + 1)
      h_small[15] = 0;       // the overflow word
      SPH_HIP_TRY(hipMemcpyAsync(gnall.p, h_small + 14, sizeof(int), hipMemcpyHostToDevice, s));
      SPH_HIP_TRY(hipMemcpyAsync(gnall.p + nsw + 1, h_small + 15, sizeof(int),
                                 hipMemcpyHostToDevice, s));
      int w = 0;
#if SPH_BRD_FUSED
      // a dimension's two swaps in three launches (k_brd_count / scan / scatter)
      for (int d = 0; d < ndim; d++) {
        if (!cfg.periodic[d]) continue;  // sendneed = 0 across a non-periodic boundary
        const double lo0 = -1.0e20, hi0 = sublo[d] + cutghost;
        const double lo1 = subhi[d] - cutghost, hi1 = 1.0e20;
        const int nb = (cap + BRD_CH - 1) / BRD_CH;
        bcnt.reserve(2 * (size_t)nb);
        hipLaunchKernelGGL(k_brd_count, dim3(nb), dim3(BRD_T), 0, s, gnall.p + w, d, lo0, hi0,
                           lo1, hi1, xf.p, bcnt.p);
        hipLaunchKernelGGL(k_brd_scan, dim3(1), dim3(1024), 0, s, nb, bcnt.p, gnall.p + w, cap,
                           gnall.p + nsw + 1);
        hipLaunchKernelGGL(k_brd_scatter, dim3(nb), dim3(BRD_T), 0, s, gnall.p + w, bcnt.p, cap,
                           nlocal, d, lo0, hi0, lo1, hi1, box.prd[d], xf.p, vr.p, en.p, ty.p,
                           gowner.p, gimg.p, pc ? gsrc.p : (int *)nullptr,
                           mp ? vel.p : (double4 *)nullptr, mp ? rm.p : (double *)nullptr,
                           mp ? cvv.p : (double *)nullptr, mp ? cg.p : (double4 *)nullptr);
        w += 2;
      }
#else
      for (int d = 0; d < ndim; d++) {
        if (!cfg.periodic[d]) continue;  // sendneed = 0 across a non-periodic boundary
        const int *const nlast = gnall.p + w;  // both swaps scan the atoms before this dim
        for (int ineed = 0; ineed < 2; ineed++, w++) {
          double lo, hi;
          int pbc;
          if (ineed == 0) {
            lo = -1.0e20;
            hi = sublo[d] + cutghost;
            pbc = 1;
          } else {
            lo = subhi[d] - cutghost;
            hi = 1.0e20;
            pbc = -1;
          }
          const double shift = pbc * box.prd[d];
          hipLaunchKernelGGL(k_slab_flags_dev, dim3(blocks(cap)), dim3(BLK), 0, s, cap, nlast,
                             d, lo, hi, xf.p, flags.p);
          hipcub::CountingInputIterator<int> it(0);
          size_t tb = 0;
          SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, flags.p, sel.p, nsel.p + w,
                                                    cap, s));
          tmp_reserve(tb);
          SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, it, flags.p, sel.p, nsel.p + w,
                                                    cap, s));
          hipLaunchKernelGGL(k_append_ghosts_dev, dim3(blocks(gcap)), dim3(BLK), 0, s, gcap,
                             nsel.p + w, sel.p, nlocal, gnall.p + w, cap, d, pbc, shift, xf.p,
                             vr.p, en.p, ty.p, gowner.p, gimg.p, pc ? gsrc.p : (int *)nullptr,
                             mp ? vel.p : (double4 *)nullptr, mp ? rm.p : (double *)nullptr,
                             mp ? cvv.p : (double *)nullptr, mp ? cg.p : (double4 *)nullptr,
                             gnall.p + nsw + 1);
        }
      }
#endif
      SPH_HIP_TRY(hipMemcpyAsync(h_small, gnall.p, (nsw + 2) * sizeof(int),
                                 hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipStreamSynchronize(s));
      if (h_small[nsw + 1] == 0) break;
      SPH_REQUIRE(gcap < 1000000000, SPH_HIP_EOVERFLOW, "ghost count exceeds 2^30");
      gcap_hint = 2 * gcap;
    }
    gswap_first.clear();
    for (int w = 0; w <= nsw; w++) gswap_first.push_back(h_small[w] - nlocal);
    nghost = h_small[nsw] - nlocal;
    // next time: this count with room (atoms drift between rebuilds)
    gcap_hint = std::max(gcap_hint, nghost + nghost / 8 + 4096);
  }

  // LAMMPS' index order of this brick's ghosts (one process): CommBrick::borders appends each
  // swap's ghosts in the order of the atoms it scans (comm_brick.cpp:741-800), i.e. by the
  // LAMMPS index of their source -- tag - 1 for an owned atom (local order = tag order on one
  // process without sorting), nlocal + slot for a ghost of an earlier swap.  Our swaps hold
  // the same ghosts in our own (Hilbert) order; sort each swap by that key: grank[g] = the
  // ghost's LAMMPS slot.  Used only when a created atom may overwrite a slot a candidate reads.
  void pc_ghost_slots() {
    pc_grank.reserve(nghost > 0 ? nghost : 1);
    for (size_t w = 0; w + 1 < gswap_first.size(); w++) {
      const int first = gswap_first[w], ns = gswap_first[w + 1] - first;
      if (ns == 0) continue;
      pc_key.reserve(2 * (size_t)ns);
      pc_val.reserve(2 * (size_t)ns);
      hipLaunchKernelGGL(k_pc_swapkeys, dim3(blocks(ns)), dim3(BLK), 0, s, ns, first, gsrc.p,
                         nlocal, lidx.p, pc_grank.p, pc_key.p, pc_val.p);
      size_t tb = 0;
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, pc_key.p, pc_key.p + ns,
                                                     pc_val.p, pc_val.p + ns, ns, 0, 32, s));
      tmp_reserve(tb);
      SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, pc_key.p, pc_key.p + ns,
                                                     pc_val.p, pc_val.p + ns, ns, 0, 32, s));
      hipLaunchKernelGGL(k_pc_swaprank, dim3(blocks(ns)), dim3(BLK), 0, s, ns, first,
                         pc_val.p + ns, pc_grank.p);
    }
  }

  // Bricks: the same slot order, but a swap's ghosts come from another rank, whose scan
  // order (owned atoms in tag order, then its ghosts in slot order) only it knows -- each
  // dimension's two swaps send that key along the send lists (one exchange), the receiver
  // sorts each swap by it.  Collective over the ranks (every rank calls it).
  void pc_ghost_slots_multi() {
    pc_grank.reserve(nghost > 0 ? nghost : 1);
    for (int k = 0; k + 1 < nswap; k += 2) {
      Swap &a = swaps[k], &b = swaps[k + 1];
      const size_t sa = (size_t)a.nsend * 4, sb = (size_t)b.nsend * 4;
      const size_t ra = (size_t)a.nrecv * 4, rb = (size_t)b.nrecv * 4;
      const size_t so = (sa + 255) & ~(size_t)255, ro = (ra + 255) & ~(size_t)255;
      cbs.reserve(std::max<size_t>(so + sb, 1), true, s);
      cbr.reserve(std::max<size_t>(ro + rb, 1), true, s);
      if (a.nsend)
        hipLaunchKernelGGL(k_pc_sendkeys, dim3(blocks(a.nsend)), dim3(BLK), 0, s, a.nsend,
                           a.list.p, nlocal, lidx.p, pc_grank.p, (int *)cbs.p);
      if (b.nsend)
        hipLaunchKernelGGL(k_pc_sendkeys, dim3(blocks(b.nsend)), dim3(BLK), 0, s, b.nsend,
                           b.list.p, nlocal, lidx.p, pc_grank.p, (int *)(cbs.p + so));
      if (a.remote) {
        tr->exchange2(cbs.p, sa, a.sendproc, cbr.p, ra, a.recvproc, cbs.p + so, sb, b.sendproc,
                      cbr.p + ro, rb, b.recvproc, s);
      } else {
        if (ra) SPH_HIP_TRY(hipMemcpyAsync(cbr.p, cbs.p, ra, hipMemcpyDeviceToDevice, s));
        if (rb) SPH_HIP_TRY(hipMemcpyAsync(cbr.p + ro, cbs.p + so, rb, hipMemcpyDeviceToDevice, s));
      }
      for (int dir = 0; dir < 2; dir++) {
        Swap &sw = dir ? b : a;
        const int ns = sw.nrecv, first = sw.firstrecv - nlocal;
        if (ns == 0) continue;
        pc_key.reserve(2 * (size_t)ns);
        pc_val.reserve(2 * (size_t)ns);
        hipLaunchKernelGGL(k_pc_keys_in, dim3(blocks(ns)), dim3(BLK), 0, s, ns,
                           (const int *)(cbr.p + (dir ? ro : 0)), pc_key.p, pc_val.p);
        size_t tb = 0;
        SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, pc_key.p, pc_key.p + ns,
                                                       pc_val.p, pc_val.p + ns, ns, 0, 31, s));
        tmp_reserve(tb);
        SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, pc_key.p, pc_key.p + ns,
                                                       pc_val.p, pc_val.p + ns, ns, 0, 31, s));
        hipLaunchKernelGGL(k_pc_swaprank, dim3(blocks(ns)), dim3(BLK), 0, s, ns, first,
                           pc_val.p + ns, pc_grank.p);
      }
    }
  }

  void setup_bins_geometry() {
    for (int k = 0; k < 3; k++) {
      double lo = sublo[k], hi = subhi[k];
      if (k < cfg.dim) {
        lo -= cutghost;
        hi += cutghost;
        const double ext = hi - lo;
        int nb = (int)(ext / cutneighmax);
        if (nb < 1) nb = 1;
        if (nb > 4096) nb = 4096;
        bn.lo[k] = lo;
        bn.nb[k] = nb;
        bn.inv[k] = nb / ext;
      } else {
        bn.lo[k] = lo;
        bn.nb[k] = 1;
        bn.inv[k] = 0.0;
      }
    }
    nbins = bn.nb[0] * bn.nb[1] * bn.nb[2];
    // half-size bins of the list builders (k_neigh3, k_blk_neigh: reach 2 in y and z; the
    // x-range of a bin-row is cut to the sphere per row, at the bins' x resolution).  The
    // multiphase engine's per-step list fill (k_neigh3 with the fused rhosum, instruction-
    // bound) takes bins three times finer in x: ~19 % fewer candidates per row, C5 11.54 ->
    // 11.17 ms per step (profiles/r06/qbx/); the block build of C2 gained nothing measurable
    const int fx = mp ? 3 : 1;
    for (int k = 0; k < 3; k++) {
      const double ext = bn.nb[k] > 0 && bn.inv[k] > 0.0 ? bn.nb[k] / bn.inv[k] : 0.0;
      int nb = 1;
      if (k < cfg.dim) {
        nb = (int)(ext / (0.5 * cutneighmax / (k == 0 ? fx : 1)));
        if (nb < 1) nb = 1;
        if (nb > 8192) nb = 8192;
      }
      qb.lo[k] = bn.lo[k];
      qb.nb[k] = nb;
      qb.inv[k] = (k < cfg.dim) ? nb / ext : 0.0;
      qb.size[k] = (k < cfg.dim) ? ext / nb : 1.0;
    }
    qb.cutmaxsq = cutneighmax * cutneighmax;
    nqbins = qb.nb[0] * qb.nb[1] * qb.nb[2];
  }

  // bin-ordered copy of all atoms over the half-size bins (xb, tb, qbeg)
  void bin_q() {
    const int nall = nlocal + nghost;
    Bins b;
    for (int k = 0; k < 3; k++) {
      b.lo[k] = qb.lo[k];
      b.inv[k] = qb.inv[k];
      b.nb[k] = qb.nb[k];
    }
    bkey.reserve(nall);
    bkey2.reserve(nall);
    bidx.reserve(nall);
    bidx2.reserve(nall);
    qbeg.reserve(nqbins + 1);
    xb.reserve(nall);
    tb.reserve(nall);
    // (mp: k_bin_copy packs the type into xb.w above bit 28, the list entries' MP_NMASK)
    SPH_REQUIRE(!mp || (long long)nall < MP_MAXALL, SPH_HIP_EOVERFLOW,
                "multiphase lists index at most 2^28 atoms per rank (%d)", nall);
    hipLaunchKernelGGL(k_bin_keys, dim3(blocks(nall)), dim3(BLK), 0, s, nall, 0, b, xf.p,
                       bkey.p, bidx.p, 0);
    int endbit = 1;
    while ((1u << endbit) < (unsigned)nqbins && endbit < 32) endbit++;
    size_t tbytes = 0;
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tbytes, bkey.p, bkey2.p, bidx.p, bidx2.p, nall, 0, endbit, s));
    tmp_reserve(tbytes);
    SPH_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tbytes, bkey.p, bkey2.p, bidx.p, bidx2.p, nall, 0, endbit, s));
    hipLaunchKernelGGL(k_lower_bound, dim3(blocks(nqbins + 1)), dim3(BLK), 0, s, nqbins, nall,
                       0, bkey2.p, qbeg.p);
    xpos.reserve(nall);
    hipLaunchKernelGGL(k_bin_copy, dim3(blocks(nall)), dim3(BLK), 0, s, nall, bidx2.p, xf.p,
                       ty.p, xb.p, tb.p, xpos.p, mp ? 1 : 0);
  }
  // Global-index full list (k_neigh3, Neighbor::full_bin membership) of the owned rows at
  // positions xi (default: the current ones, as binned by bin_q): CSR (count pass, scan,
  // fill pass) or, when `csr` is false and an earlier build sized the rows, one fill pass
  // into fixed-stride rows (ccnt = row counts; `strided` records which).
  void list_q(bool csr, const double4 *xi = nullptr) {
    const int n = nlocal, nall = nlocal + nghost;
    const double4 *const xi_src = xi ? xi : xf.p;
    // rhosum/multiphase fused into the fill passes (k_neigh3 RHO): current positions, due now
    const bool rho = mp && !xi && rhofuse_env() && mpc.rhosum_nstep > 0 &&
                     step % mpc.rhosum_nstep == 0;
    SPH_REQUIRE(!mp || (long long)nall < MP_MAXALL, SPH_HIP_EOVERFLOW,
                "multiphase lists index at most 2^28 atoms per rank (%d)", nall);
    if (rho) rho_tmp.reserve(nlocal + nghost);
    rho_fused_step = rho ? step : -1;  // (every path below ends in a fill pass)
    ccnt.reserve(n + 1);
    off.reserve(n + 1);
    constexpr int G = 8;
    dim3 grid(grid_for_rows(n, G)), block(BLK);
    auto launch = [&](bool fill, int stride, int *dst = nullptr) {
      if (n == 0) return;
      const bool t = nt1();
      int *const cnt_out = (!fill || stride > 0) ? ccnt.p : (int *)nullptr;
      int *const rows = dst ? dst : nbr.p;
#define SPH_N3P(F, T, P)                                                                       \
  hipLaunchKernelGGL((k_neigh3<G, 4, F, T, false, P>), grid, block, 0, s, n, qb, cfg.dim,       \
                     xi_src, ty.p,                                                             \
                     xb.p, tb.p, qbeg.p, dc, cnt_out,                                          \
                     (F && stride == 0) ? off.p : (const int *)nullptr,                        \
                     F ? rows : (int *)nullptr, stride, mx.p, stride > 0 ? list_perm_g : 0,    \
                     list_perm_pi, mp ? 2 : ((stride > 0 && list_tbits) ? 1 : 0))
#define SPH_N3R(T)                                                                             \
  hipLaunchKernelGGL((k_neigh3<G, 4, true, T, true, true>), grid, block, 0, s, n, qb, cfg.dim,  \
                     xi_src,                                                                   \
                     ty.p, xb.p, tb.p, qbeg.p, dc, cnt_out,                                    \
                     stride == 0 ? off.p : (const int *)nullptr, rows, stride, mx.p, 0, 0, 2, \
                     dm, rm.p, rho_tmp.p)
      // (mp: xb packs the types, k_bin_copy tpack)
#define SPH_N3(F, T)                                                                           \
  do {                                                                                        \
    if (mp) SPH_N3P(F, T, true);                                                              \
    else SPH_N3P(F, T, false);                                                                \
  } while (0)
      if (fill && rho) { if (t) SPH_N3R(true); else SPH_N3R(false); }
      else if (fill) { if (t) SPH_N3(true, true); else SPH_N3(true, false); }
      else { if (t) SPH_N3(false, true); else SPH_N3(false, false); }
#undef SPH_N3
#undef SPH_N3P
#undef SPH_N3R
    };
    mx.reserve(8);
    // single pass into fixed-stride rows when a previous build sized them and nothing
    // needs the CSR form (the setup's half-list pass)
    // (the multiphase passes index rows with 64-bit offsets, MpRow: plain rows, any size)
    const bool sfits = mp ? true : row2_fits((long)nall, (long)n * list_stride);
    bool sover = false;  // the strided fill overflowed: a CSR fill at the same stride would too
    if (!csr && list_stride > 0 && sfits) {
      // rows stored chunk-transposed for the row2 kernels' 16-B index loads; with several
      // types the neighbour's type rides in the entry's top bits
      list_perm_g = (row2_iv() && !mp) ? row2_iv_g() : 0;
      list_perm_pi = (row2_pi() && !mp) ? 1 : 0;
      list_tbits = !nt1() && tbits_env() && !mp;
      nbr.reserve((size_t)n * list_stride);
      SPH_HIP_TRY(hipMemsetAsync(mx.p, 0, sizeof(int), s));
      launch(true, list_stride);
      if (read_scalar(mx.p) == 0) {
        strided = true;
        nbr_total = -1;  // entries counted on demand (stats)
        nbr_builds++;
        return;
      }
      sover = true;
    }
    strided = false;
    list_tbits = false;
    // CSR: when an earlier build sized the rows, ONE fill pass into fixed-stride scratch rows
    // (counts as a by-product) compacted into CSR after the scan -- instead of a count pass
    // and a fill pass (the C5 stack rebuilds every step); a row past the stride falls back
    bool filled = false;
    if (!sover && list_stride > 0 && (long)n * list_stride < 0x7fffffffL) {
      list_perm_g = 0;
      list_perm_pi = 0;
      nbs.reserve((size_t)n * list_stride);
      SPH_HIP_TRY(hipMemsetAsync(mx.p, 0, sizeof(int), s));
      launch(true, list_stride, nbs.p);
      filled = read_scalar(mx.p) == 0;
    }
    if (!filled) launch(false, 0);
    hipLaunchKernelGGL(k_copy_counts, dim3(blocks(n + 1)), dim3(BLK), 0, s, n, ccnt.p, off.p);
    size_t tb2 = 0;
    SPH_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, off.p, off.p, n + 1, s));
    tmp_reserve(tb2);
    SPH_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb2, off.p, off.p, n + 1, s));
    size_t tb3 = 0;
    SPH_HIP_TRY(hipcub::DeviceReduce::Max(nullptr, tb3, ccnt.p, mx.p + 1, n, s));
    tmp_reserve(tb3);
    if (n > 0) SPH_HIP_TRY(hipcub::DeviceReduce::Max(tmp.p, tb3, ccnt.p, mx.p + 1, n, s));
    else SPH_HIP_TRY(hipMemsetAsync(mx.p + 1, 0, sizeof(int), s));
    int hm[2];
    SPH_HIP_TRY(hipMemcpyAsync(&hm[0], off.p + n, sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipMemcpyAsync(&hm[1], mx.p + 1, sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    const int tot = hm[0];
    SPH_REQUIRE(tot >= 0, SPH_HIP_EOVERFLOW, "neighbor list exceeds 2^31 entries");
    nbr.reserve(tot > 0 ? tot : 1);
    if (filled) {
      if (n)
        hipLaunchKernelGGL(k_compact_rows, dim3((unsigned)(((long)n * 32 + BLK - 1) / BLK)),
                           dim3(BLK), 0, s, n, list_stride, ccnt.p, off.p, nbs.p, nbr.p);
    } else {
      launch(true, 0);
    }
    // stride of later single-pass builds: this build's longest row + 25% + 16, 64-aligned
    // (whole chunks of the transposed layout, 16-B aligned rows)
    list_stride = ((hm[1] + hm[1] / 4 + 16) + 63) & ~63;
    nbr_maxrow = hm[1];
    nbr_total = tot;
    nbr_builds++;
  }

  // Block unions + slot rows straight from the bins (k_blk_neigh; bin_q() must have run) in
  // the SPH_BLK shape.  The row stride is the last CSR build's (list_stride), doubled if a
  // row outgrows it; false (the row path takes over) if a block overflows its LDS image.
  bool build_blk() {
    const int n = nlocal;
    if (n == 0) return false;
    mx.reserve(10);
    ccnt.reserve(n + 1);
    if (blk_rowcap == 0) blk_rowcap = std::max(list_stride, nbr_maxrow + nbr_maxrow / 4 + 16);
    // the SPH_BLK shape, then 32-row blocks (smaller unions), then 32-row blocks with the
    // build's large candidate image, if the blocks do not fit
    const int first = blk_shape_env();
    const int chain[3][2] = {{first, 0}, {1, 0}, {1, 1}};
    for (const auto &c : chain) {
      if (c[0] == 1 && first == 1 && c[1] == 0 && &c != &chain[0]) continue;
      const int r = build_blk_shape(c[0], c[1] != 0);
      if (r == 1) return true;
      if (r != 2) return false;  // (2: a block overflowed: the next, roomier variant)
    }
    return false;
  }
  // 1 = built, 2 = a block overflowed (candidates, bin table or LDS image), 0 = failed
  int build_blk_shape(int shape, bool big) {
    const int n = nlocal;
    const BlkShape sh = blk_shape(shape);
    const int chunk = sh.G * sh.U;
    // k_blk_build2 (group candidate lists, sph_blk_build2.h): measured slower than
    // k_blk_build (1.37 vs 1.11 ms at C2 1M, profiles/r05/README.md) -> study builds only
    bool try2 = study_int("SPH_BUILD2", 0) != 0;
    for (int attempt = 0; attempt < 3; attempt++) {
      blk_sstride = (std::max(blk_rowcap, 1) + chunk - 1) / chunk * chunk;
      snbr.reserve((size_t)n * blk_sstride + 2 * chunk);  // + the pair passes' prefetch pad
      const int nb = blk_blocks(n, sh.R);
      ulist.reserve((size_t)nb * BLK_UCAP);
      ucnt.reserve(nb);
      kcnt.reserve(nb);
      SPH_HIP_TRY(hipMemsetAsync(mx.p, 0, 10 * sizeof(int), s));
      // k_blk_build (ballots, inner rows in the same pass); the bitmap walk k_blk_neigh for
      // the large candidate image (and in study builds, SPH_BUILD=0)
      const bool v2 = !big && study_int("SPH_BUILD", 1) != 0;
      // the inner rows' ballots inside the build (SPH_INNER_INLINE, study; default 1), or a
      // k_blk_inner pass over the full rows afterwards (build_inner)
      const bool want_inner = inner_margin > 0.0 && inner_inline();
      if (want_inner) {
        snbi.reserve((size_t)n * blk_sstride + 2 * chunk);
        icnt.reserve(n);
        uilist.reserve((size_t)nb * BLK_UCAP);
        uicnt.reserve(nb);
      }
      // Newton-3 inside the blocks (k_blk_build N3): the passes walk the stored rows (pcnt),
      // ccnt keeps the full counts
      blk_n3 = v2 && n3_env();
      if (blk_n3) pcnt.reserve(n + 1);
      // the inner rows over their own union (not with N3: its rows-first union)
#ifdef SPH_NO_IU  // (A/B builds: inner rows over the full union)
      const bool iu = false;
#else
      const bool iu = v2 && want_inner && !blk_n3;
#endif
      // the group-list build (sph_blk_build2.h) unless a study variant needs k_blk_build
      const bool v3 = v2 && try2 && !blk_n3 && !rowsort();
#ifdef SPH_STUDY
      if (v3)
        blk_build2(shape, nt1(), want_inner, s, n, qb, cfg.dim, xf.p, ty.p, xb.p, tb.p, qbeg.p,
                   dc, BLK_UCAP, blk_sstride, ulist.p, ucnt.p, ccnt.p, snbr.p, icnt.p, snbi.p,
                   mx.p, mx.p + 1, blk_cq(), iu ? uilist.p : nullptr, iu ? uicnt.p : nullptr,
                   kcnt.p);
      else
#endif
      if (v2)
        blk_build(shape, nt1(), want_inner, blk_n3, s, n, qb, cfg.dim, xf.p, ty.p, xb.p, tb.p,
                  qbeg.p, dc, BLK_UCAP, blk_sstride, ulist.p, ucnt.p,
                  blk_n3 ? pcnt.p : ccnt.p, snbr.p, icnt.p, snbi.p, mx.p, mx.p + 1, blk_cq(),
                  study_int("SPH_BEXP", 0) | (blk_ksmall ? 0x100 : 0), ccnt.p,
                  rowsort() ? bperm_buf(nb, sh.R) : nullptr,
                  iu ? uilist.p : nullptr, iu ? uicnt.p : nullptr, kcnt.p);
      else
        blk_neigh(shape, big, nt1(), s, n, qb, cfg.dim, xf.p, ty.p, xb.p, tb.p, qbeg.p, xpos.p,
                  dc, BLK_UCAP, blk_sstride, ulist.p, ucnt.p, ccnt.p, snbr.p, mx.p, mx.p + 1,
                  blk_cq(), study_int("SPH_BEXP", 0));
      inner_written = v2 && want_inner;
      blk_iu = iu;
      blk_perm = v2 && !blk_n3 && rowsort();
      // the build's statistics: ONE read-back
      int *const hm = h_small;
      SPH_HIP_TRY(hipMemcpyAsync(hm, mx.p, 9 * sizeof(int), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipStreamSynchronize(s));
      if (env_int("SPH_DEBUG", 0))
        fprintf(stderr,
                "[sph] k_blk_neigh shape %d%s n %d rowcap %d: ovf %d union max %d mean %.1f, "
                "candidates max %d mean %.1f\n",
                shape, big ? " (large image)" : "", n, blk_rowcap, hm[0], hm[1], (double)hm[4] / nb, hm[2],
                (double)hm[3] / nb);
      if (hm[0] == (1 << 23)) {  // a group list outgrew k_blk_build2's: k_blk_build
        try2 = false;
        continue;
      }
      if (hm[0] == (1 << 24)) {  // a block outgrew the small candidate image
        blk_ksmall = false;
        blk_kover++;
        continue;
      }
      if (hm[0] == (1 << 21)) {  // a row outgrew the slot-row stride
        blk_rowcap *= 2;
        continue;
      }
      if (hm[0] != 0) return 2;
      // the rho and inner passes stage the whole largest union (24 B per slot, blk_rho_lds,
      // + their static tables): a union past the CU's 160 KiB takes the next shape or the row
      // path (only the force pass walks windows)
      if (blk_rho_lds(std::max(hm[1], 1), nt1()) + (nt1() ? 0 : sizeof(RhoPair) * NT2) +
              sizeof(double) * sh.R + 1024 > 163840)
        return 2;
      // the next build takes the small candidate image (four workgroups per CU) while this
      // one's largest block fits it (hm[2]: the largest candidate set; the blocks' sets move
      // by a few candidates between rebuilds); after two overflows it stays with the large one
      if (v2 && !v3) blk_ksmall = blk_kover < 2 && hm[2] <= BLK_SCAP_S - 24;
      // the largest union's force-pass LDS image (+ the static coefficient tables) must fit
      // the CU's 160 KiB
      blk_sh = shape;
      blk_um = std::max(hm[1], 1);
      // the force pass's LDS image: sized to the union the passes stage (the inner one when
      // the build wrote it), for as many workgroups per CU as fit; larger unions are walked
      // in windows (k_blk_force)
      if (iu)
        blk_umf = choose_umf(hm[7], (double)hm[8] / nb);
      else
        blk_umf = choose_umf(blk_um, (double)hm[4] / nb);
      hipLaunchKernelGGL(k_blk_count_big, dim3(blocks(nb)), dim3(BLK), 0, s, nb,
                         iu ? uicnt.p : ucnt.p, blk_umf, mx.p + 9);
      if (env_int("SPH_DEBUG", 0))
        fprintf(stderr, "[sph] inner union max %d mean %.1f; force image %d records\n", hm[7],
                (double)hm[8] / nb, blk_umf);
      return 1;
    }
    return 0;
  }
  // the union image's chunk size / 16 (sph_blk_kernels.h): with the heat term's e array
  int blk_cq() const { return ((force_mode & M_HEAT) ? BLK_CHE : BLK_CH) / 16; }
  // The force pass's LDS image in union records (a multiple of 16) for unions of at most
  // maxu records, meanu on average: the whole largest union if it fits three workgroups per
  // CU (6 waves per SIMD); else three workgroups' image when the mean union fits it with
  // 10 % to spare (the few larger unions walked in windows); else up to two workgroups'
  // image.  SPH_TUNE_BLKUMF caps it (tests force the windowed walk that way).
  int choose_umf(int maxu, double meanu) const {
    const bool one = nt1();
    const int cq = blk_cq();
    const size_t stat = (one ? 0 : (sizeof(TaitPair) + sizeof(HeatPair)) * NT2) + 1024;
    auto fits = [&](int w, int wgs) { return blk_lds(w, cq, one) + stat <= 163840 / wgs; };
    auto cap = [&](int wgs) {
      int w = 16;
      while (w < BLK_UCAP && fits(w + 16, wgs)) w += 16;
      return w;
    };
    const int m16 = std::max(16, (maxu + 15) / 16 * 16);
    int umf;
    if (fits(m16, 3)) umf = m16;
    else if (blk_n3) umf = std::min(m16, cap(1));  // (study N3: no windows)
    else if (meanu * 1.10 <= cap(3)) umf = cap(3);
    else umf = std::min(m16, cap(2));
    if (blkumf > 0 && !blk_n3) umf = std::min(umf, std::max(16, blkumf / 16 * 16));
    return umf;
  }
  BlkArgs blk_args() const {
    BlkArgs k;
    k.cq = blk_cq();
    k.n = nlocal;
    k.shape = blk_sh;
    k.exp = row2_exp();
    k.ucap = BLK_UCAP;
    k.um = blk_um;
    k.umf = blk_umf;
    k.sstride = blk_sstride;
    k.ulist = ulist.p;
    k.ucnt = ucnt.p;
    k.rcnt = blk_n3 ? pcnt.p : ccnt.p;
    k.n3 = blk_n3;
    k.bperm = blk_perm ? bperm.p : nullptr;
    k.snbr = snbr.p;
    if (inner) {
      k.snbi = snbi.p;
      k.icnt = icnt.p;
      k.moved = moved_flag();
      k.iu = blk_iu;
      k.uilist = blk_iu ? uilist.p : ulist.p;
      k.uicnt = blk_iu ? uicnt.p : ucnt.p;
    }
    return k;
  }

  // pbc + sort + borders + bins + list(s); `need_csr` also builds the global-index CSR
  // list (the setup's half-list pass walks it).  Block path: the block unions + slot rows
  // from the bins (no global-index list on a plain rebuild); the row path's strided list
  // if a block overflows its LDS image.
  void build_all(bool need_csr) {
    // (the multiphase passes walk global-index full rows carrying each pair's half-list
    // orientation, k_neigh3: CSR at setup, fixed-stride rows once the setup sized them)
    hipLaunchKernelGGL(k_pbc, dim3(blocks(nlocal)), dim3(BLK), 0, s, nlocal, box, xf.p, vel.p);
    if (multi()) exchange_multi();
    // Atom::sort between the exchange and borders (verlet.cpp:106, 251): only the LAMMPS
    // indices move -- the rows keep the engine's own order
    if (pc && sortfreq > 0 && step >= nextsort) atom_sort();
    // (at most every sort_every() steps, as atom_modify sort Nevery: the C5 stack rebuilds
    // every step, and its rows keep their locality over a few steps of motion)
    if (cfg.sort && (force_sort || !setup_done || step == 0 || step - last_sort >= sort_every())) {
      sort_owned();
      last_sort = step;
    }
    force_sort = false;
    borders();
    if (cfg.sort) grow_twins();
    bin_q();
    blk = false;
    if (need_csr || !want_blk() || mp) list_q(need_csr);
    if (mp) {
      ov_ready = false;
      return;
    }
    if (want_blk()) {
      blk = build_blk();
      build_inner();
      if (blk && !need_csr) {
        strided = true;  // (ccnt holds the full-list counts; list_entries sums them)
        nbr_total = -1;
        nbr_builds++;
      } else if (!blk && !need_csr) {
        list_q(false);
      }
    }
    ov_ready = false;
    if (overlap_on()) classify_rows();
  }

  // The block path's inner rows (sph_blk_kernels.h k_blk_inner), written after every block
  // build: the pair passes walk them while no atom has moved inner_margin / 2 since (owned
  // atoms: checked by the integrate kernels; bricks: the ghosts after each forward comm).
  void build_inner() {
    inner = blk && inner_margin > 0.0 && nlocal > 0;
    sc.x0 = nullptr;
    if (!inner) return;
    const BlkShape sh = blk_shape(blk_sh);
    snbi.reserve((size_t)nlocal * blk_sstride + 2 * sh.U * sh.G);
    icnt.reserve(nlocal);
    uilist.reserve((size_t)blk_blocks(nlocal, sh.R) * BLK_UCAP);
    uicnt.reserve(blk_blocks(nlocal, sh.R));
    moved.reserve(2);
    const size_t nx0 = (size_t)nlocal + (multi() ? nghost : 0);
    x0.reserve(nx0);
    if (!inner_written) {  // (k_blk_inner writes the inner unions too)
      blk_iu = true;
      BlkArgs k = blk_args();
      blk_inner(nt1(), s, k, xf.p, ty.p, dc, snbi.p, icnt.p);
    }
    SPH_HIP_TRY(hipMemcpyAsync(x0.p, xf.p, nx0 * sizeof(double4), hipMemcpyDeviceToDevice, s));
    SPH_HIP_TRY(hipMemsetAsync(moved.p, 0, 2 * sizeof(int), s));
    sc.x0 = x0.p;
    sc.lim2 = 0.25 * inner_margin * inner_margin;
    sc.moved = moved_flag();
  }
  // The moved flag of this step (two slots, by step parity: the integrate and the ghost check
  // of step k raise slot k & 1 against x0, the passes of step k read it; refresh_inner
  // clears the other slot for step k + 1).  Validity of the inner rows depends only on the
  // current displacements from x0, so a flag per step, not a sticky one, is exact.
  int *moved_flag() const { return moved.p ? moved.p + (step & 1) : nullptr; }
  // After the passes of a step between rebuilds: if this step's flag is raised, the inner
  // rows are derived again from the full rows at the current positions (x0 := them), so the
  // next steps walk ~120 instead of ~155 entries per row until the next rebuild; skipped
  // when the next step rebuilds anyway.
  void refresh_inner(bool rebuild_next) {
    if (!inner || !sc.x0 || !refresh_env()) return;
    if (rebuild_next) return;  // (the rebuild clears both slots)
    int *const cur = moved_flag();
    int *const nxt = moved.p + ((step + 1) & 1);
    BlkArgs k = blk_args();
    BlkInnerRefresh rf;
    rf.cond = cur;
    rf.zero = nxt;
    rf.x0 = x0.p;
    blk_inner(nt1(), s, k, xf.p, ty.p, dc, snbi.p, icnt.p, rf);
    if (multi() && nghost)
      hipLaunchKernelGGL(k_x0_cond, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost, cur,
                         xf.p + nlocal, x0.p + nlocal);
    inner_refreshes++;
  }

  bool overlap_on() const {
    return multi() && overlap && (blk || use_row2()) && !tight_on() &&
           (force_mode & M_TAIT) != 0 && cfg.rhosum_nstep > 0;
  }
  // interior rows (no ghost in the list) and boundary rows, each in row order; on the block
  // path interior and boundary BLOCKS (no ghost in the union, k_blk_interior)
  void classify_rows() {
    const int n = nlocal;
    if (!s2) {
      // (a lowest-priority s2 was measured: the interior rows starve, 1.31 -> 2.17 ms per
      // step on the loopback bench)
      SPH_HIP_TRY(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      SPH_HIP_TRY(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
      SPH_HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    }
    if (blk) {
      const int nb = blk_blocks(n, blk_shape(blk_sh).R);
      fl_in.reserve(nb > 0 ? nb : 1);
      fl_bd.reserve(nb > 0 ? nb : 1);
      if (nb)
        hipLaunchKernelGGL(k_blk_interior, dim3(nb), dim3(64), 0, s, nb, ulist.p, ucnt.p,
                           BLK_UCAP, nlocal, fl_in.p, fl_bd.p);
      n_in = select_flagged(fl_in.p, nb, rows_in);
      n_bd = select_flagged(fl_bd.p, nb, rows_bd);
      SPH_REQUIRE(n_in + n_bd == nb, SPH_HIP_ERUNTIME, "block classification lost blocks");
      ov_ready = true;
      return;
    }
    fl_in.reserve(n > 0 ? n : 1);
    fl_bd.reserve(n > 0 ? n : 1);
    if (n)
      hipLaunchKernelGGL(k_row_ghost_flags, dim3((unsigned)(((long)n * 8 + 255) / 256)),
                         dim3(256), 0, s, n, nlocal, strided ? nullptr : off.p,
                         strided ? list_stride : 0, ccnt.p, nbr.p, list_perm_g, list_perm_pi,
                         (strided && list_tbits) ? 1 : 0, fl_in.p, fl_bd.p);
    n_in = select_flagged(fl_in.p, n, rows_in);
    n_bd = select_flagged(fl_bd.p, n, rows_bd);
    SPH_REQUIRE(n_in + n_bd == n, SPH_HIP_ERUNTIME, "row classification lost rows");
    ov_ready = true;
  }
  void fork() {  // s2 continues after everything queued on s so far
    SPH_HIP_TRY(hipEventRecord(ev_fork, s));
    SPH_HIP_TRY(hipStreamWaitEvent(s2, ev_fork, 0));
  }
  void join() {  // s continues after everything queued on s2 so far
    SPH_HIP_TRY(hipEventRecord(ev_join, s2));
    SPH_HIP_TRY(hipStreamWaitEvent(s, ev_join, 0));
  }

  // Forward comm + rhosum + forward rho + taitwater(+heat) of a non-rebuild step with the
  // halos overlapped: interior rows read no ghost, so their rhosum runs (on s2) while the
  // x/vest/rho/e halo moves, and their force pass while the rho halo moves; boundary rows
  // follow each exchange on s.  Same per-row arithmetic as pair_compute (bit-identical).
  // The forward pack may read an interior row's rho/EOS term before or after this
  // step's rhosum wrote it: ghost rho and P/rho^2 are only read after the rho halo has
  // overwritten them, so either value is harmless.
  void pair_compute_overlap() {
    if (blk) {  // the same on the block path: interior blocks first, on s2
      BlkArgs ka = blk_args(), ki = ka, kb = ka;
      ki.blist = rows_in.p;
      ki.nlist = n_in;
      kb.blist = rows_bd.p;
      kb.nlist = n_bd;
      {
        Scope t(this, T_RHO);  // (this class then includes the forward halo)
        fork();
        blk_rhosum(nt1(), s2, ki, xf.p, ty.p, vr.p, dc);
        forward_multi();
        // (the ghosts' displacement check of forward(): the interior blocks read no ghost,
        // so whether they saw the flag before or after it is harmless)
        if (inner && sc.x0 && nghost)
          hipLaunchKernelGGL(k_inner_ghosts, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost,
                             nlocal, sc, xf.p);
        blk_rhosum(nt1(), s, kb, xf.p, ty.p, vr.p, dc);
        join();
      }
      {
        Scope t(this, (force_mode & M_TAIT) ? T_TAIT : T_HEAT);  // (includes the rho halo)
        fork();
        blk_force(nt1(), blk_visc(), force_mode, s2, ki, row_args());
        forward_rho_multi();
        blk_force(nt1(), blk_visc(), force_mode, s, kb, row_args());
        join();
      }
      return;
    }
    Row2Args b = row2_args(), bi = b, bb = b;
    bi.a.n = n_in;
    bi.rows = rows_in.p;
    bb.a.n = n_bd;
    bb.rows = rows_bd.p;
    {
      Scope t(this, T_RHO);  // (this class then includes the forward halo)
      fork();
      row2_rhosum(nt1(), s2, bi);
      forward_multi();
      row2_rhosum(nt1(), s, bb);
      join();
    }
    {
      Scope t(this, (force_mode & M_TAIT) ? T_TAIT : T_HEAT);  // (includes the rho halo)
      fork();
      row2_force(nt1(), cfg.tait_visc, force_mode, s2, bi);
      forward_rho_multi();
      row2_force(nt1(), cfg.tait_visc, force_mode, s, bb);
      join();
    }
  }

  void rebuild() {
    Scope t(this, T_NEIGH);
    build_all(false);
  }

  void forward() {
    if (multi()) {
      Scope t(this, T_COMM);
      forward_multi();
      if (inner && sc.x0 && nghost)
        hipLaunchKernelGGL(k_inner_ghosts, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost,
                           nlocal, sc, xf.p);
      return;
    }
    if (nghost == 0) return;
    Scope t(this, T_COMM);
    hipLaunchKernelGGL(k_forward, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost, nlocal, box,
                       gowner.p, gimg.p, xf.p, vr.p, en.p);
    mpx_copy(nghost, gowner.p, nlocal, xbuf);
  }

  RowArgs row_args() {
    RowArgs a;
    a.n = nlocal;
    a.off = off.p;
    a.nbr = nbr.p;
    a.xf = xf.p;
    a.vr = vr.p;
    a.ty = ty.p;
    a.en = en.p;
    a.cf = dc;
    a.fo = fo.p;
    a.de = de.p;
    a.gx = cfg.gravity[0];
    a.gy = cfg.gravity[1];
    a.gz = cfg.gravity[2];
    return a;
  }
  // extent of the list array the kernels may address
  int64_t list_span() const { return strided ? (int64_t)nlocal * list_stride : nbr_total; }
  // entries of the current list (sum of row counts for a strided list)
  int64_t list_entries() {
    if (!strided) return nbr_total;
    if (nlocal == 0) return 0;
    blen.reserve(1);
    size_t tb = 0;
    SPH_HIP_TRY(hipcub::DeviceReduce::Sum(nullptr, tb, ccnt.p, blen.p, nlocal, s));
    tmp_reserve(tb);
    SPH_HIP_TRY(hipcub::DeviceReduce::Sum(tmp.p, tb, ccnt.p, blen.p, nlocal, s));
    long long v = 0;
    SPH_HIP_TRY(hipMemcpyAsync(&v, blen.p, sizeof(long long), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    return v;
  }
  Row2Args row2_args() {
    Row2Args b;
    b.a = row_args();
    b.nall = nlocal + nghost;
    b.ntot = (int)list_span();
    if (strided) {
      b.stride = list_stride;
      b.rcnt = ccnt.p;
    }
    b.lp = row2_lp();
    b.pi = row2_pi();
    b.iv = strided && list_perm_g > 0 && list_perm_g == row2_iv_g() &&
           list_perm_pi == (b.pi ? 1 : 0);
    b.exp = row2_exp();
    b.tbits = strided && list_tbits;
    return b;
  }
  bool use_row2() const { return row2_fits((long)nlocal + nghost, (long)list_span()); }

  // rhosum (+ the EOS epilogue) -> forward rho -> taitwater[/morris][+heat] on the current
  // list: block path, row path (row2 kernels), or the generic CSR kernels for a list past
  // the row2 kernels' 32-bit offsets.  The setup step's force pass walks the half list.
  void pair_compute(bool do_rhosum, bool setup = false) {
    if (mp) {
      pair_compute_mp();
      return;
    }
    const int nall = nlocal + nghost;
    bool tight = false;
    if (do_rhosum) {
      {
        Scope t(this, T_RHO);
        if (blk) {
          blk_rhosum(nt1(), s, blk_args(), xf.p, ty.p, vr.p, dc);
        } else if (use_row2()) {
          Row2Args b = row2_args();
          if (strided && row2_lp() && tight_on() && force_mode && !setup) {
            tnbr.reserve((size_t)list_span());
            tcnt.reserve(nlocal > 0 ? nlocal : 1);
            b.tnbr = tnbr.p;
            b.tcnt = tcnt.p;
            tight = true;
          }
          row2_rhosum(nt1(), s, b);
        } else {
          RhoArgs ra{nlocal, nullptr, off.p, nbr.p, xf.p, ty.p, vr.p, nullptr, dc};
          launch_rhosum(cfg.dim, true, nt1(), s, ra);
        }
      }
      if (multi()) {
        Scope t(this, T_COMM);
        forward_rho_multi();
      } else if (nghost) {
        Scope t(this, T_COMM);
        hipLaunchKernelGGL(k_forward_rho, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost,
                           nlocal, gowner.p, xf.p, vr.p);
      }
    } else if (force_mode & M_TAIT) {
      hipLaunchKernelGGL(k_eos, dim3(blocks(nall)), dim3(BLK), 0, s, nall, xf.p, vr.p, ty.p, dc);
    }
    if (force_mode && setup) {
      setup_forces_full();
    } else if (force_mode && blk) {
      Scope t(this, (force_mode & M_TAIT) ? T_TAIT : T_HEAT);
      blk_force(nt1(), blk_visc(), force_mode, s, blk_args(), row_args());
    } else if (force_mode && use_row2()) {
      Scope t(this, (force_mode & M_TAIT) ? T_TAIT : T_HEAT);
      Row2Args b = row2_args();
      if (tight) {  // this step's in-cut list from the rhosum pass (same strided rows)
        b.a.nbr = tnbr.p;
        b.rcnt = tcnt.p;
        b.iv = false;
      }
      row2_force(nt1(), cfg.tait_visc, force_mode, s, b);
    } else if (force_mode) {
      Scope t(this, (force_mode & M_TAIT) ? T_TAIT : T_HEAT);
      ForceArgs a{};
      a.inum = nlocal;
      a.nlocal = nlocal;
      a.newton = 1;
      a.ilist = nullptr;
      a.off = off.p;
      a.nbr = nbr.p;
      a.xf = xf.p;
      a.vr = vr.p;
      a.ty = ty.p;
      a.en = en.p;
      a.fo = fo.p;
      a.de = de.p;
      a.accum = 0;
      a.cf = dc;
      a.gx = cfg.gravity[0];
      a.gy = cfg.gravity[1];
      a.gz = cfg.gravity[2];
      a.virial = nullptr;
      launch_force(cfg.dim, nt1(), s, cfg.tait_visc, force_mode, a);
    } else {
      SPH_HIP_TRY(hipMemsetAsync(fo.p, 0, nlocal * sizeof(double4), s));
      SPH_HIP_TRY(hipMemsetAsync(de.p, 0, nlocal * sizeof(double), s));
    }
  }

  // Force pass of Verlet::setup with the reference's half-list ownership (see
  // k_half_from_full): exact even though ghost vest is stale at this point.
  // The setup step's force pass (Verlet::setup, verlet.cpp:88-139): borders() ran before
  // FixMeso::setup_pre_force, so the reference's half-list pass sees a ghost's vest as it
  // was bordered.  Walked as a full-list gather (the global-index CSR rows of the setup
  // build) that picks, for each ghost pair, the vest pair the reference's one evaluation
  // uses (k_force: vso / vsg) -- no half list, no atomics, no reverse comm.
  DBuf<double4> vso, vsg;  // owned vest before setup_pre_force; ghosts' vest as bordered
  void setup_forces_full() {
    const int n = nlocal, nall = nlocal + nghost;
    if (force_mode == 0 || n == 0) return;
    vsg.reserve(nghost > 0 ? nghost : 1);
    if (nghost)
      SPH_HIP_TRY(hipMemcpyAsync(vsg.p, vr.p + n, (size_t)nghost * sizeof(double4),
                                 hipMemcpyDeviceToDevice, s));
    forward();  // the ghosts' vest as setup_pre_force left their owners' (x, rho, e unchanged)
    fo.reserve(nall, true, s);
    de.reserve(nall, true, s);
    ForceArgs a{};
    a.inum = n;
    a.nlocal = n;
    a.newton = 1;
    a.off = off.p;
    a.nbr = nbr.p;
    a.xf = xf.p;
    a.vr = vr.p;
    a.ty = ty.p;
    a.en = en.p;
    a.fo = fo.p;
    a.de = de.p;
    a.cf = dc;
    a.gx = cfg.gravity[0];
    a.gy = cfg.gravity[1];
    a.gz = cfg.gravity[2];
    a.vso = vso.p;
    a.vsg = vsg.p;
    launch_force(cfg.dim, nt1(), s, cfg.tait_visc, force_mode, a);
  }

  // ---- multiphase stack -------------------------------------------------------------
  static dim3 mp_rows(int rows) { return dim3((unsigned)(((long long)rows * 8 + 255) / 256)); }
  // hybrid/overlay of bubble.lmp:57-73 in order: rhosum/multiphase and colorgradient over
  // the full list (owned rows; no forward comm of either, A.6-1), then taitwater/multiphase,
  // surfacetension and heatconduction/phasechange fused in one gather over the full list,
  // each pair in its half-list orientation (k_mp_gather: the reference's Newton-3 scatter +
  // reverse comm, without atomics or comm)
  void pair_compute_mp() {
    const int n = nlocal, nall = nlocal + nghost;
    fo.reserve(n > 0 ? n : 1, true, s);
    de.reserve(n > 0 ? n : 1, true, s);
    if (n == 0) return;
    MpArgs a{};
    a.stride = strided ? list_stride : 0;  // (else CSR: off)
    a.cnt = ccnt.p;
    a.inum = n;
    a.nlocal = n;
    a.newton = 1;
    a.dim = cfg.dim;
    a.ilist = nullptr;  // (rows = owned atoms)
    a.off = off.p;
    a.nbr = nbr.p;
    a.xf = xf.p;
    a.vr = vr.p;
    a.ty = ty.p;
    a.rm = rm.p;
    a.en = en.p;
    a.cv = cvv.p;
    a.mc = dm;
    a.typed = mp_typed_env() ? 1 : 0;  // (k_neigh3 tbits 2 writes the types)
    // the stale version: rho and colorgradient as communicated (k_mp_gather)
    rhoS.reserve(nall);
    cgS.reserve(nall);
    hipLaunchKernelGGL(k_mp_snap, dim3(blocks(nall)), dim3(BLK), 0, s, nall, vr.p, cg.p, rhoS.p,
                       cgS.p);
    const bool rdue = mpc.rhosum_nstep > 0 && step % mpc.rhosum_nstep == 0;
    const bool cdue = mpc.cg_nstep > 0 && step % mpc.cg_nstep == 0;
    {
      Scope t(this, T_RHO);
      if (rdue) {
        rho_tmp.reserve(nall);
        a.rho = rho_tmp.p;
        if (rho_fused_step != step)  // (else the list fill of this step summed it)
          hipLaunchKernelGGL(k_mp2_rhosum<8>, mp_rows(n), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_mp_rho_store, dim3(blocks(n)), dim3(BLK), 0, s, n, rho_tmp.p, vr.p);
      }
      if (cdue) {
        a.cg = cg.p;
        recA.reserve(nall);  // (free until the force pass packs its records)
        hipLaunchKernelGGL(k_mp_pack_sigma, dim3(blocks(nall)), dim3(BLK), 0, s, nall, xf.p, vr.p,
                           rm.p, recA.p);
        a.xs = recA.p;
        hipLaunchKernelGGL(k_mp2_colorgradient<8>, mp_rows(n), dim3(256), 0, s, a);
        a.xs = nullptr;
      }
    }
    // the fresh version: the owned atoms' new values, forwarded to the ghosts
    const double *rF = rhoS.p;
    const double4 *cF = cgS.p;
    if (rdue || cdue) {
      Scope t(this, T_COMM);
      rhoF.reserve(nall);
      cgF.reserve(nall);
      hipLaunchKernelGGL(k_mp_snap, dim3(blocks(n)), dim3(BLK), 0, s, n, vr.p, cg.p, rhoF.p,
                         cgF.p);
      forward_fresh();
      rF = rhoF.p;
      cF = cgF.p;
    }
    Scope t(this, T_TAIT);
    if (!mpc.tait_on && !mpc.st_on)
      SPH_HIP_TRY(hipMemsetAsync(fo.p, 0, n * sizeof(double4), s));
    if (!mpc.heat_on) SPH_HIP_TRY(hipMemsetAsync(de.p, 0, n * sizeof(double), s));
    MpArgs h = a;
    h.vel = vel.p;
    h.rhoS = rhoS.p;
    h.rhoF = rF;
    h.cgS = cgS.p;
    h.cgF = cF;
    h.fo = fo.p;
    h.de = de.p;
    recA.reserve(nall);
    recK.reserve(nall);
    recF.reserve(nall);
    recS.reserve(nall);
    // symmetric styles (mp2_symmetric): the issue-rate gather of sph_mp2_kernels.h
    const bool sym = mp2_symmetric(hm);
    if (sym)
      hipLaunchKernelGGL(k_mp2_pack_rec, dim3(blocks(nall)), dim3(BLK), 0, s, nall, cfg.dim,
                         xf.p, vel.p, rm.p, en.p, cvv.p, rF, rhoS.p, cF, cgS.p,
                         mpc.heat_on ? 1 : 0, recA.p, recK.p, recF.p, recS.p);
    else
      hipLaunchKernelGGL(k_mp_pack_rec, dim3(blocks(nall)), dim3(BLK), 0, s, nall, xf.p, vel.p,
                         rm.p, en.p, cvv.p, rF, rhoS.p, cF, cgS.p, mpc.heat_on ? 1 : 0, recA.p,
                         recK.p, recF.p, recS.p);
    h.pA = recA.p;
    h.pK = recK.p;
    h.pF = recF.p;
    h.pS = recS.p;
    const int sel = (mpc.tait_on ? 1 : 0) | (mpc.st_on ? 2 : 0) | (mpc.heat_on ? 4 : 0);
    const bool g1 = mp2_gamma1(hm);
    switch (sel) {
#define SPH_MPG(k, T, S, H)                                                                   \
  case k:                                                                                     \
    if (sym && g1)                                                                            \
      hipLaunchKernelGGL((k_mp2_gather_w4<8, T, S, H>), mp_rows(n), dim3(256), 0, s, h);      \
    else if (sym)                                                                             \
      hipLaunchKernelGGL((k_mp2_gather<8, T, S, H, true>), mp_rows(n), dim3(256), 0, s, h);   \
    else hipLaunchKernelGGL((k_mp_gather<8, T, S, H>), mp_rows(n), dim3(256), 0, s, h);       \
    break;
      SPH_MPG(1, true, false, false)
      SPH_MPG(2, false, true, false)
      SPH_MPG(3, true, true, false)
      SPH_MPG(4, false, false, true)
      SPH_MPG(5, true, false, true)
      SPH_MPG(6, false, true, true)
      SPH_MPG(7, true, true, true)
#undef SPH_MPG
      default: break;
    }
  }

  // rhoF / cgF of the ghosts from their owners (the values the reference's half-list pass
  // uses for a pair evaluated in the owner's row, k_mp_gather)
  void forward_fresh() {
    if (!multi()) {
      if (nghost)
        hipLaunchKernelGGL(k_mp_fwd_fresh, dim3(blocks(nghost)), dim3(BLK), 0, s, nghost, nlocal,
                           gowner.p, rhoF.p, cgF.p);
      return;
    }
    forward_dims(
        4 * sizeof(double),
        [&](Swap &sw, unsigned char *buf) {
          hipLaunchKernelGGL(k_mp_pack_fresh, dim3(blocks(sw.nsend)), dim3(BLK), 0, s, sw.nsend,
                             sw.list.p, rhoF.p, cgF.p, (double *)buf);
        },
        [&](Swap &sw, unsigned char *buf) {
          hipLaunchKernelGGL(k_mp_unpack_fresh, dim3(blocks(sw.nrecv)), dim3(BLK), 0, s,
                             sw.nrecv, sw.firstrecv, (const double *)buf, rhoF.p, cgF.p);
        });
  }

  // ordered indices i in [0, n) with flag[i] != 0 (int flags) -> out; host sync
  int select_flagged_i(const int *flag, int n, DBuf<int> &out) {
    out.reserve(n > 0 ? n : 1);
    nsel.reserve(1);
    if (n == 0) return 0;
    hipcub::CountingInputIterator<int> it(0);
    size_t tb = 0;
    SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, flag, out.p, nsel.p, n, s));
    tmp_reserve(tb);
    SPH_HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, it, flag, out.p, nsel.p, n, s));
    return read_scalar(nsel.p);
  }

  // FixPhaseChange::pre_exchange (fix_phase_change.cpp:167-352) on the last build's full
  // list, owned atoms as integrated, ghosts as last communicated; the rebuild follows.
  // Bricks: every rank runs the call on its own atoms with its own RanPark of the same seed
  // (:116), creating atoms only inside its sub-box; the ghosts' dmass goes back over the
  // swaps (reverse_comm_fix, :324), and the created atoms take the next tags rank by rank
  // (MPI_Allreduce + Atom::tag_extend, :338-351).  A rank with no candidate still takes part
  // in the collectives (slot keys, reverse comm, counts) and in the finish loop.
  void phase_change() {
    Scope t(this, T_NEIGH);
    // (SPH_DEBUG: host time between the stages of this call)
    const bool dbg = env_int("SPH_DEBUG", 0) != 0;
    std::vector<std::pair<const char *, std::chrono::steady_clock::time_point>> tm;
    auto mark = [&](const char *w) {
      if (dbg) tm.emplace_back(w, std::chrono::steady_clock::now());
    };
    mark("start");
    if (!lidx_valid) lidx_from_tags();  // (read_restart: the file's tag order)
    const bool mul = multi();
    const int n = nlocal, nall = nlocal + nghost;
    if (n == 0 && !mul) return;
    sph_phasechange_params p = pcp;
    for (int k = 0; k < 3; k++) {
      p.sublo[k] = sublo[k];
      p.subhi[k] = subhi[k];
      p.boxhi[k] = box.hi[k];
      p.top[k] = myloc[k] == pg[k] - 1;
    }
    const PcDev pd{cfg.dim, p.from_type, p.to_type, p.Tc, p.to_mass, p.cutoff};
    DBuf<int> &flag = pc_flag, &cand = pc_cand, &otag = pc_otag, &idx = pc_idx;
    DBuf<double> &rec = pc_rec, &gat = pc_gat, &Wd = pc_Wd, &vals = pc_vals, &nrec = pc_nrec;
    int ncand = 0;
    if (n > 0) {
      flag.reserve(n);
      hipLaunchKernelGGL(k_pc_flags, dim3(blocks(n)), dim3(BLK), 0, s, n, (const int *)nullptr,
                         ty.p, en.p, cvv.p, pd, flag.p);
      ncand = select_flagged_i(flag.p, n, cand);
    }
    if (ncand == 0 && !mul) return;  // (dmass 0: the finish loop leaves rmass and e as they are)
    const int lst = strided ? list_stride : 0;
    PcRank rk{n, 1, nullptr};
    auto walk = [&](const PcRank &r) {
      hipLaunchKernelGGL(k_pc_candidates<8>, mp_rows(ncand), dim3(256), 0, s, ncand, cand.p,
                         (const int *)nullptr, off.p, nbr.p, xf.p, vr.p, (const double *)vel.p,
                         4, ty.p, rm.p, pd, rec.p, lst, ccnt.p, r, 0, 0, pc_minr.p);
    };
    std::vector<int> hm(ncand), hc(ncand), ht(ncand);
    std::vector<double> hr((size_t)8 * ncand), hg((size_t)9 * ncand);
    if (mul) {  // slot ranks first (collective), then one walk with them
      pc_ghost_slots_multi();
      rk = PcRank{n, 2, pc_grank.p};
    }
    if (ncand > 0) {
      rec.reserve((size_t)8 * ncand);
      gat.reserve((size_t)9 * ncand);
      otag.reserve(ncand);
      // one brick: the first pass screens -- every ghost ranks 0, so minr < NORANK flags the
      // candidates whose row holds a from_type ghost at all; only then are LAMMPS' ghost
      // slots worked out
      pc_minr.reserve(ncand);
      walk(rk);
      if (!mul) {
        SPH_HIP_TRY(hipMemcpyAsync(hm.data(), pc_minr.p, ncand * sizeof(int), hipMemcpyDeviceToHost, s));
        SPH_HIP_TRY(hipStreamSynchronize(s));
        if (std::any_of(hm.begin(), hm.end(), [](int v) { return v != PC_NORANK; })) {
          pc_ghost_slots();
          rk = PcRank{n, 2, pc_grank.p};
          walk(rk);
        }
      }
      hipLaunchKernelGGL(k_pc_gather, dim3(blocks(ncand)), dim3(BLK), 0, s, ncand, cand.p, xf.p,
                         vr.p, en.p, cvv.p, cg.p, lidx.p, gat.p, otag.p);
      SPH_HIP_TRY(hipMemcpyAsync(hm.data(), pc_minr.p, ncand * sizeof(int), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipMemcpyAsync(hc.data(), cand.p, ncand * sizeof(int), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipMemcpyAsync(ht.data(), otag.p, ncand * sizeof(int), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipMemcpyAsync(hr.data(), rec.p, hr.size() * sizeof(double), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipMemcpyAsync(hg.data(), gat.p, hg.size() * sizeof(double), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipStreamSynchronize(s));
    }
    mark("readback");
    // the reference meets the candidates in its local order (lidx: read order, exchange hole
    // fill, Atom::sort)
    std::vector<int> ord(ncand);
    for (int k = 0; k < ncand; k++) ord[k] = k;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return ht[a] < ht[b]; });
    std::vector<PcCand> cands(ncand);
    for (int q = 0; q < ncand; q++) {
      const int k = ord[q];
      PcCand &c = cands[q];
      const double *g = &hg[(size_t)9 * k];
      for (int d = 0; d < 3; d++) {
        c.x[d] = g[d];
        c.cg[d] = g[3 + d];
      }
      c.e = g[6];
      c.cv = g[7];
      c.rho = g[8];
      for (int d = 0; d < 8; d++) c.rec[d] = hr[(size_t)8 * k + d];
      c.minr = hm[k];
    }
    auto recompute = [&](size_t q, int dead_a, int dead_w, double *out) {
      pc_one.reserve(1);
      SPH_HIP_TRY(hipMemcpyAsync(pc_one.p, &hc[ord[q]], sizeof(int), hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_pc_candidates<8>, dim3(1), dim3(256), 0, s, 1, pc_one.p,
                         (const int *)nullptr, off.p, nbr.p, xf.p, vr.p, (const double *)vel.p,
                         4, ty.p, rm.p, pd, Wd.p, lst, ccnt.p, rk, dead_a, dead_w, (int *)nullptr);
      SPH_HIP_TRY(hipMemcpyAsync(out, Wd.p, 8 * sizeof(double), hipMemcpyDeviceToHost, s));
      SPH_HIP_TRY(hipStreamSynchronize(s));
    };
    Wd.reserve(8);
    std::vector<int> ins_k;
    std::vector<double> ins_rec, ins_W;
    mark("candidates");
    pc_replay(p, cfg.dim, pc_seed, cands, ins_k, ins_W, ins_rec, recompute);
    mark("replay");
    const int nins = (int)ins_k.size();
    // MPI_Allreduce(nins) and the tag base of this rank's created atoms (tag_extend: rank
    // order); the first call also agrees on the next free tag
    int ninsall = nins, tag0 = tag_next;
    if (mul) {
      std::vector<int> all(tr->size());
      if (!pc_tags_agreed) {
        tr->allgather_int(tag_next, all.data(), s);
        tag_next = *std::max_element(all.begin(), all.end());
        pc_tags_agreed = true;
      }
      tr->allgather_int(nins, all.data(), s);
      ninsall = 0;
      tag0 = tag_next;
      for (int r = 0; r < (int)all.size(); r++) {
        if (r < tr->rank()) tag0 += all[r];
        ninsall += all[r];
      }
    }
    if (nins == 0 && !mul) return;
    std::vector<int> hidx(nins);
    std::vector<double> hval(nins), hW(nins);
    for (int q = 0; q < nins; q++) {
      const int k = ord[ins_k[q]];
      hidx[q] = hc[k];  // the candidate's row = its atom (identity row list)
      hval[q] = ins_rec[(size_t)13 * q + 9];
      hW[q] = ins_W[q];
    }
    dmass.reserve(nall > 0 ? nall : 1);
    mark("host");
    if (nall) SPH_HIP_TRY(hipMemsetAsync(dmass.p, 0, nall * sizeof(double), s));
    if (nins) {
      idx.reserve(nins);
      vals.reserve(nins);
      Wd.reserve(nins);
      nrec.reserve((size_t)13 * nins);
      SPH_HIP_TRY(hipMemcpyAsync(idx.p, hidx.data(), nins * sizeof(int), hipMemcpyHostToDevice, s));
      SPH_HIP_TRY(hipMemcpyAsync(vals.p, hval.data(), nins * sizeof(double), hipMemcpyHostToDevice, s));
      SPH_HIP_TRY(hipMemcpyAsync(Wd.p, hW.data(), nins * sizeof(double), hipMemcpyHostToDevice, s));
      SPH_HIP_TRY(hipMemcpyAsync(nrec.p, ins_rec.data(), ins_rec.size() * sizeof(double), hipMemcpyHostToDevice, s));
      // e_i = (e_i - Hwv)/2 of the atoms that changed phase, the donors' dmass
      hipLaunchKernelGGL(k_pc_set_e, dim3(blocks(nins)), dim3(BLK), 0, s, nins, idx.p, vals.p, en.p);
      // (in candidate order per donor: the reference's sum, fix_phase_change.cpp:289-299)
      const long long cap = (long long)nins * std::max(lst > 0 ? lst : nbr_maxrow, 1);
      pc_dmass_ordered<8>(s, nins, idx.p, Wd.p, (const int *)nullptr, off.p, nbr.p, xf.p, ty.p,
                          rm.p, pd, lst, ccnt.p, rk, cap, pc_k0, pc_k1, pc_v0, pc_v1, pc_cnt,
                          tmp, dmass.p);
    }
    // its reverse comm, rmass -= dmass and e renormalised, then the new atoms
    reverse1(dmass.p);
    if (n)
      hipLaunchKernelGGL(k_pc_finish, dim3(blocks(n)), dim3(BLK), 0, s, n, dmass.p, rm.p, en.p);
    if (nins) {
      ensure_atoms((size_t)n + nins, true);  // (over the ghost slots: the rebuild follows)
      vel.reserve((size_t)n + nins, true, s);
      tag.reserve((size_t)n + nins, true, s);
      fo.reserve((size_t)n + nins, true, s);
      de.reserve((size_t)n + nins, true, s);
      hipLaunchKernelGGL(k_pc_append, dim3(blocks(nins)), dim3(BLK), 0, s, nins, nrec.p, n,
                         p.to_type, tag0, xf.p, vr.p, vel.p, en.p, rm.p, cvv.p, cg.p, ty.p,
                         tag.p, fo.p, de.p);
      lidx.reserve((size_t)n + nins, true, s);  // (create_atom: at the end, in creation order)
      hipLaunchKernelGGL(k_lidx_iota, dim3(blocks(nins)), dim3(BLK), 0, s, nins, n, lidx.p + n);
    }
    SPH_HIP_TRY(hipStreamSynchronize(s));  // (the host staging vectors go out of scope)
    mark("end");
    if (dbg) {
      fprintf(stderr, "[sph] phase change: %d candidates, %d inserted;", ncand, nins);
      for (size_t k = 1; k < tm.size(); k++)
        fprintf(stderr, " %s %.1f us", tm[k].first,
                std::chrono::duration<double, std::micro>(tm[k].second - tm[k - 1].second).count());
      fprintf(stderr, "\n");
    }
    if (ninsall == 0) return;  // (natoms unchanged: the ghosts stay, the rebuild follows)
    nlocal = n + nins;
    nghost = 0;
    tag_next += ninsall;
    pc_inserted += nins;
  }

  bool rhosum_due() const {
    return cfg.rhosum_nstep > 0 && (step % cfg.rhosum_nstep) == 0;
  }

  // Verlet::setup (verlet.cpp:88-139)
  void setup() {
    step = 0;
    Scope t(this, T_NEIGH);
    if (pc) {  // (every setup sorts: verlet.cpp:106)
      if (!lidx_valid) lidx_from_tags();
      nextsort = 0;
    }
    // borders() runs before setup_pre_force: ghosts carry vest as it was (reference order);
    // the setup force pass needs the global-index list for its half-list walk
    build_all(true);
    vso.reserve(nlocal > 0 ? nlocal : 1);  // (vest before setup_pre_force: setup_forces_full)
    if (nlocal)
      SPH_HIP_TRY(hipMemcpyAsync(vso.p, vr.p, (size_t)nlocal * sizeof(double4),
                                 hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_vest_from_v, dim3(blocks(nlocal)), dim3(BLK), 0, s, nlocal,
                       cfg.stationary_mask, ty.p, vel.p, vr.p);
    pair_compute(rhosum_due(), /*setup=*/true);
    last_build = 0;
    setup_done = true;
  }

  // Verlet::run (verlet.cpp:222-308)
  void run(int nsteps) {
    // the final_integrate of step k-1 runs fused with the initial_integrate of step k;
    // the last step's final_integrate runs on its own after the loop
    for (int k = 0; k < nsteps; k++) {
      step++;
      if (sc.x0) sc.moved = moved_flag();
      {
        Scope t(this, T_INT);
        if (k == 0)
          hipLaunchKernelGGL(k_initial_integrate, dim3(blocks(nlocal)), dim3(BLK), 0, s,
                             nlocal, sc, xf.p, vr.p, en.p, ty.p, vel.p, fo.p, de.p, rm.p);
        else
          hipLaunchKernelGGL(k_final_initial, dim3(blocks(nlocal)), dim3(BLK), 0, s, nlocal,
                             sc, xf.p, vr.p, en.p, ty.p, vel.p, fo.p, de.p, rm.p);
      }
      const int every = cfg.neigh_every > 0 ? cfg.neigh_every : 1;
      const bool pc_due = pc && step == pc_next;  // (the fix forces this reneighbor)
      if (pc_due) {
        phase_change();
        pc_next += pc_nevery;
      }
      if (pc_due || (step - last_build) % every == 0) {
        rebuild();
        last_build = (int)step;
        pair_compute(rhosum_due());
      } else if (ov_ready && rhosum_due() && overlap_on()) {
        pair_compute_overlap();
      } else {
        forward();
        pair_compute(rhosum_due());
      }
      refresh_inner(!pc && (step + 1 - last_build) % every == 0);
      if (timing && pending.size() > 4096) harvest();
    }
    if (nsteps > 0) {
      Scope t(this, T_INT);
      hipLaunchKernelGGL(k_final_integrate, dim3(blocks(nlocal)), dim3(BLK), 0, s, nlocal, sc,
                         vr.p, en.p, ty.p, vel.p, fo.p, de.p, rm.p);
    }
    SPH_HIP_TRY(hipGetLastError());
  }
};

// MpCoefs of the multiphase stack from the engine's (SPH_MAXTYPES+1)^2 tables (upper
// triangle mirrored like init_one; the coeff() formulas as sph_multiphase.hip's), and the
// stack's cutoffs into cutmax ((nt+1)^2, upper triangle)
static void coef_mp(MpCoefs &m, const sph_engine_mp_config &c, int dim, int nt,
                    std::vector<double> &cutmax) {
  const int n1 = nt + 1, M1 = SPH_MAXTYPES + 1;
  m = MpCoefs{};
  m.ntypes = nt;
  m.dim = dim;
  auto up = [&](const double *t, int i, int j) { return j >= i ? t[i * M1 + j] : t[j * M1 + i]; };
  auto upi = [&](const int *t, int i, int j) { return j >= i ? t[i * M1 + j] : t[j * M1 + i]; };
  auto cut = [&](bool on, const double *t) {
    if (!on) return;
    for (int i = 0; i <= nt; i++)
      for (int j = i; j <= nt; j++) cutmax[i * n1 + j] = std::max(cutmax[i * n1 + j], t[i * M1 + j]);
  };
  for (int i = 0; i <= nt; i++)
    for (int j = 0; j <= nt; j++) {
      const int k = i * n1 + j;
      m.rcut[k] = up(c.rhosum_cut, i, j);
      m.rcutsq[k] = m.rcut[k] * m.rcut[k];
      m.calpha[k] = up(c.cg_alpha, i, j);
      m.ccut[k] = up(c.cg_cut, i, j);
      m.ccutsq[k] = m.ccut[k] * m.ccut[k];
      m.tvisc[k] = up(c.tait_visc, i, j);
      m.tcut[k] = up(c.tait_cut, i, j);
      m.tcutsq[k] = m.tcut[k] * m.tcut[k];
      m.scut[k] = up(c.st_cut, i, j);
      m.scutsq[k] = m.scut[k] * m.scut[k];
      m.halpha[k] = up(c.heat_alpha, i, j);
      m.hcut[k] = up(c.heat_cut, i, j);
      m.hcutsq[k] = m.hcut[k] * m.hcut[k];
      m.htc[k] = up(c.heat_tc, i, j);
      m.hfix[k] = upi(c.heat_fixflag, i, j);
    }
  if (c.tait_on)
    for (int t = 1; t <= nt; t++) {
      SPH_REQUIRE(c.gamma[t] != 0.0 && c.rho0[t] != 0.0, SPH_HIP_EINVAL,
                  "type %d: gamma and rho0 must be non-zero", t);
      m.rho0[t] = c.rho0[t];
      m.gamma[t] = c.gamma[t];
      m.rbg[t] = c.rbackground[t];
      // B = c^2 rho0 / gamma, pair_sph_taitwater_multiphase.cpp:243-250
      m.B[t] = c.soundspeed[t] * c.soundspeed[t] * c.rho0[t] / c.gamma[t];
    }
  cut(c.rhosum_nstep > 0, c.rhosum_cut);
  cut(c.cg_nstep > 0, c.cg_cut);
  cut(c.tait_on != 0, c.tait_cut);
  cut(c.st_on != 0, c.st_cut);
  cut(c.heat_on != 0, c.heat_cut);
}

extern "C" {

int sph_engine_create(int device, const sph_engine_config *cfg, sph_engine **out) {
  SPH_API_BEGIN
  SPH_REQUIRE(cfg && out, SPH_HIP_EINVAL, "sph_engine_create: NULL argument");
  g_alloc_log = env_int("SPH_ALLOC_LOG", 0);
  SPH_REQUIRE(cfg->dim == 2 || cfg->dim == 3, SPH_HIP_EINVAL, "dimension must be 2 or 3");
  SPH_REQUIRE(cfg->ntypes >= 1 && cfg->ntypes <= SPH_MAXTYPES, SPH_HIP_EINVAL,
              "ntypes %d outside [1,%d]", cfg->ntypes, SPH_MAXTYPES);
  const int pgn = cfg->procgrid[0] * cfg->procgrid[1] * cfg->procgrid[2];
  SPH_REQUIRE(pgn == 0 || (cfg->procgrid[0] >= 1 && cfg->procgrid[1] >= 1 &&
                           cfg->procgrid[2] >= 1 && cfg->rank >= 0 && cfg->rank < pgn),
              SPH_HIP_EINVAL, "bad procgrid %dx%dx%d / rank %d", cfg->procgrid[0],
              cfg->procgrid[1], cfg->procgrid[2], cfg->rank);
  SPH_REQUIRE(pgn <= 1 || cfg->dim == 3 || cfg->procgrid[2] == 1, SPH_HIP_EINVAL,
              "2-D runs cannot split z");
  require_device(device);
  sph_engine *e = new sph_engine;
  try {
    e->device = device;
    e->cfg = *cfg;
    const int nt = cfg->ntypes;
    Coefs &c = e->hc;
    c.ntypes = nt;
    c.dim = cfg->dim;
    // the body-force mass: the types of the gravity fix's group (gravity_mask, 0 = all)
    for (int t = 0; t <= nt; t++)
      c.mass[t] = (cfg->gravity_mask == 0 || ((cfg->gravity_mask >> t) & 1)) ? cfg->mass[t] : 0.0;
    // per-type-pair tables are passed in the engine's fixed (SPH_MAXTYPES+1)^2 layout
    auto repack = [&](const double *src, std::vector<double> &dst) {
      dst.assign((nt + 1) * (nt + 1), 0.0);
      for (int i = 0; i <= nt; i++)
        for (int j = 0; j <= nt; j++) dst[i * (nt + 1) + j] = src[i * (SPH_MAXTYPES + 1) + j];
    };
    std::vector<double> cutmax((nt + 1) * (nt + 1), 0.0), tmpv, tmpc;
    if (cfg->rhosum_nstep > 0) {
      repack(cfg->rhosum_cut, tmpc);
      coef_rhosum(c, cfg->dim, nt, tmpc.data(), cfg->mass);
      for (size_t k = 0; k < cutmax.size(); k++) cutmax[k] = std::max(cutmax[k], tmpc[k]);
    }
    if (cfg->tait_on) {
      repack(cfg->tait_cut, tmpc);
      repack(cfg->tait_visc_coef, tmpv);
      coef_tait(c, cfg->dim, nt, cfg->tait_visc, cfg->rho0, cfg->soundspeed, cfg->B,
                tmpv.data(), tmpc.data(), cfg->mass);
      for (size_t k = 0; k < cutmax.size(); k++) cutmax[k] = std::max(cutmax[k], tmpc[k]);
      e->force_mode |= M_TAIT;
    }
    if (cfg->heat_on) {
      repack(cfg->heat_cut, tmpc);
      repack(cfg->heat_alpha, tmpv);
      coef_heat(c, cfg->dim, nt, tmpv.data(), tmpc.data(), cfg->mass);
      for (size_t k = 0; k < cutmax.size(); k++) cutmax[k] = std::max(cutmax[k], tmpc[k]);
      e->force_mode |= M_HEAT;
    }
    if (cfg->mp) {
      SPH_REQUIRE(cfg->rhosum_nstep == 0 && !cfg->tait_on && !cfg->heat_on, SPH_HIP_EINVAL,
                  "the multiphase stack replaces the single-phase styles (turn them off)");
      e->mp = true;
      e->mpc = *cfg->mp;
      e->cfg.mp = nullptr;
      coef_mp(e->hm, e->mpc, cfg->dim, nt, cutmax);
    }
    // mirror upper triangle into a symmetric max-cut table (init_one semantics)
    for (int i = 1; i <= nt; i++)
      for (int j = 1; j < i; j++) cutmax[i * (nt + 1) + j] = cutmax[j * (nt + 1) + i];
    // inner rows of the block path (sph_blk_kernels.h k_blk_inner): a sixteenth of the skin
    // -- rows of ~110 instead of ~120 entries at C2 (with 16-entry walk chunks 114.5 instead
    // of 128 pair evaluations), valid while no atom has moved skin/32 since the build
    e->inner_margin = SPH_INNER_FRAC * cfg->skin;
    e->cutneighmax = coef_cutneigh(c, nt, cutmax.data(), cfg->skin, e->inner_margin);
    for (int k = 0; k < NT2; k++)  // tight-list test: the largest force-style cutoff
      c.fcutsq[k] = std::max((e->force_mode & M_TAIT) ? c.tait[k].cutsq : 0.0,
                             (e->force_mode & M_HEAT) ? c.heat[k].cutsq : 0.0);
    SPH_REQUIRE(e->cutneighmax > 0.0, SPH_HIP_EINVAL, "no pair style enabled / zero cutoff");
    e->cutghost = e->cutneighmax;  // CommBrick::setup: cutghost = cutneighmax (:166)
    if (pgn > 1) {
      for (int k = 0; k < 3; k++) e->pg[k] = cfg->procgrid[k];
      e->nprocs = pgn;
      e->me = cfg->rank;
    }
    // brick of this rank, x fastest (Domain::set_local_box with uniform xsplit, domain.cpp)
    e->myloc[0] = e->me % e->pg[0];
    e->myloc[1] = (e->me / e->pg[0]) % e->pg[1];
    e->myloc[2] = e->me / (e->pg[0] * e->pg[1]);
    for (int k = 0; k < 3; k++) {
      e->box.lo[k] = cfg->boxlo[k];
      e->box.hi[k] = cfg->boxhi[k];
      e->box.prd[k] = cfg->boxhi[k] - cfg->boxlo[k];
      e->box.periodic[k] = (k < cfg->dim) ? cfg->periodic[k] : 0;
      const double lo = (double)e->myloc[k] / e->pg[k], hi = (double)(e->myloc[k] + 1) / e->pg[k];
      e->sublo[k] = cfg->boxlo[k] + e->box.prd[k] * lo;
      e->subhi[k] = (e->myloc[k] + 1 == e->pg[k]) ? cfg->boxhi[k]
                                                   : cfg->boxlo[k] + e->box.prd[k] * hi;
      auto at = [&](int dx, int dy, int dz) {
        const int l[3] = {(e->myloc[0] + dx + e->pg[0]) % e->pg[0],
                          (e->myloc[1] + dy + e->pg[1]) % e->pg[1],
                          (e->myloc[2] + dz + e->pg[2]) % e->pg[2]};
        return (l[2] * e->pg[1] + l[1]) * e->pg[0] + l[0];
      };
      e->procneigh[k][0] = at(k == 0 ? -1 : 0, k == 1 ? -1 : 0, k == 2 ? -1 : 0);
      e->procneigh[k][1] = at(k == 0 ? 1 : 0, k == 1 ? 1 : 0, k == 2 ? 1 : 0);
      if (e->box.periodic[k])
        SPH_REQUIRE(e->cutghost < e->box.prd[k], SPH_HIP_EINVAL,
                    "ghost cutoff %g >= box length %g in dim %d (multi-hop borders unsupported)",
                    e->cutghost, e->box.prd[k], k);
      if (e->pg[k] > 1)  // CommBrick maxneed = 1: a brick must be wider than the ghost cut
        SPH_REQUIRE(e->cutghost < e->subhi[k] - e->sublo[k], SPH_HIP_EINVAL,
                    "ghost cutoff %g >= brick width %g in dim %d (multi-hop swaps unsupported)",
                    e->cutghost, e->subhi[k] - e->sublo[k], k);
    }
    e->sc.dtv = cfg->dt;
    e->sc.dtf = 0.5 * cfg->dt * (cfg->ftm2v > 0 ? cfg->ftm2v : 1.0);  // fix_meso.cpp:63-66
    for (int t = 0; t <= nt; t++) e->sc.mass[t] = cfg->mass[t];
    e->sc.stationary_mask = cfg->stationary_mask;
    e->setup_bins_geometry();
    SPH_HIP_TRY(hipStreamCreateWithFlags(&e->s, hipStreamNonBlocking));
    SPH_HIP_TRY(hipMalloc(&e->dc, sizeof(Coefs)));
    SPH_HIP_TRY(hipMemcpy(e->dc, &e->hc, sizeof(Coefs), hipMemcpyHostToDevice));
    if (e->mp) {
      SPH_HIP_TRY(hipMalloc(&e->dm, sizeof(MpCoefs)));
      mp_inverses(e->hm);
      SPH_HIP_TRY(hipMemcpy(e->dm, &e->hm, sizeof(MpCoefs), hipMemcpyHostToDevice));
    }
    SPH_HIP_TRY(hipHostMalloc(&e->h_scalar, sizeof(int)));
    SPH_HIP_TRY(hipHostMalloc(&e->h_small, 16 * sizeof(int)));
  } catch (...) {
    delete e;
    throw;
  }
  e->overlap = false;
  *out = e;
  SPH_API_END
}

int sph_engine_destroy(sph_engine *e) {
  if (!e) return SPH_HIP_OK;
  (void)hipSetDevice(e->device);
  if (e->s) (void)hipStreamSynchronize(e->s);
  if (e->s2) (void)hipStreamSynchronize(e->s2);
  for (auto *b : {&e->xf, &e->vr, &e->vel, &e->fo, &e->xf2, &e->vr2, &e->vel2, &e->xb}) b->release();
  for (auto *b : {&e->en, &e->en2, &e->de, &e->rm, &e->cvv, &e->rho_tmp, &e->dmass, &e->xbuf,
                  &e->xbuf2})
    b->release();
  for (auto *b : {&e->rhoS, &e->rhoF}) b->release();
  for (auto *b : {&e->cg, &e->cgS, &e->cgF, &e->recA, &e->recK, &e->recF, &e->recS}) b->release();
  if (e->dm) (void)hipFree(e->dm);
  for (auto *b : {&e->nbs, &e->gorank, &e->goidx, &e->dr_sidx, &e->dr_rslot, &e->dr_self, &e->dr_req, &e->dr_byq, &e->dr_byg, &e->dr_hist, &e->pc_flag,
                  &e->pc_cand, &e->pc_otag, &e->pc_idx})
    b->release();
  for (auto *b : {&e->pc_rec, &e->pc_gat, &e->pc_Wd, &e->pc_vals, &e->pc_nrec, &e->pc_v0,
                  &e->pc_v1})
    b->release();
  e->pc_k0.release();
  e->pc_k1.release();
  e->pc_cnt.release();
  for (auto *b : {&e->ty, &e->ty2, &e->tag, &e->tag2, &e->gowner, &e->gimg, &e->sel, &e->nsel,
                  &e->bidx, &e->bidx2, &e->cnt, &e->off, &e->nbr, &e->mx,
                  &e->ccnt, &e->pcnt, &e->qbeg, &e->tb, &e->xpos, &e->sel2, &e->rows_in, &e->rows_bd, &e->tnbr,
                  &e->tcnt, &e->ulist, &e->ucnt, &e->kcnt, &e->uilist, &e->uicnt})
    b->release();
  for (auto *b : {&e->bkey, &e->bkey2}) b->release();
  for (auto *b : {&e->flags, &e->tmp, &e->cbs, &e->cbr, &e->flag2, &e->fl_in, &e->fl_bd}) b->release();
  e->snbr.release();
  e->snbi.release();
  e->icnt.release();
  e->moved.release();
  e->x0.release();
  e->blen.release();
  for (auto &sw : e->swaps) sw.list.release();
  for (auto &p : e->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto ev : e->evpool) (void)hipEventDestroy(ev);
  if (e->h_scalar) (void)hipHostFree(e->h_scalar);
  if (e->h_small) (void)hipHostFree(e->h_small);
  delete e->tr;
  if (e->dc) (void)hipFree(e->dc);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  if (e->s2) (void)hipStreamDestroy(e->s2);
  if (e->s) (void)hipStreamDestroy(e->s);
  delete e;
  return SPH_HIP_OK;
}

int sph_engine_set_atoms(sph_engine *e, int n, const double *x, const double *v,
                         const int *type, const double *rho, const double *en,
                         const double *cv) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && n >= 0 && (n == 0 || (x && v && type && rho)), SPH_HIP_EINVAL,
              "sph_engine_set_atoms: bad argument");
  SPH_HIP_TRY(hipSetDevice(e->device));
  for (int i = 0; i < n; i++)
    SPH_REQUIRE(type[i] >= 1 && type[i] <= e->cfg.ntypes, SPH_HIP_EINVAL,
                "atom %d has type %d outside [1,%d]", i, type[i], e->cfg.ntypes);
  e->nlocal = n;
  e->nghost = 0;
  e->tag_next = n;
  e->pc_tags_agreed = false;
  e->pc_inserted = 0;
  e->cv_by_tag.assign(n, 1.0);
  if (cv)
    for (int i = 0; i < n; i++) e->cv_by_tag[i] = cv[i];
  e->ensure_atoms(n > 0 ? n : 1, false);
  e->vel.reserve(n > 0 ? n : 1);
  e->fo.reserve(n > 0 ? n : 1);
  e->de.reserve(n > 0 ? n : 1);
  e->tag.reserve(n > 0 ? n : 1);
  std::vector<double4> hx(n), hv(n), hvel(n);
  std::vector<double> he(n);
  std::vector<int> ht(n), hty(n);
  for (int i = 0; i < n; i++) {
    hx[i] = make_double4(x[3 * i], x[3 * i + 1], x[3 * i + 2], 0.0);
    hv[i] = make_double4(0.0, 0.0, 0.0, rho[i]);  // vest = 0 until setup_pre_force
    hvel[i] = make_double4(v[3 * i], v[3 * i + 1], v[3 * i + 2], (double)IMG_ZERO);
    he[i] = en ? en[i] : 0.0;
    ht[i] = i;
    hty[i] = type[i];
  }
  if (n > 0) {
    SPH_HIP_TRY(hipMemcpyAsync(e->xf.p, hx.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->vr.p, hv.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->vel.p, hvel.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->en.p, he.data(), n * sizeof(double), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->ty.p, hty.data(), n * sizeof(int), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->tag.p, ht.data(), n * sizeof(int), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemsetAsync(e->fo.p, 0, n * sizeof(double4), e->s));
    SPH_HIP_TRY(hipMemsetAsync(e->de.p, 0, n * sizeof(double), e->s));
  }
  // LAMMPS' local order starts as the read order (data-file lines / create_atoms), which is
  // the order handed here -- not necessarily tag order (sph_engine_set_tags may permute)
  e->lidx.reserve(n > 0 ? n : 1);
  if (n > 0) hipLaunchKernelGGL(k_lidx_iota, dim3(blocks(n)), dim3(BLK), 0, e->s, n, 0, e->lidx.p);
  e->lidx_valid = true;
  if (e->mp && n > 0) {  // per-type mass, cv (default 1, create_atom), colorgradient 0
    std::vector<double> hm(n), hc(n);
    for (int i = 0; i < n; i++) {
      hm[i] = e->cfg.mass[type[i]];
      hc[i] = cv ? cv[i] : 1.0;
    }
    SPH_HIP_TRY(hipMemcpyAsync(e->rm.p, hm.data(), n * sizeof(double), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->cvv.p, hc.data(), n * sizeof(double), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemsetAsync(e->cg.p, 0, n * sizeof(double4), e->s));
  }
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  e->setup_done = false;
  SPH_API_END
}

int sph_engine_set_atoms_multiphase(sph_engine *e, const double *rmass, const double *cv,
                                    const double *cg) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && e->mp, SPH_HIP_EINVAL,
              "sph_engine_set_atoms_multiphase: not a multiphase engine (cfg.mp)");
  const int n = e->nlocal;
  SPH_REQUIRE(n == 0 || rmass, SPH_HIP_EINVAL, "sph_engine_set_atoms_multiphase: NULL rmass");
  SPH_HIP_TRY(hipSetDevice(e->device));
  if (n == 0) return SPH_HIP_OK;
  for (int i = 0; i < n; i++)
    SPH_REQUIRE(rmass[i] > 0.0, SPH_HIP_EINVAL, "atom %d has rmass %g <= 0", i, rmass[i]);
  std::vector<double> hc(n, 1.0);
  std::vector<double4> hg(n, make_double4(0.0, 0.0, 0.0, 0.0));
  for (int i = 0; i < n; i++) {
    if (cv) hc[i] = cv[i];
    if (cg) hg[i] = make_double4(cg[3 * i], cg[3 * i + 1], cg[3 * i + 2], 0.0);
  }
  SPH_HIP_TRY(hipMemcpyAsync(e->rm.p, rmass, n * sizeof(double), hipMemcpyHostToDevice, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(e->cvv.p, hc.data(), n * sizeof(double), hipMemcpyHostToDevice, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(e->cg.p, hg.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->s));
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  e->setup_done = false;
  SPH_API_END
}

int sph_engine_phase_change(sph_engine *e, const sph_phasechange_params *p, int nevery,
                            int seed) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && p, SPH_HIP_EINVAL, "sph_engine_phase_change: NULL argument");
  SPH_REQUIRE(e->mp, SPH_HIP_EINVAL,
              "fix phase_change needs atom_style meso/multiphase (a multiphase engine)");
  SPH_REQUIRE(seed > 0, SPH_HIP_EINVAL, "Invalid seed for Park random # generator");
  SPH_REQUIRE(!e->setup_done, SPH_HIP_EINVAL,
              "sph_engine_phase_change: arm the fix before sph_engine_setup (its local-order "
              "bookkeeping starts at set_atoms)");
  SPH_REQUIRE(nevery >= 1, SPH_HIP_EINVAL, "sph_engine_phase_change: nevery < 1");
  SPH_REQUIRE(p->to_mass > 0.0 && p->maxattempt >= 1 && p->cutoff > 0.0, SPH_HIP_EINVAL,
              "sph_engine_phase_change: bad parameters");
  SPH_REQUIRE(p->from_type >= 1 && p->from_type <= e->cfg.ntypes && p->to_type >= 1 &&
                  p->to_type <= e->cfg.ntypes,
              SPH_HIP_EINVAL, "sph_engine_phase_change: type outside [1,%d]", e->cfg.ntypes);
  e->pc = true;
  e->pcp = *p;
  e->pcp.dt = e->cfg.dt;
  e->pc_nevery = nevery;
  e->pc_seed = seed;
  e->pc_next = e->step + 1;  // next_reneighbor = ntimestep + 1 (fix_phase_change.cpp:120)
  SPH_API_END
}

int sph_engine_get_atoms_multiphase(sph_engine *e, double *rmass, double *cv, double *cg,
                                    double *vest, int *type, int64_t *ninserted) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_get_atoms_multiphase: NULL engine");
  SPH_HIP_TRY(hipSetDevice(e->device));
  if (ninserted) *ninserted = e->pc_inserted;
  const int n = e->nlocal;
  if (n == 0) return SPH_HIP_OK;
  std::vector<double> hm(n, 0.0), hc(n, 1.0);
  std::vector<double4> hg(n, make_double4(0, 0, 0, 0)), hv(n);
  std::vector<int> ht(n), hty(n);
  if (e->mp) {
    SPH_HIP_TRY(hipMemcpyAsync(hm.data(), e->rm.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(hc.data(), e->cvv.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(hg.data(), e->cg.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  }
  SPH_HIP_TRY(hipMemcpyAsync(hv.data(), e->vr.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hty.data(), e->ty.p, n * sizeof(int), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(ht.data(), e->tag.p, n * sizeof(int), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  const bool local_order = e->multi() || e->global_tags;
  for (int i = 0; i < n; i++) {
    const int t = local_order ? i : ht[i];
    SPH_REQUIRE(t >= 0 && t < n, SPH_HIP_ERUNTIME, "corrupt tag %d", t);
    if (rmass) rmass[t] = e->mp ? hm[i] : e->cfg.mass[hty[i]];
    if (cv) cv[t] = hc[i];
    if (cg) {
      cg[3 * t] = hg[i].x;
      cg[3 * t + 1] = hg[i].y;
      cg[3 * t + 2] = hg[i].z;
    }
    if (vest) {
      vest[3 * t] = hv[i].x;
      vest[3 * t + 1] = hv[i].y;
      vest[3 * t + 2] = hv[i].z;
    }
    if (type) type[t] = hty[i];
  }
  SPH_API_END
}

// LAMMPS ubuf (lmptype.h): an integer stored as the bit pattern of an int64 in a double
static double ubuf_d(int64_t v) {
  double d;
  memcpy(&d, &v, sizeof d);
  return d;
}
static int64_t ubuf_i(double d) {
  int64_t v;
  memcpy(&v, &d, sizeof v);
  return v;
}

int sph_engine_write_restart(sph_engine *e, double *buf, int64_t cap, int *rec_size) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_write_restart: NULL engine");
  SPH_REQUIRE(!e->multi() && !e->global_tags, SPH_HIP_EINVAL,
              "sph_engine_write_restart: one brick with implicit tags");
  const int rec = e->mp ? 21 : 17;
  if (rec_size) *rec_size = rec;
  if (!buf) return SPH_HIP_OK;
  const int n = e->nlocal;
  SPH_REQUIRE(cap >= (int64_t)n * rec, SPH_HIP_EINVAL,
              "sph_engine_write_restart: buffer of %lld doubles < %lld", (long long)cap,
              (long long)n * rec);
  if (n == 0) return SPH_HIP_OK;
  SPH_HIP_TRY(hipSetDevice(e->device));
  std::vector<double4> hx(n), hv(n), hr(n), hg(n, make_double4(0, 0, 0, 0));
  std::vector<double> he(n), hm(n, 0.0), hc(n, 1.0);
  std::vector<int> ht(n), hty(n);
  SPH_HIP_TRY(hipMemcpyAsync(hx.data(), e->xf.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hv.data(), e->vel.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hr.data(), e->vr.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(he.data(), e->en.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hty.data(), e->ty.p, n * sizeof(int), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(ht.data(), e->tag.p, n * sizeof(int), hipMemcpyDeviceToHost, e->s));
  if (e->mp) {
    SPH_HIP_TRY(hipMemcpyAsync(hm.data(), e->rm.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(hc.data(), e->cvv.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(hg.data(), e->cg.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  }
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  for (int i = 0; i < n; i++) {
    const int t = ht[i];
    SPH_REQUIRE(t >= 0 && t < n, SPH_HIP_ERUNTIME, "corrupt tag %d", t);
    const double cv = e->mp ? hc[i] : (t < (int)e->cv_by_tag.size() ? e->cv_by_tag[t] : 1.0);
    double *o = buf + (size_t)rec * t;
    const int img = (int)hv[i].w;
    int m = 0;
    o[m++] = rec;
    o[m++] = hx[i].x;
    o[m++] = hx[i].y;
    o[m++] = hx[i].z;
    if (e->mp) {  // plain doubles (atom_vec_meso_multiphase.cpp:892-895)
      o[m++] = t + 1;
      o[m++] = hty[i];
      o[m++] = 1;
      o[m++] = img;
    } else {  // ubuf bit patterns (atom_vec_meso.cpp:731-734)
      o[m++] = ubuf_d(t + 1);
      o[m++] = ubuf_d(hty[i]);
      o[m++] = ubuf_d(1);
      o[m++] = ubuf_d(img);
    }
    o[m++] = hv[i].x;
    o[m++] = hv[i].y;
    o[m++] = hv[i].z;
    o[m++] = hr[i].w;
    if (e->mp) {
      o[m++] = hg[i].x;
      o[m++] = hg[i].y;
      o[m++] = hg[i].z;
      o[m++] = hm[i];
    }
    o[m++] = he[i];
    o[m++] = cv;
    o[m++] = hr[i].x;
    o[m++] = hr[i].y;
    o[m++] = hr[i].z;
  }
  SPH_API_END
}

int sph_engine_read_restart(sph_engine *e, int n, const double *buf) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && n >= 0 && (n == 0 || buf), SPH_HIP_EINVAL,
              "sph_engine_read_restart: bad argument");
  SPH_REQUIRE(!e->multi(), SPH_HIP_EINVAL, "sph_engine_read_restart: one brick");
  const int rec = e->mp ? 21 : 17;
  std::vector<double> x(3 * (size_t)n), v(3 * (size_t)n), vest(3 * (size_t)n), rho(n), en(n),
      cv(n), rm(n), cg(3 * (size_t)n);
  std::vector<int> type(n), img(n), seen(n, 0);
  for (int k = 0; k < n; k++) {
    const double *o = buf + (size_t)rec * k;
    SPH_REQUIRE((int)o[0] == rec, SPH_HIP_EINVAL,
                "record %d has %g values, this engine's layout has %d", k, o[0], rec);
    int64_t tg, ty, im;
    if (e->mp) {
      tg = (int64_t)o[4];
      ty = (int64_t)o[5];
      im = (int64_t)o[7];
    } else {
      tg = ubuf_i(o[4]);
      ty = ubuf_i(o[5]);
      im = ubuf_i(o[7]);
    }
    SPH_REQUIRE(tg >= 1 && tg <= n && !seen[tg - 1], SPH_HIP_EINVAL,
                "record %d: tag %lld is not a new one of 1..%d", k, (long long)tg, n);
    const int i = (int)tg - 1;
    seen[i] = 1;
    type[i] = (int)ty;
    img[i] = (int)im;
    int m = 8;
    for (int d = 0; d < 3; d++) {
      x[3 * i + d] = o[1 + d];
      v[3 * i + d] = o[m++];
    }
    rho[i] = o[m++];
    if (e->mp) {
      for (int d = 0; d < 3; d++) cg[3 * i + d] = o[m++];
      rm[i] = o[m++];
    }
    en[i] = o[m++];
    cv[i] = o[m++];
    for (int d = 0; d < 3; d++) vest[3 * i + d] = o[m++];
  }
  int rc = sph_engine_set_atoms(e, n, x.data(), v.data(), type.data(), rho.data(), en.data(),
                                cv.data());
  if (rc != SPH_HIP_OK) return rc;
  if (e->mp) {
    rc = sph_engine_set_atoms_multiphase(e, rm.data(), cv.data(), cg.data());
    if (rc != SPH_HIP_OK) return rc;
  }
  if (n > 0) {  // vest and the image flags, which set_atoms does not take
    std::vector<double4> hr(n), hv(n);
    for (int i = 0; i < n; i++) {
      hr[i] = make_double4(vest[3 * i], vest[3 * i + 1], vest[3 * i + 2], rho[i]);
      hv[i] = make_double4(v[3 * i], v[3 * i + 1], v[3 * i + 2], (double)img[i]);
    }
    SPH_HIP_TRY(hipMemcpyAsync(e->vr.p, hr.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipMemcpyAsync(e->vel.p, hv.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->s));
    SPH_HIP_TRY(hipStreamSynchronize(e->s));
  }
  SPH_API_END
}

int sph_engine_setup(sph_engine *e) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_setup: NULL engine");
  SPH_REQUIRE(!e->multi() || e->tr, SPH_HIP_ECOMM,
              "brick %d of %d: attach a communicator (sph_engine_comm_init / _comm_local) first",
              e->me, e->nprocs);
  SPH_HIP_TRY(hipSetDevice(e->device));
  e->setup();
  SPH_HIP_TRY(hipGetLastError());
  SPH_API_END
}

int sph_engine_run(sph_engine *e, int nsteps) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && nsteps >= 0, SPH_HIP_EINVAL, "sph_engine_run: bad argument");
  SPH_REQUIRE(e->setup_done, SPH_HIP_EINVAL, "sph_engine_run: call sph_engine_setup first");
  SPH_HIP_TRY(hipSetDevice(e->device));
  e->run(nsteps);
  SPH_API_END
}

int sph_engine_pair_passes(sph_engine *e, int n) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && n >= 0, SPH_HIP_EINVAL, "sph_engine_pair_passes: bad argument");
  SPH_REQUIRE(e->setup_done, SPH_HIP_EINVAL, "sph_engine_pair_passes: call setup first");
  SPH_HIP_TRY(hipSetDevice(e->device));
  for (int k = 0; k < n; k++) e->pair_compute(e->cfg.rhosum_nstep > 0);
  SPH_HIP_TRY(hipGetLastError());
  SPH_API_END
}

int sph_engine_rebuild_passes(sph_engine *e, int n) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && n >= 0, SPH_HIP_EINVAL, "sph_engine_rebuild_passes: bad argument");
  SPH_REQUIRE(e->setup_done, SPH_HIP_EINVAL, "sph_engine_rebuild_passes: call setup first");
  SPH_HIP_TRY(hipSetDevice(e->device));
  for (int k = 0; k < n; k++) {
    e->force_sort = true;  // (the full rebuild, sort included)
    e->rebuild();
  }
  SPH_HIP_TRY(hipGetLastError());
  SPH_API_END
}

int sph_engine_nlocal(sph_engine *e) { return e ? e->nlocal : 0; }

int sph_engine_get_atoms(sph_engine *e, double *x, double *v, double *rho, double *en,
                         double *f, double *drho, double *de, int *tag) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_get_atoms: NULL engine");
  SPH_HIP_TRY(hipSetDevice(e->device));
  const int n = e->nlocal;
  if (n == 0) return SPH_HIP_OK;
  std::vector<double4> hx(n), hv(n), hvel(n), hf(n);
  std::vector<double> hen(n), hde(n);
  std::vector<int> ht(n);
  SPH_HIP_TRY(hipMemcpyAsync(hx.data(), e->xf.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hv.data(), e->vr.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hvel.data(), e->vel.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hf.data(), e->fo.p, n * sizeof(double4), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hen.data(), e->en.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(hde.data(), e->de.p, n * sizeof(double), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(ht.data(), e->tag.p, n * sizeof(int), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  // one brick of a decomposition (or caller tags): local slot order, tag[] names the atom;
  // otherwise the set_atoms order
  const bool local_order = e->multi() || e->global_tags;
  for (int i = 0; i < n; i++) {
    const int t = local_order ? i : ht[i];
    SPH_REQUIRE(t >= 0 && t < n, SPH_HIP_ERUNTIME, "corrupt tag %d", t);
    if (x) {
      x[3 * t] = hx[i].x;
      x[3 * t + 1] = hx[i].y;
      x[3 * t + 2] = hx[i].z;
    }
    if (v) {
      v[3 * t] = hvel[i].x;
      v[3 * t + 1] = hvel[i].y;
      v[3 * t + 2] = hvel[i].z;
    }
    if (rho) rho[t] = hv[i].w;
    if (en) en[t] = hen[i];
    if (f) {
      f[3 * t] = hf[i].x;
      f[3 * t + 1] = hf[i].y;
      f[3 * t + 2] = hf[i].z;
    }
    if (drho) drho[t] = hf[i].w;
    if (de) de[t] = hde[i];
    if (tag) tag[t] = ht[i];
  }
  SPH_API_END
}

int sph_engine_neighbor_counts(sph_engine *e, int *numneigh) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && numneigh, SPH_HIP_EINVAL, "sph_engine_neighbor_counts: bad argument");
  SPH_HIP_TRY(hipSetDevice(e->device));
  const int n = e->nlocal;
  if (n == 0) return SPH_HIP_OK;
  std::vector<int> hc(n), ht(n);
  SPH_HIP_TRY(hipMemcpyAsync(hc.data(), e->ccnt.p, n * sizeof(int),
                             hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipMemcpyAsync(ht.data(), e->tag.p, n * sizeof(int), hipMemcpyDeviceToHost, e->s));
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  const bool local_order = e->multi() || e->global_tags;
  for (int i = 0; i < n; i++) numneigh[local_order ? i : ht[i]] = hc[i];
  SPH_API_END
}

int sph_engine_stats_get(sph_engine *e, sph_engine_stats *st) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && st, SPH_HIP_EINVAL, "sph_engine_stats_get: bad argument");
  SPH_HIP_TRY(hipSetDevice(e->device));
  e->harvest();
  st->step = e->step;
  st->nlocal = e->nlocal;
  st->nghost = e->nghost;
  st->nbr_full = e->list_entries();
  st->nbr_builds = e->nbr_builds;
  st->nbr_maxrow = e->nbr_maxrow;
  st->staged = e->blk ? 1 : 0;
  st->stage_max = e->blk ? e->blk_um : 0;
  st->ms_rhosum = e->ms[T_RHO];
  st->ms_tait = e->ms[T_TAIT];
  st->ms_heat = e->ms[T_HEAT];
  st->ms_integrate = e->ms[T_INT];
  st->ms_comm = e->ms[T_COMM];
  st->ms_neigh = e->ms[T_NEIGH];
  st->n_rhosum = e->nlaunch[T_RHO];
  st->n_tait = e->nlaunch[T_TAIT];
  st->n_heat = e->nlaunch[T_HEAT];
  st->n_neigh = e->nlaunch[T_NEIGH];
  st->blk_nbig = 0;
  if (e->blk && e->mx.p) {  // (k_blk_count_big of the last block build)
    SPH_HIP_TRY(hipMemcpyAsync(&st->blk_nbig, e->mx.p + 9, sizeof(int), hipMemcpyDeviceToHost,
                               e->s));
    SPH_HIP_TRY(hipStreamSynchronize(e->s));
  }
  st->inner_rows = e->inner ? 1 : 0;
  st->inner_live = 0;
  if (e->inner && e->moved.p) {
    int mv = 1;
    SPH_HIP_TRY(hipMemcpyAsync(&mv, e->moved_flag(), sizeof(int), hipMemcpyDeviceToHost, e->s));
    SPH_HIP_TRY(hipStreamSynchronize(e->s));
    st->inner_live = mv == 0 ? 1 : 0;
  }
  st->flags = (e->rho_fused_step >= 0 && e->rho_fused_step == e->step) ? 1 : 0;
  st->inner_refresh = e->inner_refreshes;
  SPH_API_END
}

int sph_engine_set_timing(sph_engine *e, int on) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_set_timing: NULL engine");
  SPH_HIP_TRY(hipSetDevice(e->device));
  e->harvest();
  // 1: every class; (mask << 1): the classes of mask (a timed run records an event pair per
  // timed scope, which at small sizes is a visible share of a step)
  e->timing_mask = on == 1 ? (1 << T_NCLASS) - 1 : (on > 1 ? (on >> 1) & ((1 << T_NCLASS) - 1) : 0);
  e->timing = e->timing_mask != 0;
  for (int k = 0; k < T_NCLASS; k++) {
    e->ms[k] = 0.0;
    e->nlaunch[k] = 0;
  }
  SPH_API_END
}

int sph_engine_sync(sph_engine *e) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_sync: NULL engine");
  SPH_HIP_TRY(hipSetDevice(e->device));
  SPH_HIP_TRY(hipStreamSynchronize(e->s));
  SPH_API_END
}

int sph_engine_comm_uid(void *uid128) {
  SPH_API_BEGIN
  SPH_REQUIRE(uid128, SPH_HIP_EINVAL, "sph_engine_comm_uid: NULL buffer");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  SPH_NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(uid128, &id, sizeof(id));
  SPH_API_END
}

static void attach(sph_engine *e, Transport *t) {
  const int sz = t->size(), rk = t->rank();
  if (sz != e->nprocs || rk != e->me) {
    delete t;
    SPH_REQUIRE(false, SPH_HIP_EINVAL,
                "communicator rank %d/%d does not match the engine's brick %d/%d", rk, sz,
                e->me, e->nprocs);
  }
  delete e->tr;
  e->tr = t;
}

int sph_engine_comm_init(sph_engine *e, const void *uid128, int nranks, int rank) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && uid128, SPH_HIP_EINVAL, "sph_engine_comm_init: NULL argument");
  SPH_HIP_TRY(hipSetDevice(e->device));
  ncclUniqueId id;
  memcpy(&id, uid128, sizeof(id));
  attach(e, new RcclTransport(id, nranks, rank));
  SPH_API_END
}

int sph_engine_comm_loopback(sph_engine *e, int on) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_comm_loopback: NULL engine");
  SPH_REQUIRE(e->nprocs == 1 && e->tr, SPH_HIP_ECOMM,
              "sph_engine_comm_loopback: needs a one-brick engine with a communicator attached");
  e->loopback = on != 0;
  e->setup_done = false;
  SPH_API_END
}

int sph_local_world_create(int nranks, sph_local_world **out) {
  SPH_API_BEGIN
  SPH_REQUIRE(out && nranks >= 1, SPH_HIP_EINVAL, "sph_local_world_create: bad argument");
  *out = reinterpret_cast<sph_local_world *>(new LocalWorld(nranks));
  SPH_API_END
}

int sph_local_world_destroy(sph_local_world *w) {
  delete reinterpret_cast<LocalWorld *>(w);
  return SPH_HIP_OK;
}

int sph_engine_comm_local(sph_engine *e, sph_local_world *w, int rank) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && w, SPH_HIP_EINVAL, "sph_engine_comm_local: NULL argument");
  LocalWorld *lw = reinterpret_cast<LocalWorld *>(w);
  SPH_REQUIRE(rank >= 0 && rank < lw->n, SPH_HIP_EINVAL, "rank %d outside [0,%d)", rank, lw->n);
  attach(e, new LocalTransport(lw, rank));
  SPH_API_END
}

int sph_engine_comm_ipc(sph_engine *e, const char *name, int nranks, int rank, int mode) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && name, SPH_HIP_EINVAL, "sph_engine_comm_ipc: NULL argument");
  SPH_HIP_TRY(hipSetDevice(e->device));
  attach(e, new IpcTransport(name, nranks, rank, mode, e->device));
  SPH_API_END
}

int sph_engine_tune(sph_engine *e, int key, int value) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_tune: NULL engine");
  SPH_REQUIRE(!e->setup_done, SPH_HIP_EINVAL, "sph_engine_tune: before sph_engine_setup");
  switch (key) {
    case SPH_TUNE_OVERLAP: e->overlap = value != 0; break;
    case SPH_TUNE_BLKUMF:
      SPH_REQUIRE(value >= 0, SPH_HIP_EINVAL, "sph_engine_tune: BLKUMF %d < 0", value);
      e->blkumf = value;
      break;
    default: SPH_REQUIRE(false, SPH_HIP_EINVAL, "sph_engine_tune: unknown key %d", key);
  }
  SPH_API_END
}

int sph_engine_set_tags(sph_engine *e, const int *tags) {
  SPH_API_BEGIN
  SPH_REQUIRE(e && (tags || e->nlocal == 0), SPH_HIP_EINVAL, "sph_engine_set_tags: bad argument");
  SPH_HIP_TRY(hipSetDevice(e->device));
  int mx = -1;
  for (int i = 0; i < e->nlocal; i++) {
    SPH_REQUIRE(tags[i] >= 0 && tags[i] < (1 << 30), SPH_HIP_EINVAL,
                "sph_engine_set_tags: tag %d outside [0, 2^30)", tags[i]);
    mx = std::max(mx, tags[i]);
  }
  if (e->nlocal)
    SPH_HIP_TRY(hipMemcpy(e->tag.p, tags, e->nlocal * sizeof(int), hipMemcpyHostToDevice));
  e->global_tags = true;
  e->tag_next = mx + 1;  // (bricks: the ranks agree on the largest at the first phase change)
  e->pc_tags_agreed = false;
  e->lidx_valid = false;  // (read order = tag order, taken at setup)
  SPH_API_END
}

int sph_engine_atom_sort(sph_engine *e, int sortfreq, double binsize) {
  SPH_API_BEGIN
  SPH_REQUIRE(e, SPH_HIP_EINVAL, "sph_engine_atom_sort: NULL engine");
  SPH_REQUIRE(sortfreq >= 0 && binsize >= 0.0, SPH_HIP_EINVAL, "Illegal atom_modify command");
  e->sortfreq = sortfreq;
  e->sort_binsize = binsize;
  SPH_API_END
}

}  // extern "C"
