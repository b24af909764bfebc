// sph_comm.h -- brick decomposition transport and the halo/migration pack kernels.
//
// The engine splits the box into procgrid bricks exactly like CommBrick
// (comm_brick.cpp:150-400 setup, :573-680 exchange, :690-880 borders, :400-560 forward and
// reverse comm): per dimension two swaps, the first sending atoms within cutghost of the
// lower face to the lower neighbour (shifted by +prd across the periodic boundary), the
// second the upper face to the upper neighbour; later dimensions forward earlier ghosts
// (edges and corners).  A swap whose neighbour is this brick itself (procgrid[d] == 1) is
// a device copy; a remote one goes through a Transport:
//   * RcclTransport  -- one process per GPU, ncclSend/ncclRecv pairs on the engine's
//                       stream (RCCL over xGMI); the production multi-GPU path;
//   * LocalTransport -- several bricks in one process (threads, one engine each, any GPU),
//                       device-to-device copies between their buffers; used to test the
//                       decomposition on a single GPU and for bricks sharing a device.
// Only the counts of a swap need the host (buffer sizing at borders/exchange time); the
// per-step forward comm is stream-ordered.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <mutex>
#include <vector>

#include "sph_engine_kernels.h"
#include "sph_util.h"

namespace sph {

struct Transport {
  virtual ~Transport() {}
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // exchange one int with two peers (send to dest, receive from src); host-synchronous
  virtual int exchange_count(int nsend, int dest, int src, hipStream_t s) = 0;
  // the two directions of one dimension at once: send n0 to d0 and n1 to d1, receive from
  // src0 into nrecv[0] and from src1 into nrecv[1]; host-synchronous
  virtual void exchange_count2(int n0, int d0, int src0, int n1, int d1, int src1,
                               hipStream_t s, int nrecv[2]) {
    nrecv[0] = exchange_count(n0, d0, src0, s);
    nrecv[1] = exchange_count(n1, d1, src1, s);
  }
  // exchange device buffers (stream-ordered on s)
  virtual void exchange(const void *sbuf, size_t sbytes, int dest, void *rbuf, size_t rbytes,
                        int src, hipStream_t s) = 0;
  // two independent exchanges (the two directions of one dimension) at once
  virtual void exchange2(const void *s0, size_t sb0, int d0, void *r0, size_t rb0, int src0,
                         const void *s1, size_t sb1, int d1, void *r1, size_t rb1, int src1,
                         hipStream_t s) {
    exchange(s0, sb0, d0, r0, rb0, src0, s);
    exchange(s1, sb1, d1, r1, rb1, src1, s);
  }
  virtual void barrier(hipStream_t s) = 0;
  // exchange_count2 with the two send counts in DEVICE words dsend[0..1] (written by kernels
  // on s): h[0..1] = the sends, h[2..3] = the receives (from src0, src1); one host sync
  virtual void exchange_count2_dev(const int *dsend, int d0, int src0, int d1, int src1,
                                   hipStream_t s, int h[4]) {
    SPH_HIP_TRY(hipMemcpyAsync(h, dsend, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    int nr[2];
    exchange_count2(h[0], d0, src0, h[1], d1, src1, s, nr);
    h[2] = nr[0];
    h[3] = nr[1];
  }
  // every other rank r: send scnt[r] to r, receive rcnt[r] from r (scnt/rcnt hold size()
  // ints; the own entry is ignored); host-synchronous
  virtual void exchange_counts_all(const int *scnt, int *rcnt, hipStream_t s) = 0;
  // n exchanges in ONE group: send sb[k] (sbytes[k]) to peer[k] and receive rb[k]
  // (rbytes[k]) from peer[k]; at most one entry per peer; stream-ordered on s
  virtual void exchange_multi(int n, const int *peer, const void *const *sb,
                              const size_t *sbytes, void *const *rb, const size_t *rbytes,
                              hipStream_t s) = 0;
  // every rank's v into out[size()] (MPI_Allgather of one int); host-synchronous
  void allgather_int(int v, int *out, hipStream_t s) {
    const int P = size(), me = rank();
    std::vector<int> sc(P, v);
    exchange_counts_all(sc.data(), out, s);
    out[me] = v;
  }
};

#define SPH_NCCL_TRY(call)                                                             \
  do {                                                                                 \
    ncclResult_t r_ = (call);                                                          \
    SPH_REQUIRE(r_ == ncclSuccess, SPH_HIP_ECOMM, "%s: %s", #call, ncclGetErrorString(r_)); \
  } while (0)

class RcclTransport : public Transport {
 public:
  RcclTransport(const ncclUniqueId &id, int nranks, int rank) : n_(nranks), me_(rank) {
    SPH_NCCL_TRY(ncclCommInitRank(&comm_, nranks, id, rank));
    SPH_HIP_TRY(hipMalloc(&dcnt_, 4 * sizeof(int)));
  }
  ~RcclTransport() override {
    if (dcnt_) (void)hipFree(dcnt_);
    if (dall_) (void)hipFree(dall_);
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  int rank() const override { return me_; }
  int size() const override { return n_; }
  int exchange_count(int nsend, int dest, int src, hipStream_t s) override {
    int h[2] = {nsend, 0};
    SPH_HIP_TRY(hipMemcpyAsync(dcnt_, h, sizeof(int), hipMemcpyHostToDevice, s));
    SPH_NCCL_TRY(ncclGroupStart());
    SPH_NCCL_TRY(ncclSend(dcnt_, 1, ncclInt32, dest, comm_, s));
    SPH_NCCL_TRY(ncclRecv(dcnt_ + 1, 1, ncclInt32, src, comm_, s));
    SPH_NCCL_TRY(ncclGroupEnd());
    SPH_HIP_TRY(hipMemcpyAsync(&h[1], dcnt_ + 1, sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    return h[1];
  }
  void exchange(const void *sbuf, size_t sbytes, int dest, void *rbuf, size_t rbytes, int src,
                hipStream_t s) override {
    SPH_NCCL_TRY(ncclGroupStart());
    if (sbytes) SPH_NCCL_TRY(ncclSend(sbuf, sbytes, ncclUint8, dest, comm_, s));
    if (rbytes) SPH_NCCL_TRY(ncclRecv(rbuf, rbytes, ncclUint8, src, comm_, s));
    SPH_NCCL_TRY(ncclGroupEnd());
  }
  // one RCCL group and one host sync for both directions' counts (sends to the same peer
  // are matched in posting order, so direction 0 meets direction 0)
  void exchange_count2(int n0, int d0, int src0, int n1, int d1, int src1, hipStream_t s,
                       int nrecv[2]) override {
    int h[4] = {n0, n1, 0, 0};
    SPH_HIP_TRY(hipMemcpyAsync(dcnt_, h, 2 * sizeof(int), hipMemcpyHostToDevice, s));
    SPH_NCCL_TRY(ncclGroupStart());
    SPH_NCCL_TRY(ncclSend(dcnt_, 1, ncclInt32, d0, comm_, s));
    SPH_NCCL_TRY(ncclRecv(dcnt_ + 2, 1, ncclInt32, src0, comm_, s));
    SPH_NCCL_TRY(ncclSend(dcnt_ + 1, 1, ncclInt32, d1, comm_, s));
    SPH_NCCL_TRY(ncclRecv(dcnt_ + 3, 1, ncclInt32, src1, comm_, s));
    SPH_NCCL_TRY(ncclGroupEnd());
    SPH_HIP_TRY(hipMemcpyAsync(&h[2], dcnt_ + 2, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    nrecv[0] = h[2];
    nrecv[1] = h[3];
  }
  // the counts straight from the device words: one RCCL group and one host read of all four
  void exchange_count2_dev(const int *dsend, int d0, int src0, int d1, int src1, hipStream_t s,
                           int h[4]) override {
    SPH_HIP_TRY(hipMemcpyAsync(dcnt_, dsend, 2 * sizeof(int), hipMemcpyDeviceToDevice, s));
    SPH_NCCL_TRY(ncclGroupStart());
    SPH_NCCL_TRY(ncclSend(dcnt_, 1, ncclInt32, d0, comm_, s));
    SPH_NCCL_TRY(ncclRecv(dcnt_ + 2, 1, ncclInt32, src0, comm_, s));
    SPH_NCCL_TRY(ncclSend(dcnt_ + 1, 1, ncclInt32, d1, comm_, s));
    SPH_NCCL_TRY(ncclRecv(dcnt_ + 3, 1, ncclInt32, src1, comm_, s));
    SPH_NCCL_TRY(ncclGroupEnd());
    SPH_HIP_TRY(hipMemcpyAsync(h, dcnt_, 4 * sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
  }
  // one RCCL group for both directions of a dimension: one launch/sync round instead of two
  void exchange2(const void *s0, size_t sb0, int d0, void *r0, size_t rb0, int src0,
                 const void *s1, size_t sb1, int d1, void *r1, size_t rb1, int src1,
                 hipStream_t s) override {
    SPH_NCCL_TRY(ncclGroupStart());
    if (sb0) SPH_NCCL_TRY(ncclSend(s0, sb0, ncclUint8, d0, comm_, s));
    if (rb0) SPH_NCCL_TRY(ncclRecv(r0, rb0, ncclUint8, src0, comm_, s));
    if (sb1) SPH_NCCL_TRY(ncclSend(s1, sb1, ncclUint8, d1, comm_, s));
    if (rb1) SPH_NCCL_TRY(ncclRecv(r1, rb1, ncclUint8, src1, comm_, s));
    SPH_NCCL_TRY(ncclGroupEnd());
  }
  void barrier(hipStream_t s) override {
    SPH_NCCL_TRY(ncclAllReduce(dcnt_, dcnt_, 1, ncclInt32, ncclSum, comm_, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
  }
  void exchange_counts_all(const int *scnt, int *rcnt, hipStream_t s) override {
    if (!dall_) SPH_HIP_TRY(hipMalloc(&dall_, 2 * (size_t)n_ * sizeof(int)));
    SPH_HIP_TRY(hipMemcpyAsync(dall_, scnt, n_ * sizeof(int), hipMemcpyHostToDevice, s));
    SPH_NCCL_TRY(ncclGroupStart());
    for (int r = 0; r < n_; r++) {
      if (r == me_) continue;
      SPH_NCCL_TRY(ncclSend(dall_ + r, 1, ncclInt32, r, comm_, s));
      SPH_NCCL_TRY(ncclRecv(dall_ + n_ + r, 1, ncclInt32, r, comm_, s));
    }
    SPH_NCCL_TRY(ncclGroupEnd());
    SPH_HIP_TRY(hipMemcpyAsync(rcnt, dall_ + n_, n_ * sizeof(int), hipMemcpyDeviceToHost, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    rcnt[me_] = 0;
  }
  void exchange_multi(int n, const int *peer, const void *const *sb, const size_t *sbytes,
                      void *const *rb, const size_t *rbytes, hipStream_t s) override {
    SPH_NCCL_TRY(ncclGroupStart());
    for (int k = 0; k < n; k++) {
      if (sbytes[k]) SPH_NCCL_TRY(ncclSend(sb[k], sbytes[k], ncclUint8, peer[k], comm_, s));
      if (rbytes[k]) SPH_NCCL_TRY(ncclRecv(rb[k], rbytes[k], ncclUint8, peer[k], comm_, s));
    }
    SPH_NCCL_TRY(ncclGroupEnd());
  }

 private:
  int n_, me_;
  ncclComm_t comm_ = nullptr;
  int *dcnt_ = nullptr, *dall_ = nullptr;
};

// Bricks of one process: every brick runs in its own host thread; a swap posts its send
// buffer, meets the others at a barrier, copies its peer's buffer, meets them again.
struct LocalWorld {
  explicit LocalWorld(int n) : n(n), post(n), mpost(n), cpost(n) {}
  struct Post {
    const void *buf = nullptr;
    size_t bytes = 0;
    int dest = -1, count = 0;
  };
  int n;
  std::vector<Post> post;
  std::vector<std::vector<Post>> mpost;  // exchange_multi: every rank's sends
  std::vector<std::vector<int>> cpost;   // exchange_counts_all: every rank's counts
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long generation = 0;
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long g = generation;
    if (++arrived == n) {
      arrived = 0;
      generation++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != g; });
    }
  }
};

class LocalTransport : public Transport {
 public:
  LocalTransport(LocalWorld *w, int rank) : w_(w), me_(rank) {}
  int rank() const override { return me_; }
  int size() const override { return w_->n; }
  int exchange_count(int nsend, int dest, int src, hipStream_t s) override {
    w_->post[me_].count = nsend;
    w_->post[me_].dest = dest;
    w_->barrier();
    SPH_REQUIRE(w_->post[src].dest == me_, SPH_HIP_ECOMM, "local swap mismatch (%d -> %d)", src,
                me_);
    const int nrecv = w_->post[src].count;
    w_->barrier();
    return nrecv;
  }
  void exchange(const void *sbuf, size_t sbytes, int dest, void *rbuf, size_t rbytes, int src,
                hipStream_t s) override {
    SPH_HIP_TRY(hipStreamSynchronize(s));  // my send buffer is packed
    w_->post[me_].buf = sbuf;
    w_->post[me_].bytes = sbytes;
    w_->post[me_].dest = dest;
    w_->barrier();
    SPH_REQUIRE(w_->post[src].dest == me_ && w_->post[src].bytes == rbytes, SPH_HIP_ECOMM,
                "local swap mismatch (%d -> %d: %zu vs %zu bytes)", src, me_,
                w_->post[src].bytes, rbytes);
    if (rbytes)
      SPH_HIP_TRY(hipMemcpyAsync(rbuf, w_->post[src].buf, rbytes, hipMemcpyDeviceToDevice, s));
    SPH_HIP_TRY(hipStreamSynchronize(s));
    w_->barrier();  // the sender may reuse its buffer now
  }
  void barrier(hipStream_t s) override {
    SPH_HIP_TRY(hipStreamSynchronize(s));
    w_->barrier();
  }
  void exchange_counts_all(const int *scnt, int *rcnt, hipStream_t s) override {
    w_->cpost[me_].assign(scnt, scnt + w_->n);
    w_->barrier();
    for (int r = 0; r < w_->n; r++) rcnt[r] = r == me_ ? 0 : w_->cpost[r][me_];
    w_->barrier();
  }
  void exchange_multi(int n, const int *peer, const void *const *sb, const size_t *sbytes,
                      void *const *rb, const size_t *rbytes, hipStream_t s) override {
    SPH_HIP_TRY(hipStreamSynchronize(s));  // my send buffers are packed
    auto &mine = w_->mpost[me_];
    mine.clear();
    for (int k = 0; k < n; k++) {
      LocalWorld::Post p;
      p.buf = sb[k];
      p.bytes = sbytes[k];
      p.dest = peer[k];
      mine.push_back(p);
    }
    w_->barrier();
    for (int k = 0; k < n; k++) {
      const LocalWorld::Post *q = nullptr;
      for (const auto &c : w_->mpost[peer[k]])
        if (c.dest == me_) q = &c;
      SPH_REQUIRE((q && q->bytes == rbytes[k]) || (!q && rbytes[k] == 0), SPH_HIP_ECOMM,
                  "local multi exchange mismatch (%d -> %d: %zu bytes expected)", peer[k], me_,
                  rbytes[k]);
      if (rbytes[k])
        SPH_HIP_TRY(hipMemcpyAsync(rb[k], q->buf, rbytes[k], hipMemcpyDeviceToDevice, s));
    }
    SPH_HIP_TRY(hipStreamSynchronize(s));
    w_->barrier();  // the senders may reuse their buffers now
  }

 private:
  LocalWorld *w_;
  int me_;
};

// ---- pack / unpack kernels -------------------------------------------------------------
// border record (AtomVecMeso::pack_border/unpack_border, atom_vec_meso.cpp:422-600):
// x (shifted), vest + rho, e, type -- plus the ghost's ORIGIN: the rank and owned index of
// the atom it images and the accumulated periodic image (a ghost forwarded along a later
// dimension keeps its origin), from which the per-step forward comm goes straight from
// owner to ghost in one exchange (sph_engine::build_direct)
struct BorderRec {
  double4 x, v;
  double e;
  int type, orank, oidx, img;
};

__device__ __forceinline__ double4 shift_x(double4 x, int dim, double shift) {
  if (dim == 0) x.x += shift;
  else if (dim == 1) x.y += shift;
  else x.z += shift;
  return x;
}

static __global__ void k_pack_border(int n, const int *__restrict__ list, int dim, double shift,
                                     int pbc, int me, int nlocal,
                                     const double4 *__restrict__ xf,
                                     const double4 *__restrict__ vr,
                                     const double *__restrict__ en, const int *__restrict__ ty,
                                     const int *__restrict__ gorank,
                                     const int *__restrict__ goidx,
                                     const int *__restrict__ gimg, BorderRec *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];
  BorderRec r;
  r.x = shift_x(xf[i], dim, shift);
  r.v = vr[i];
  r.e = en[i];
  r.type = ty[i];
  const bool own = i < nlocal;
  r.orank = own ? me : gorank[i - nlocal];
  r.oidx = own ? i : goidx[i - nlocal];
  r.img = img_add(own ? 0 : gimg[i - nlocal], dim, pbc);
  out[k] = r;
}

static __global__ void k_unpack_border(int n, int first, int nlocal,
                                       const BorderRec *__restrict__ in,
                                       double4 *__restrict__ xf, double4 *__restrict__ vr,
                                       double *__restrict__ en, int *__restrict__ ty,
                                       int *__restrict__ gorank, int *__restrict__ goidx,
                                       int *__restrict__ gimg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const BorderRec r = in[k];
  xf[first + k] = r.x;
  vr[first + k] = r.v;
  en[first + k] = r.e;
  ty[first + k] = r.type;
  const int g = first + k - nlocal;
  gorank[g] = r.orank;
  goidx[g] = r.oidx;
  gimg[g] = r.img;
}

// ---- direct forward comm (owner -> ghost in one exchange) -----------------------------
// pack: the listed owned atoms' x (unshifted), vest, rho, e, P/rho^2 (9 doubles); unpack:
// into ghost slots, each coordinate shifted by its own image (one add per coordinate, as the
// hop-by-hop forward adds it: every hop shifts exactly one coordinate, atom_vec_meso.cpp:
// 246-288)
static __global__ void k_pack_direct(int n, const int *__restrict__ idx,
                                     const double4 *__restrict__ xf,
                                     const double4 *__restrict__ vr,
                                     const double *__restrict__ en, double *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = idx[k];
  const double4 x = xf[i], v = vr[i];
  double *o = out + 9 * (size_t)k;
  o[0] = x.x;
  o[1] = x.y;
  o[2] = x.z;
  o[3] = v.x;
  o[4] = v.y;
  o[5] = v.z;
  o[6] = v.w;
  o[7] = en[i];
  o[8] = x.w;
}
static __global__ void k_unpack_direct(int n, const int *__restrict__ slot, int nlocal, Box b,
                                       const int *__restrict__ gimg,
                                       const double *__restrict__ in, double4 *__restrict__ xf,
                                       double4 *__restrict__ vr, double *__restrict__ en) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int g = slot[k], img = gimg[g];
  const double *o = in + 9 * (size_t)k;
  double4 x = make_double4(o[0], o[1], o[2], o[8]);
  const int ix = img_get(img, 0), iy = img_get(img, 1), iz = img_get(img, 2);
  if (ix) x.x = x.x + ix * b.prd[0];
  if (iy) x.y = x.y + iy * b.prd[1];
  if (iz) x.z = x.z + iz * b.prd[2];
  xf[nlocal + g] = x;
  vr[nlocal + g] = make_double4(o[3], o[4], o[5], o[6]);
  en[nlocal + g] = o[7];
}
// ghosts imaging this rank's own atoms: straight device copies
static __global__ void k_forward_self(int n, const int *__restrict__ slot, int nlocal, Box b,
                                      const int *__restrict__ goidx,
                                      const int *__restrict__ gimg, double4 *__restrict__ xf,
                                      double4 *__restrict__ vr, double *__restrict__ en) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int g = slot[k], o = goidx[g], img = gimg[g];
  double4 x = xf[o];
  const int ix = img_get(img, 0), iy = img_get(img, 1), iz = img_get(img, 2);
  if (ix) x.x = x.x + ix * b.prd[0];
  if (iy) x.y = x.y + iy * b.prd[1];
  if (iz) x.z = x.z + iz * b.prd[2];
  xf[nlocal + g] = x;
  vr[nlocal + g] = vr[o];
  en[nlocal + g] = en[o];
}
static __global__ void k_unpack_rho_direct(int n, const int *__restrict__ slot, int nlocal,
                                           const double2 *__restrict__ in,
                                           double4 *__restrict__ xf, double4 *__restrict__ vr) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int g = nlocal + slot[k];
  const double2 r = in[k];
  vr[g].w = r.x;
  xf[g].w = r.y;
}
static __global__ void k_forward_rho_self(int n, const int *__restrict__ slot, int nlocal,
                                          const int *__restrict__ goidx,
                                          double4 *__restrict__ xf, double4 *__restrict__ vr) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int g = slot[k], o = goidx[g];
  vr[nlocal + g].w = vr[o].w;
  xf[nlocal + g].w = xf[o].w;
}

// forward comm (AtomVecMeso::pack_comm_vel, atom_vec_meso.cpp:246-360): x (shifted),
// vest + rho, e as 9 doubles per atom
static __global__ void k_pack_forward(int n, const int *__restrict__ list, int dim,
                                      double shift, const double4 *__restrict__ xf,
                                      const double4 *__restrict__ vr,
                                      const double *__restrict__ en, double *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];
  const double4 x = shift_x(xf[i], dim, shift);
  const double4 v = vr[i];
  double *o = out + 9 * (size_t)k;
  o[0] = x.x;
  o[1] = x.y;
  o[2] = x.z;
  o[3] = v.x;
  o[4] = v.y;
  o[5] = v.z;
  o[6] = v.w;
  o[7] = en[i];
  o[8] = x.w;
}

static __global__ void k_unpack_forward(int n, int first, const double *__restrict__ in,
                                        double4 *__restrict__ xf, double4 *__restrict__ vr,
                                        double *__restrict__ en) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double *o = in + 9 * (size_t)k;
  xf[first + k] = make_double4(o[0], o[1], o[2], o[8]);
  vr[first + k] = make_double4(o[3], o[4], o[5], o[6]);
  en[first + k] = o[7];
}

// forward_comm_pair of sph/rhosum (pair_sph_rhosum.cpp:290-313): rho, plus the EOS term
// P/rho^2 the force pass reads from the same record
static __global__ void k_pack_rho(int n, const int *__restrict__ list,
                                  const double4 *__restrict__ xf,
                                  const double4 *__restrict__ vr, double2 *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];
  out[k] = make_double2(vr[i].w, xf[i].w);
}

static __global__ void k_unpack_rho(int n, int first, const double2 *__restrict__ in,
                                    double4 *__restrict__ xf, double4 *__restrict__ vr) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double2 r = in[k];
  vr[first + k].w = r.x;
  xf[first + k].w = r.y;
}

// reverse comm (AtomVecMeso::pack_reverse/unpack_reverse, atom_vec_meso.cpp:387-418):
// f, drho, de of the swap's ghosts back onto the sender's atoms
static __global__ void k_pack_reverse(int n, int first, const double4 *__restrict__ fo,
                                      const double *__restrict__ de, double *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double4 f = fo[first + k];
  double *o = out + 5 * (size_t)k;
  o[0] = f.x;
  o[1] = f.y;
  o[2] = f.z;
  o[3] = f.w;
  o[4] = de[first + k];
}

static __global__ void k_unpack_reverse(int n, const int *__restrict__ list,
                                        const double *__restrict__ in,
                                        double4 *__restrict__ fo, double *__restrict__ de) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];  // distinct within one swap
  const double *o = in + 5 * (size_t)k;
  double4 f = fo[i];
  f.x += o[0];
  f.y += o[1];
  f.z += o[2];
  f.w += o[3];
  fo[i] = f;
  de[i] += o[4];
}

// migration record (AtomVecMeso::pack_exchange, atom_vec_meso.cpp:620-700)
struct MigRec {
  double4 x, v, vel;
  double e;
  int type, tag;
};

static __global__ void k_flag_leave(int n, int dim, double lo, double hi,
                                    const double4 *__restrict__ xf,
                                    unsigned char *__restrict__ leave,
                                    unsigned char *__restrict__ stay) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double4 x = xf[i];
  const double c = dim == 0 ? x.x : (dim == 1 ? x.y : x.z);
  const bool out = c < lo || c >= hi;  // comm_brick.cpp:601-615
  leave[i] = out ? 1 : 0;
  stay[i] = out ? 0 : 1;
}

static __global__ void k_pack_mig(int n, const int *__restrict__ list,
                                  const double4 *__restrict__ xf,
                                  const double4 *__restrict__ vr,
                                  const double4 *__restrict__ vel,
                                  const double *__restrict__ en, const int *__restrict__ ty,
                                  const int *__restrict__ tag, MigRec *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int i = list[k];
  MigRec r;
  r.x = xf[i];
  r.v = vr[i];
  r.vel = vel[i];
  r.e = en[i];
  r.type = ty[i];
  r.tag = tag[i];
  out[k] = r;
}

// keep the received atoms that fall in this brick along dim (comm_brick.cpp:650-672)
static __global__ void k_flag_mine(int n, int dim, double lo, double hi,
                                   const MigRec *__restrict__ in,
                                   unsigned char *__restrict__ flag) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double4 x = in[k].x;
  const double c = dim == 0 ? x.x : (dim == 1 ? x.y : x.z);
  flag[k] = (c >= lo && c < hi) ? 1 : 0;
}

// gather the listed records (staying atoms or accepted arrivals) into slots first..
static __global__ void k_gather_mig(int n, const int *__restrict__ list,
                                    const MigRec *__restrict__ in, int first,
                                    double4 *__restrict__ xf, double4 *__restrict__ vr,
                                    double4 *__restrict__ vel, double *__restrict__ en,
                                    int *__restrict__ ty, int *__restrict__ tag) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const MigRec r = in[list ? list[k] : k];
  const int d = first + k;
  xf[d] = r.x;
  vr[d] = r.v;
  vel[d] = r.vel;
  en[d] = r.e;
  ty[d] = r.type;
  tag[d] = r.tag;
}

}  // namespace sph
