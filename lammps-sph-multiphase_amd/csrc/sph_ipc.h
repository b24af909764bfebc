// sph_ipc.h -- IpcTransport: the brick decomposition's byte mover between PROCESSES of one
// node without RCCL.
//
// RCCL refuses two ranks on one device (ncclCommInitRank: "invalid usage",
// profiles/r01/rccl_two_ranks_one_gpu.log), so a one-GPU box could never run the engine as
// two processes.  This transport moves the same bytes the RcclTransport does -- the engine
// calls the same Transport methods in the same order (comm_brick.cpp:444-506 forward,
// :696-864 borders, :999-1030 reverse_comm_fix; fix_phase_change.cpp:338-351 and
// atom.cpp:598-630 through allgather_int) -- so everything above the byte mover (the per-rank
// setup, the uid/name sharing, the tag_extend allgather, the direct-forward peer grouping,
// max-over-ranks timing) runs exactly as across GPUs.
//
//   * control plane: one POSIX shared-memory segment per world (name chosen by rank 0 and
//     shared by the launcher); a sense-counting host barrier, per-rank post tables;
//   * data plane, mode SPH_IPC_DEVICE: every rank stages what it sends in one device
//     "outbox" exported with hipIpcGetMemHandle; receivers open the peer's handle
//     (hipIpcOpenMemHandle, re-opened when the outbox grows) and copy device-to-device on
//     their stream -- works across GPUs of a node (peer access over xGMI) and between two
//     processes sharing one GPU;
//   * data plane, mode SPH_IPC_HOST: the outbox is a shared-memory segment per rank and
//     growth generation; senders copy device-to-host into it, receivers host-to-device.
//
// Every Transport call here is collective over ALL ranks of the world (as LocalTransport's:
// the engine issues the same sequence of calls on every brick); a send is matched to the
// receiver's request by (source, order of posting), as ncclSend/ncclRecv pairs are.
// Liveness: every rank runs a heartbeat thread that stamps its slot (CLOCK_MONOTONIC, shared
// by the node's processes) every 50 ms while its world exists, so a waiting rank tells a peer
// that is busy (a long setup or first rebuild: it still beats) from one that is gone (its
// beat stops when the process exits or is killed): a barrier fails with SPH_HIP_ECOMM once a
// peer has not beaten for SPH_IPC_DEAD seconds (default 10), or has never beaten within the
// attach time (it died before it joined), and otherwise waits as long as the work takes, up to
// SPH_IPC_TIMEOUT seconds (default 1800: a peer whose main thread hangs -- a stuck kernel, a
// mismatched collective -- still beats from its heartbeat thread, so the wait stays bounded;
// <= 0 waits without bound).  Rank 0 removes host outboxes a killed run of the same world
// name left in /dev/shm.
#pragma once
#include <dirent.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sph_comm.h"

namespace sph {

enum { SPH_IPC_DEVICE = 0, SPH_IPC_HOST = 1 };

constexpr int IPC_MAXR = 64;      // ranks of one node-local world
constexpr int IPC_MAXPOST = 128;  // sends of one collective call per rank
constexpr uint32_t IPC_MAGIC = 0x53504849u;  // "SPHI"

struct IpcPost {
  int dest;
  int val;        // exchange_count*: the count; data posts: unused
  uint64_t off;   // byte offset of the payload in the sender's outbox
  uint64_t bytes;
};

struct IpcRankSlot {
  hipIpcMemHandle_t handle;   // SPH_IPC_DEVICE: the outbox
  std::atomic<uint64_t> gen;  // outbox generation (bumped when it grows)
  uint64_t cap;
  int npost;
  IpcPost post[IPC_MAXPOST];
  int cnt[IPC_MAXR];          // exchange_counts_all: what this rank sends to each rank
  std::atomic<int64_t> beat;  // CLOCK_MONOTONIC ns of the rank's last heartbeat (0: none)
};

struct IpcShm {
  std::atomic<uint32_t> magic;
  int n, mode;
  std::atomic<int> arrived;
  std::atomic<long> generation;
  std::atomic<int> attached;
  IpcRankSlot r[IPC_MAXR];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "process-shared atomics");
static_assert(std::atomic<int>::is_always_lock_free, "process-shared atomics");

class IpcTransport : public Transport {
 public:
  IpcTransport(const char *name, int nranks, int rank, int mode, int device)
      : name_(name), n_(nranks), me_(rank), mode_(mode) {
    (void)device;  // the caller's hipSetDevice picked it: the outbox lives there
    SPH_REQUIRE(nranks >= 1 && nranks <= IPC_MAXR && rank >= 0 && rank < nranks, SPH_HIP_EINVAL,
                "ipc world: rank %d of %d (at most %d ranks)", rank, nranks, IPC_MAXR);
    SPH_REQUIRE(mode == SPH_IPC_DEVICE || mode == SPH_IPC_HOST, SPH_HIP_EINVAL,
                "ipc world: mode %d", mode);
    SPH_REQUIRE(name && name[0] == '/' && strlen(name) < 200 && !strchr(name + 1, '/'),
                SPH_HIP_EINVAL, "ipc world name must be '/word' (got '%s')", name ? name : "");
    const char *t = getenv("SPH_IPC_TIMEOUT");
    timeout_s_ = t ? atof(t) : 1800.0;
    born_ = std::chrono::steady_clock::now();
    const char *dd = getenv("SPH_IPC_DEAD");
    dead_s_ = dd ? atof(dd) : 10.0;
    const size_t sz = sizeof(IpcShm);
    int fd = -1;
    if (rank == 0) {
      shm_unlink(name);  // a stale segment of a killed run
      unlink_stale_outboxes();
      fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
      SPH_REQUIRE(fd >= 0, SPH_HIP_ECOMM, "shm_open(%s): %s", name, strerror(errno));
      if (ftruncate(fd, (off_t)sz) != 0) {
        close(fd);
        SPH_REQUIRE(false, SPH_HIP_ECOMM, "ftruncate(%s): %s", name, strerror(errno));
      }
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        fd = shm_open(name, O_RDWR, 0600);
        if (fd >= 0) {
          struct stat st;
          if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sz) break;
          close(fd);
          fd = -1;
        }
        SPH_REQUIRE(elapsed(t0) < attach_s_, SPH_HIP_ECOMM,
                    "ipc world %s: rank 0 never created it", name);
        usleep(2000);
      }
    }
    void *p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    SPH_REQUIRE(p != MAP_FAILED, SPH_HIP_ECOMM, "mmap(%s): %s", name, strerror(errno));
    w_ = static_cast<IpcShm *>(p);
    if (rank == 0) {
      w_->n = nranks;
      w_->mode = mode;
      w_->arrived.store(0);
      w_->generation.store(0);
      w_->attached.store(0);
      w_->magic.store(IPC_MAGIC, std::memory_order_release);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (w_->magic.load(std::memory_order_acquire) != IPC_MAGIC) {
        SPH_REQUIRE(elapsed(t0) < attach_s_, SPH_HIP_ECOMM, "ipc world %s never initialised", name);
        usleep(1000);
      }
      SPH_REQUIRE(w_->n == nranks && w_->mode == mode, SPH_HIP_ECOMM,
                  "ipc world %s: %d ranks mode %d, joined as %d ranks mode %d", name, w_->n,
                  w_->mode, nranks, mode);
    }
    w_->r[me_].gen.store(0);
    w_->r[me_].npost = 0;
    w_->r[me_].beat.store(now_ns(), std::memory_order_release);
    beater_ = std::thread([this] {
      while (!stop_.load(std::memory_order_acquire)) {
        w_->r[me_].beat.store(now_ns(), std::memory_order_release);
        struct timespec ts = {0, 50000000};
        nanosleep(&ts, nullptr);
      }
    });
    w_->attached.fetch_add(1);
    peer_.assign(n_, Peer());
    try {
      host_barrier();  // everyone attached: the name can go (no leftover in /dev/shm)
    } catch (...) {
      // (the destructor does not run for a constructor that throws: stop the heartbeat
      // thread and unmap here, or the joinable thread's destructor would terminate)
      stop_.store(true, std::memory_order_release);
      beater_.join();
      if (rank == 0) shm_unlink(name);
      munmap(w_, sizeof(IpcShm));
      w_ = nullptr;
      throw;
    }
    if (rank == 0) shm_unlink(name);
  }

  ~IpcTransport() override {
    stop_.store(true, std::memory_order_release);
    if (beater_.joinable()) beater_.join();
    for (auto &p : peer_) close_peer(p);
    if (dbox_) (void)hipFree(dbox_);
    if (hbox_) munmap(hbox_, hcap_);
    if (hname_.size()) shm_unlink(hname_.c_str());
    if (w_) munmap(w_, sizeof(IpcShm));
  }

  int rank() const override { return me_; }
  int size() const override { return n_; }

  int exchange_count(int nsend, int dest, int src, hipStream_t s) override {
    int nr[1];
    counts(1, &dest, &nsend, &src, nr);
    return nr[0];
  }
  void exchange_count2(int n0, int d0, int src0, int n1, int d1, int src1, hipStream_t s,
                       int nrecv[2]) override {
    const int dd[2] = {d0, d1}, vv[2] = {n0, n1}, ss[2] = {src0, src1};
    counts(2, dd, vv, ss, nrecv);
  }
  void exchange(const void *sbuf, size_t sbytes, int dest, void *rbuf, size_t rbytes, int src,
                hipStream_t s) override {
    Send sd{dest, sbuf, sbytes};
    Recv rv{src, rbuf, rbytes};
    xchg(1, &sd, 1, &rv, s);
  }
  void exchange2(const void *s0, size_t sb0, int d0, void *r0, size_t rb0, int src0,
                 const void *s1, size_t sb1, int d1, void *r1, size_t rb1, int src1,
                 hipStream_t s) override {
    Send sd[2] = {{d0, s0, sb0}, {d1, s1, sb1}};
    Recv rv[2] = {{src0, r0, rb0}, {src1, r1, rb1}};
    xchg(2, sd, 2, rv, s);
  }
  void barrier(hipStream_t s) override {
    SPH_HIP_TRY(hipStreamSynchronize(s));
    host_barrier();
  }
  void exchange_counts_all(const int *scnt, int *rcnt, hipStream_t s) override {
    for (int r = 0; r < n_; r++) w_->r[me_].cnt[r] = scnt[r];
    host_barrier();
    for (int r = 0; r < n_; r++) rcnt[r] = r == me_ ? 0 : w_->r[r].cnt[me_];
    host_barrier();
  }
  void exchange_multi(int n, const int *peer, const void *const *sb, const size_t *sbytes,
                      void *const *rb, const size_t *rbytes, hipStream_t s) override {
    SPH_REQUIRE(n <= IPC_MAXPOST, SPH_HIP_ECOMM, "ipc exchange_multi: %d peers", n);
    std::vector<Send> sd(n);
    std::vector<Recv> rv(n);
    for (int k = 0; k < n; k++) {
      sd[k] = Send{peer[k], sb[k], sbytes[k]};
      rv[k] = Recv{peer[k], rb[k], rbytes[k]};
    }
    xchg(n, sd.data(), n, rv.data(), s);
  }

 private:
  struct Send {
    int dest;
    const void *buf;
    size_t bytes;
  };
  struct Recv {
    int src;
    void *buf;
    size_t bytes;
  };
  struct Peer {
    uint64_t gen = 0;   // generation of the mapping below (0: none)
    void *base = nullptr;
    size_t cap = 0;
    bool host = false;
  };

  static double elapsed(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  static int64_t now_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
  }
  // a peer that has beaten once and not for dead_s_ seconds is gone (its process exited); one
  // that has never beaten attach_s_ after this rank joined died before it attached
  void check_peers() const {
    const int64_t now = now_ns();
    for (int r = 0; r < n_; r++) {
      if (r == me_) continue;
      const int64_t b = w_->r[r].beat.load(std::memory_order_acquire);
      SPH_REQUIRE(b != 0 || elapsed(born_) < attach_s_, SPH_HIP_ECOMM,
                  "ipc world %s: rank %d never joined (%.0f s)", name_.c_str(), r, attach_s_);
      SPH_REQUIRE(b == 0 || (double)(now - b) * 1e-9 < dead_s_, SPH_HIP_ECOMM,
                  "ipc world %s: rank %d has not beaten for %.1f s (its process exited?)",
                  name_.c_str(), r, (double)(now - b) * 1e-9);
    }
  }
  // the host outboxes (name.rR.gG) a killed run of this world name left behind
  void unlink_stale_outboxes() const {
    DIR *d = opendir("/dev/shm");
    if (!d) return;
    const std::string pre = name_.substr(1) + ".r";
    std::vector<std::string> gone;
    while (const struct dirent *e = readdir(d))
      if (strncmp(e->d_name, pre.c_str(), pre.size()) == 0) gone.push_back(std::string("/") + e->d_name);
    closedir(d);
    for (const auto &g : gone) shm_unlink(g.c_str());
  }

  // all ranks meet; bounded wait
  void host_barrier() {
    const long g = w_->generation.load(std::memory_order_acquire);
    if (w_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == n_) {
      w_->arrived.store(0, std::memory_order_relaxed);
      w_->generation.store(g + 1, std::memory_order_release);
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (long spin = 0; w_->generation.load(std::memory_order_acquire) == g; spin++) {
      if (spin < 2000) {
        sched_yield();
        continue;
      }
      if ((spin & 255) == 0) {
        check_peers();
        SPH_REQUIRE(timeout_s_ <= 0.0 || elapsed(t0) < timeout_s_, SPH_HIP_ECOMM,
                    "ipc world %s: rank %d waited %.0f s at a barrier", name_.c_str(), me_,
                    timeout_s_);
      }
      struct timespec ts = {0, 20000};
      nanosleep(&ts, nullptr);
    }
  }

  // the j-th post of rank src addressed to me (j counts earlier requests from src)
  const IpcPost *find_post(int src, int j) const {
    const IpcRankSlot &r = w_->r[src];
    for (int k = 0; k < r.npost; k++)
      if (r.post[k].dest == me_ && j-- == 0) return &r.post[k];
    return nullptr;
  }

  void counts(int n, const int *dest, const int *val, const int *src, int *out) {
    IpcRankSlot &mine = w_->r[me_];
    for (int k = 0; k < n; k++) mine.post[k] = IpcPost{dest[k], val[k], 0, 0};
    mine.npost = n;
    host_barrier();
    std::vector<int> used(n_, 0);
    for (int k = 0; k < n; k++) {
      const IpcPost *p = find_post(src[k], used[src[k]]++);
      SPH_REQUIRE(p, SPH_HIP_ECOMM, "ipc count exchange: nothing from rank %d to %d", src[k], me_);
      out[k] = p->val;
    }
    host_barrier();
  }

  // make room for `bytes` in my outbox (a new generation when it grows; the old one is no
  // longer read: every exchange ends at a barrier after the receivers' copies completed)
  void reserve_box(size_t bytes) {
    IpcRankSlot &mine = w_->r[me_];
    const size_t have = mode_ == SPH_IPC_DEVICE ? dcap_ : hcap_;
    if (bytes <= have && mine.gen.load() != 0) return;
    const size_t cap = std::max<size_t>(bytes + bytes / 4, 1 << 20);
    const uint64_t gen = mine.gen.load() + 1;
    if (mode_ == SPH_IPC_DEVICE) {
      if (dbox_) (void)hipFree(dbox_);
      dbox_ = nullptr;
      SPH_HIP_TRY(hipMalloc(&dbox_, cap));
      dcap_ = cap;
      SPH_HIP_TRY(hipIpcGetMemHandle(&mine.handle, dbox_));
    } else {
      if (hbox_) munmap(hbox_, hcap_);
      if (hname_.size()) shm_unlink(hname_.c_str());
      hbox_ = nullptr;
      hname_ = host_box_name(me_, gen);
      shm_unlink(hname_.c_str());
      int fd = shm_open(hname_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      SPH_REQUIRE(fd >= 0, SPH_HIP_ECOMM, "shm_open(%s): %s", hname_.c_str(), strerror(errno));
      const bool ok = ftruncate(fd, (off_t)cap) == 0;
      void *p = ok ? mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
      close(fd);
      SPH_REQUIRE(p != MAP_FAILED, SPH_HIP_ECOMM, "ipc host outbox %s: %s", hname_.c_str(),
                  strerror(errno));
      hbox_ = static_cast<unsigned char *>(p);
      hcap_ = cap;
    }
    mine.cap = cap;
    mine.gen.store(gen, std::memory_order_release);
  }

  std::string host_box_name(int r, uint64_t gen) const {
    return name_ + ".r" + std::to_string(r) + ".g" + std::to_string(gen);
  }

  void close_peer(Peer &p) {
    if (!p.base) return;
    if (p.host) munmap(p.base, p.cap);
    else (void)hipIpcCloseMemHandle(p.base);
    p = Peer();
  }

  // the peer's current outbox, (re)opened when its generation changed
  const unsigned char *peer_box(int src) {
    if (src == me_)  // loopback: my own outbox (a handle cannot be opened by its exporter)
      return mode_ == SPH_IPC_DEVICE ? dbox_ : hbox_;
    IpcRankSlot &r = w_->r[src];
    const uint64_t gen = r.gen.load(std::memory_order_acquire);
    Peer &p = peer_[src];
    if (p.gen == gen && p.base) return static_cast<const unsigned char *>(p.base);
    close_peer(p);
    if (mode_ == SPH_IPC_DEVICE) {
      void *b = nullptr;
      SPH_HIP_TRY(hipIpcOpenMemHandle(&b, r.handle, hipIpcMemLazyEnablePeerAccess));
      p.base = b;
    } else {
      const std::string nm = host_box_name(src, gen);
      int fd = shm_open(nm.c_str(), O_RDONLY, 0600);
      SPH_REQUIRE(fd >= 0, SPH_HIP_ECOMM, "shm_open(%s): %s", nm.c_str(), strerror(errno));
      void *b = mmap(nullptr, r.cap, PROT_READ, MAP_SHARED, fd, 0);
      close(fd);
      SPH_REQUIRE(b != MAP_FAILED, SPH_HIP_ECOMM, "mmap(%s): %s", nm.c_str(), strerror(errno));
      p.base = b;
      p.host = true;
    }
    p.cap = r.cap;
    p.gen = gen;
    return static_cast<const unsigned char *>(p.base);
  }

  void xchg(int ns, const Send *sd, int nr, const Recv *rv, hipStream_t s) {
    SPH_REQUIRE(ns <= IPC_MAXPOST, SPH_HIP_ECOMM, "ipc exchange: %d sends", ns);
    // stage the sends (256-B aligned) into my outbox
    std::vector<uint64_t> off(ns);
    uint64_t tot = 0;
    for (int k = 0; k < ns; k++) {
      off[k] = tot;
      tot += (sd[k].bytes + 255) & ~(uint64_t)255;
    }
    reserve_box(tot);
    for (int k = 0; k < ns; k++) {
      if (!sd[k].bytes) continue;
      if (mode_ == SPH_IPC_DEVICE)
        SPH_HIP_TRY(hipMemcpyAsync(dbox_ + off[k], sd[k].buf, sd[k].bytes,
                                   hipMemcpyDeviceToDevice, s));
      else
        SPH_HIP_TRY(hipMemcpyAsync(hbox_ + off[k], sd[k].buf, sd[k].bytes,
                                   hipMemcpyDeviceToHost, s));
    }
    SPH_HIP_TRY(hipStreamSynchronize(s));  // staged (and the caller's packing done)
    IpcRankSlot &mine = w_->r[me_];
    for (int k = 0; k < ns; k++) mine.post[k] = IpcPost{sd[k].dest, 0, off[k], sd[k].bytes};
    mine.npost = ns;
    host_barrier();
    std::vector<int> used(n_, 0);
    for (int k = 0; k < nr; k++) {
      const int src = rv[k].src;
      const IpcPost *p = find_post(src, used[src]++);
      SPH_REQUIRE((p && p->bytes == rv[k].bytes) || (!p && rv[k].bytes == 0), SPH_HIP_ECOMM,
                  "ipc exchange mismatch (%d -> %d: %zu bytes expected, %llu posted)", src, me_,
                  rv[k].bytes, p ? (unsigned long long)p->bytes : 0ull);
      if (!rv[k].bytes) continue;
      const unsigned char *b = peer_box(src);
      SPH_HIP_TRY(hipMemcpyAsync(rv[k].buf, b + p->off, rv[k].bytes,
                                 mode_ == SPH_IPC_DEVICE ? hipMemcpyDeviceToDevice
                                                         : hipMemcpyHostToDevice,
                                 s));
    }
    SPH_HIP_TRY(hipStreamSynchronize(s));
    host_barrier();  // the senders may restage their outboxes now
  }

  std::string name_;
  int n_, me_, mode_;
  double timeout_s_ = 0.0;   // SPH_IPC_TIMEOUT: bound on a barrier wait (0: none)
  double dead_s_ = 10.0;     // SPH_IPC_DEAD: a peer silent this long is gone
  double attach_s_ = 120.0;  // creating / joining the world
  std::chrono::steady_clock::time_point born_;
  std::atomic<bool> stop_{false};
  std::thread beater_;
  IpcShm *w_ = nullptr;
  std::vector<Peer> peer_;
  unsigned char *dbox_ = nullptr;
  size_t dcap_ = 0;
  unsigned char *hbox_ = nullptr;
  size_t hcap_ = 0;
  std::string hname_;
};

}  // namespace sph
