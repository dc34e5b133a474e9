// mx_comm.cpp -- communicators for device data.
//
// Replaces the MPI layer PETSc uses inside MatMult (VecScatter/PetscSF
// Isend/Irecv) and inside VecDot/VecNorm (MPI_Allreduce), SURVEY.md §2 N5/N6.
//   * RcclComm : one process per GPU, RCCL over xGMI.  Halo = grouped
//                ncclSend/ncclRecv with the neighbour ranks; reductions =
//                ncclAllReduce(SUM) of a handful of doubles, all on the
//                rank's compute stream so the solve never syncs the host.
//   * LocalComm: P virtual ranks inside one process sharing one GPU, each
//                driven from its own host thread.  Same semantics, payloads
//                moved by D2D copies ordered with events.  Used to exercise
//                the N>1 path on a single-GPU box (RCCL refuses two ranks on
//                one device).
//   * ShmComm  : P processes of one node that may share GPUs (more ranks than
//                devices, where RCCL refuses two ranks on one device): device
//                payloads staged through a POSIX shared-memory segment, host
//                ordered.  A correctness transport (mpiexec -n 2 of test.py on
//                a one-GPU machine), not a fast path.
//   * SelfComm : size 1.
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>

#include "mx_internal.hpp"
#include "mx_shm_barrier.hpp"

namespace mx {

Comm::~Comm() {}

void Comm::wait_until(const std::function<bool()> &ready, hipStream_t s, const std::function<long long()> &,
                      long long) {
  hipStream_t q = s ? s : stream;
  for (int spins = 0; !ready(); ++spins) {
    if ((spins & 63) == 63) {
      const hipError_t e = hipStreamQuery(q);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) HIPCHECK(e);
      if (spins > 4096) sched_yield();
    }
  }
}

static hipStream_t new_stream(int device) {
  HIPCHECK(hipSetDevice(device));
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}

// ------------------------------------------------------------------ self
struct SelfComm : Comm {
  explicit SelfComm(int dev) { device = dev; rank = 0; size = 1; stream = new_stream(dev); }
  ~SelfComm() override { if (stream) (void)hipStreamDestroy(stream); }
  void allreduce_sum(double *, int) override {}
  void exchange(const std::vector<Msg> &s, const std::vector<Msg> &r, hipStream_t) override {
    if (!s.empty() || !r.empty()) fail(MX_ERR_INTERNAL, "self communicator has no peers");
  }
  void alltoall_i64(const int64_t *s, int64_t *r) override { r[0] = s[0]; }
  void allgather_i64(int64_t v, int64_t *all) override { all[0] = v; }
  void barrier() override {}
};

Comm *make_self_comm(int device) { return new SelfComm(device); }

// ------------------------------------------------------------------ RCCL
#define NCCLCHECK(x)                                                                   \
  do {                                                                                 \
    ncclResult_t _r = (x);                                                             \
    if (_r != ncclSuccess)                                                             \
      fail(MX_ERR_COMM, std::string(#x) + ": " + ncclGetErrorString(_r));              \
  } while (0)

void get_unique_id(void *out, size_t len) {
  if (len < sizeof(ncclUniqueId)) fail(MX_ERR_ARG, "unique id buffer too small");
  ncclUniqueId id;
  NCCLCHECK(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
}

struct RcclComm : Comm {
  ncclComm_t nc = nullptr;
  DBuf<int64_t> i64buf;
  RcclComm(int r, int s, int dev, const void *uid, size_t len) {
    rank = r; size = s; device = dev;
    if (len < sizeof(ncclUniqueId)) fail(MX_ERR_ARG, "bad RCCL unique id length");
    stream = new_stream(dev);
    comm_stream = new_stream(dev);
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    NCCLCHECK(ncclCommInitRank(&nc, s, id, r));
    i64buf.alloc(2 * (size_t)s);
  }
  ~RcclComm() override {
    if (nc && !aborted) ncclCommDestroy(nc);   // (an aborted communicator is freed by ncclCommAbort)
    if (stream) (void)hipStreamDestroy(stream);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
  }
  void allreduce_sum(double *dev, int n) override {
    if ((size == 1 && !g_knobs.force_coll) || n <= 0) return;
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    NCCLCHECK(ncclAllReduce(dev, dev, (size_t)n, ncclDouble, ncclSum, nc, stream));
  }
  void exchange(const std::vector<Msg> &sends, const std::vector<Msg> &recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return;
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    if (!s) s = stream;
    NCCLCHECK(ncclGroupStart());
    for (const Msg &m : sends) NCCLCHECK(ncclSend(m.buf, m.bytes, ncclUint8, m.peer, nc, s));
    for (const Msg &m : recvs) NCCLCHECK(ncclRecv(m.buf, m.bytes, ncclUint8, m.peer, nc, s));
    NCCLCHECK(ncclGroupEnd());
  }
  void alltoall_i64(const int64_t *send, int64_t *recv) override {
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    HIPCHECK(hipMemcpyAsync(i64buf.p, send, sizeof(int64_t) * size, hipMemcpyHostToDevice, stream));
    NCCLCHECK(ncclGroupStart());
    for (int q = 0; q < size; ++q) {
      NCCLCHECK(ncclSend(i64buf.p + q, 1, ncclInt64, q, nc, stream));
      NCCLCHECK(ncclRecv(i64buf.p + size + q, 1, ncclInt64, q, nc, stream));
    }
    NCCLCHECK(ncclGroupEnd());
    HIPCHECK(hipMemcpyAsync(recv, i64buf.p + size, sizeof(int64_t) * size, hipMemcpyDeviceToHost, stream));
    wait_stream(stream);
  }
  void allgather_i64(int64_t v, int64_t *all) override {
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    HIPCHECK(hipMemcpyAsync(i64buf.p, &v, sizeof(int64_t), hipMemcpyHostToDevice, stream));
    NCCLCHECK(ncclAllGather(i64buf.p, i64buf.p + size, 1, ncclInt64, nc, stream));
    HIPCHECK(hipMemcpyAsync(all, i64buf.p + size, sizeof(int64_t) * size, hipMemcpyDeviceToHost, stream));
    wait_stream(stream);
  }
  void barrier() override {
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    HIPCHECK(hipMemsetAsync(i64buf.p, 0, sizeof(int64_t), stream));
    NCCLCHECK(ncclAllReduce(i64buf.p, i64buf.p, 1, ncclInt64, ncclSum, nc, stream));
    wait_stream(stream);
  }
  // Failure detection: poll the device work and RCCL's
  // asynchronous error state.  An RCCL error aborts the communicator at once
  // (this rank fails with MX_ERR_COMM rather than waiting forever on a peer
  // that died).  Deadlines: a wait that can observe progress (the KSP poller:
  // the count of iterations begun, which the device advances) fails after
  // knob 33 ms (default 120 s) WITHOUT progress -- the timer re-arms whenever
  // the count moves, so a long healthy solve never trips it; a wait that
  // cannot (stream/event waits, setup collectives, barrier) fails after knob
  // 47 ms (default 600 s: a slow peer, e.g. one still building its CSR on the
  // host, is not an error, but a dead one on a transport that reports no
  // asynchronous error does not hang the rank forever; 0 = no deadline).
  // GMRES's restart read-back observes progress (gm_step_kernel stores a step
  // count into the host word), so it runs under knob 33 like the CG poller.
  // A progress wait is armed (knob 33) only once the count has moved off the
  // caller's baseline -- the device has begun the waited-for work, so every
  // rank has entered it; before that a rank whose peers enter the solve late
  // (host work between solves) waits under knob 47 like any other wait.
  template <class Q> void watch(Q query, const char *what, const std::function<long long()> &progress = {},
                                long long baseline = 0) {
    int limit = g_knobs.comm_wait_ms;
    auto t0 = std::chrono::steady_clock::now();
    long long seen = baseline;
    bool armed = false;
    for (int spins = 0;; ++spins) {
      const hipError_t e = query();
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) HIPCHECK(e);
      // aborted from another thread (mx_comm_abort: a caller's wall-time
      // budget ran out): the RCCL kernels have been told to stop
      if (aborted) fail(MX_ERR_COMM, std::string(what) + ": RCCL communicator aborted");
      ncclResult_t ar = ncclSuccess;
      if (ncclCommGetAsyncError(nc, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress) {
        abort_comm();
        fail(MX_ERR_COMM, std::string(what) + ": RCCL asynchronous error: " + ncclGetErrorString(ar));
      }
      const auto now = std::chrono::steady_clock::now();
      if (progress) {
        const long long p = progress();
        if (p != seen) {
          seen = p;
          t0 = now;
          if (!armed) { armed = true; limit = g_knobs.comm_timeout_ms; }
        }
      }
      if (limit > 0) {
        if (now - t0 > std::chrono::milliseconds(limit)) {
          abort_comm();
          fail(MX_ERR_COMM, std::string(what) + ": no progress for " + std::to_string(limit) +
                                " ms; RCCL communicator aborted");
        }
      }
      if (spins > 200) usleep(50); else sched_yield();
    }
  }
  // Callable from any thread (mx_comm_abort), once: ncclCommAbort stops the
  // communicator's in-flight kernels and frees it; every later call on this
  // rank fails with MX_ERR_COMM (nc is kept, and never used again)
  void abort_comm() {
    if (!aborted.exchange(true) && nc) (void)ncclCommAbort(nc);
  }
  std::atomic<bool> aborted{false};
  void wait_stream(hipStream_t s) override {
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    hipStream_t q = s ? s : stream;
    watch([&] { return hipStreamQuery(q); }, "stream wait");
  }
  void wait_event(hipEvent_t ev) override {
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    watch([&] { return hipEventQuery(ev); }, "event wait");
  }
  void wait_until(const std::function<bool()> &ready, hipStream_t s,
                  const std::function<long long()> &progress, long long baseline) override {
    if (aborted) fail(MX_ERR_COMM, "RCCL communicator was aborted");
    hipStream_t q = s ? s : stream;
    watch([&] { return ready() ? hipSuccess : hipStreamQuery(q); }, "progress wait", progress, baseline);
  }
};

Comm *make_rccl_comm(int rank, int size, int device, const void *uid, size_t len) {
  return new RcclComm(rank, size, device, uid, len);
}

// ------------------------------------------------------------------ local (in-process)
constexpr int LOCAL_MAX = 16;

struct LocalWorld {
  int size;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  std::vector<double *> red_ptr;
  std::vector<std::vector<Msg>> posted;
  std::vector<int64_t> slots;
  // collective each rank entered, one row per generation parity: a rank
  // released from generation g may enter g+1 (and write its tag there) while
  // a slower one still checks the tags of g; g+2 cannot start before every
  // rank has left g.  Unchecked barriers record tag 0, so a checked barrier
  // meeting an unchecked one fails too (mismatch = error, not a race).
  std::vector<int> tags[2];
  bool broken = false;          // a rank failed: every barrier throws instead of waiting
  explicit LocalWorld(int s) : size(s), red_ptr(s), posted(s), slots((size_t)s * s) { tags[0].resize(s); tags[1].resize(s); }
  // tag: which collective the caller is in (0: not checked); all ranks must agree
  void barrier(int rank, int tag = 0) {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) fail(MX_ERR_COMM, "local world: another rank failed");
    long g = gen;
    std::vector<int> &tg = tags[g & 1];
    tg[rank] = tag;
    if (++arrived == size) { arrived = 0; gen++; cv.notify_all(); }
    else cv.wait(lk, [&] { return gen != g || broken; });
    if (broken) fail(MX_ERR_COMM, "local world: another rank failed");
    if (tag != 0)
      for (int q = 0; q < size; ++q)
        if (tg[q] != tag) {
          broken = true;
          cv.notify_all();
          fail(MX_ERR_COMM, "local world: ranks entered different collectives");
        }
  }
  void abort_all() {
    std::lock_guard<std::mutex> lk(mu);
    broken = true;
    cv.notify_all();
  }
};

struct PtrPack { const double *p[LOCAL_MAX]; };

// out[j] = sum_q in[q][j], ranks in order (deterministic).
__global__ void local_sum_kernel(PtrPack in, int P, int n, double *out) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = in.p[0][j];
  for (int q = 1; q < P; ++q) s = s + in.p[q][j];
  out[j] = s;
}

struct LocalComm : Comm {
  LocalWorld *w;
  DBuf<double> tmp;
  LocalComm(LocalWorld *world, int r, int dev) : w(world) {
    rank = r; size = world->size; device = dev; stream = new_stream(dev);
    capturable = false;
    comm_stream = new_stream(dev);
  }
  ~LocalComm() override {
    if (stream) (void)hipStreamDestroy(stream);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
  }

  // Host-ordered: a rank's stream is drained before its buffers are
  // published and again before peers may reuse them, so no HIP object is
  // shared between the rank threads (test-only communicator).
  void allreduce_sum(double *dev, int n) override {
    if (size == 1 || n <= 0) return;
    if ((int)tmp.n < n) tmp.alloc((size_t)n < 64 ? 64 : (size_t)n);
    HIPCHECK(hipStreamSynchronize(stream));
    w->red_ptr[rank] = dev;
    w->barrier(rank, 1000 + n);
    PtrPack pk;
    for (int q = 0; q < size; ++q) pk.p[q] = w->red_ptr[q];
    local_sum_kernel<<<grid_for(n, 256), 256, 0, stream>>>(pk, size, n, tmp.p);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(stream));
    w->barrier(rank);              // every rank has read every dev
    HIPCHECK(hipMemcpyAsync(dev, tmp.p, sizeof(double) * n, hipMemcpyDeviceToDevice, stream));
  }

  void exchange(const std::vector<Msg> &sends, const std::vector<Msg> &recvs, hipStream_t st) override {
    if (!st) st = stream;
    HIPCHECK(hipStreamSynchronize(st));
    w->posted[rank] = sends;
    w->barrier(rank, 2);
    for (const Msg &r : recvs) {
      const Msg *src = nullptr;
      for (const Msg &s : w->posted[r.peer]) if (s.peer == rank) { src = &s; break; }
      if (!src || src->bytes != r.bytes) fail(MX_ERR_COMM, "local exchange: unmatched message");
      if (r.bytes) HIPCHECK(hipMemcpyAsync(r.buf, src->buf, r.bytes, hipMemcpyDeviceToDevice, st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    w->barrier(rank);              // the senders' buffers may be overwritten now
  }

  void alltoall_i64(const int64_t *send, int64_t *recv) override {
    for (int q = 0; q < size; ++q) w->slots[(size_t)rank * size + q] = send[q];
    w->barrier(rank, 3);
    for (int q = 0; q < size; ++q) recv[q] = w->slots[(size_t)q * size + rank];
    w->barrier(rank);
  }
  void allgather_i64(int64_t v, int64_t *all) override {
    w->slots[rank] = v;
    w->barrier(rank, 4);
    for (int q = 0; q < size; ++q) all[q] = w->slots[q];
    w->barrier(rank);
  }
  void barrier() override {
    HIPCHECK(hipStreamSynchronize(stream));
    w->barrier(rank, 5);
  }
};

// ------------------------------------------------------------------ shared memory (processes)
// Segment: a header (barrier words, an abort flag, per-rank int64 scratch and
// message directories) followed by one staging slot per rank.  Every
// collective is a sequence of "write my slot -> barrier -> read peers' slots
// -> barrier"; device data moves by synchronous copies on the rank's stream.
constexpr int SHM_DIR = 2 * SHM_MAX;       // message directory entries per rank
struct ShmDirEnt { int64_t peer, off, bytes; };
struct ShmHeader {
  ShmBarrierWords bar;                      // mx_shm_barrier.hpp
  std::atomic<int> opened;
  int size, pad;
  int64_t slot_bytes;
  int64_t scratch[SHM_MAX][SHM_MAX];        // [rank][k]: small all-to-all / all-gather payloads
  int64_t ndir[SHM_MAX];
  ShmDirEnt dir[SHM_MAX][SHM_DIR];
};

struct ShmComm : Comm {
  ShmHeader *h = nullptr;
  char *base = nullptr;
  size_t map_bytes = 0;
  std::vector<double> tmp;
  ShmComm(int r, int s, int dev, const char *name, int64_t slot_kib) {
    rank = r; size = s; device = dev;
    capturable = false;
    if (s < 1 || s > SHM_MAX) fail(MX_ERR_ARG, "shared-memory communicator size must be in [1, 64]");
    if (slot_kib < 1) slot_kib = 64 << 10;
    const int64_t slot = slot_kib << 10;
    map_bytes = sizeof(ShmHeader) + (size_t)s * (size_t)slot;
    int fd = -1;
    if (r == 0) {
      fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) fail(MX_ERR_COMM, std::string("shm_open(create) failed for ") + name);
      if (ftruncate(fd, (off_t)map_bytes) != 0) { close(fd); shm_unlink(name); fail(MX_ERR_MEM, "ftruncate of the shared segment failed"); }
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while ((fd = shm_open(name, O_RDWR, 0600)) < 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
          fail(MX_ERR_COMM, std::string("shm_open timed out for ") + name);
        usleep(1000);
      }
      // wait until rank 0 has sized it
      const auto t1 = std::chrono::steady_clock::now();
      for (;;) {
        off_t sz = lseek(fd, 0, SEEK_END);
        if (sz >= (off_t)map_bytes) break;
        if (std::chrono::steady_clock::now() - t1 > std::chrono::seconds(120)) { close(fd); fail(MX_ERR_COMM, "shared segment never sized"); }
        usleep(1000);
      }
    }
    void *m = mmap(nullptr, map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) fail(MX_ERR_MEM, "mmap of the shared segment failed");
    h = static_cast<ShmHeader *>(m);
    base = static_cast<char *>(m) + sizeof(ShmHeader);
    if (r == 0) {
      h->size = s;
      h->slot_bytes = slot;
      shm_barrier_init(&h->bar);
      h->opened.store(1, std::memory_order_release);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (h->opened.load(std::memory_order_acquire) < 1) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) fail(MX_ERR_COMM, "shared segment never initialised");
        usleep(1000);
      }
      if (h->size != s || h->slot_bytes != slot) fail(MX_ERR_COMM, "shared segment size mismatch between ranks");
      h->opened.fetch_add(1);
    }
    stream = new_stream(dev);
    comm_stream = new_stream(dev);
    wait_barrier(-1, 0);                    // everyone mapped it
    if (r == 0) shm_unlink(name);           // the mappings keep it alive
  }
  ~ShmComm() override {
    if (stream) (void)hipStreamDestroy(stream);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
    if (h) munmap(h, map_bytes);
  }
  char *slot(int q) { return base + (size_t)q * (size_t)h->slot_bytes; }

  // generation barrier with collective tags (mx_shm_barrier.hpp)
  void wait_barrier(int tag, int check) {
    switch (shm_barrier_wait(&h->bar, rank, size, tag, check != 0, std::chrono::seconds(600))) {
      case BarrierResult::ok: return;
      case BarrierResult::peer_failed: fail(MX_ERR_COMM, "shared-memory world: another rank failed");
      case BarrierResult::timeout: fail(MX_ERR_COMM, "shared-memory barrier timed out");
      case BarrierResult::mismatch: fail(MX_ERR_COMM, "shared-memory world: ranks entered different collectives");
    }
  }

  void allreduce_sum(double *dev, int n) override {
    if (size == 1 || n <= 0) return;
    if ((int64_t)n * 8 > h->slot_bytes) fail(MX_ERR_ARG, "all-reduce larger than the shared slot");
    HIPCHECK(hipMemcpyAsync(slot(rank), dev, sizeof(double) * n, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    wait_barrier(1000 + n, 1);
    tmp.assign((size_t)n, 0.0);
    for (int j = 0; j < n; ++j) {                 // ranks in order: the same bits everywhere
      double t = reinterpret_cast<double *>(slot(0))[j];
      for (int q = 1; q < size; ++q) t = t + reinterpret_cast<double *>(slot(q))[j];
      tmp[(size_t)j] = t;
    }
    wait_barrier(0, 0);                           // every rank has read every slot
    HIPCHECK(hipMemcpyAsync(dev, tmp.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }

  // Each rank's messages form one byte stream staged slot_bytes at a time;
  // all ranks run the same number of rounds (the largest stream decides).
  void exchange(const std::vector<Msg> &sends, const std::vector<Msg> &recvs, hipStream_t st) override {
    if (!st) st = stream;
    HIPCHECK(hipStreamSynchronize(st));
    if ((int)sends.size() > SHM_DIR) fail(MX_ERR_ARG, "too many messages for the shared-memory directory");
    int64_t total = 0;
    h->ndir[rank] = (int64_t)sends.size();
    for (size_t i = 0; i < sends.size(); ++i) {
      h->dir[rank][i] = ShmDirEnt{sends[i].peer, total, (int64_t)sends[i].bytes};
      total += (int64_t)sends[i].bytes;
    }
    const int64_t cap = h->slot_bytes;
    h->scratch[rank][0] = (total + cap - 1) / cap;
    wait_barrier(2, 1);
    int64_t rounds = 0;
    for (int q = 0; q < size; ++q) rounds = std::max(rounds, h->scratch[q][0]);
    for (const Msg &r : recvs) {                  // the sender must have one message for us, of this size
      bool ok = false;
      for (int64_t e = 0; e < h->ndir[r.peer]; ++e)
        if (h->dir[r.peer][e].peer == rank) { ok = h->dir[r.peer][e].bytes == (int64_t)r.bytes; break; }
      if (!ok) { h->bar.abort.store(1); fail(MX_ERR_COMM, "shared-memory exchange: unmatched message"); }
    }
    for (int64_t rd = 0; rd < rounds; ++rd) {
      const int64_t lo = rd * cap, hi = lo + cap;
      for (size_t i = 0; i < sends.size(); ++i) {   // stage my part of this round
        const ShmDirEnt &d = h->dir[rank][i];
        const int64_t a = std::max(lo, d.off), b = std::min(hi, d.off + d.bytes);
        if (a < b)
          HIPCHECK(hipMemcpyAsync(slot(rank) + (a - lo), static_cast<const char *>(sends[i].buf) + (a - d.off),
                                  (size_t)(b - a), hipMemcpyDeviceToHost, st));
      }
      HIPCHECK(hipStreamSynchronize(st));
      wait_barrier(0, 0);
      for (const Msg &r : recvs) {                  // collect what peers staged for me
        for (int64_t e = 0; e < h->ndir[r.peer]; ++e) {
          const ShmDirEnt &d = h->dir[r.peer][e];
          if (d.peer != rank) continue;
          const int64_t a = std::max(lo, d.off), b = std::min(hi, d.off + d.bytes);
          if (a < b)
            HIPCHECK(hipMemcpyAsync(static_cast<char *>(r.buf) + (a - d.off), slot(r.peer) + (a - lo),
                                    (size_t)(b - a), hipMemcpyHostToDevice, st));
          break;
        }
      }
      HIPCHECK(hipStreamSynchronize(st));
      wait_barrier(0, 0);
    }
    // no rounds: peers may still read this rank's directory and round count
    if (rounds == 0) wait_barrier(0, 0);
  }

  void alltoall_i64(const int64_t *send, int64_t *recv) override {
    for (int q = 0; q < size; ++q) h->scratch[rank][q] = send[q];
    wait_barrier(3, 1);
    for (int q = 0; q < size; ++q) recv[q] = h->scratch[q][rank];
    wait_barrier(0, 0);
  }
  void allgather_i64(int64_t v, int64_t *all) override {
    h->scratch[rank][0] = v;
    wait_barrier(4, 1);
    for (int q = 0; q < size; ++q) all[q] = h->scratch[q][0];
    wait_barrier(0, 0);
  }
  void barrier() override {
    HIPCHECK(hipStreamSynchronize(stream));
    wait_barrier(5, 1);
  }
  void abort_world() { if (h) h->bar.abort.store(1); }
};

Comm *make_shm_comm(int rank, int size, int device, const char *name, int64_t slot_kib) {
  return new ShmComm(rank, size, device, name, slot_kib);
}
void abort_comm_async(Comm *c) {
  if (auto *s = dynamic_cast<ShmComm *>(c)) s->abort_world();
  else if (auto *r = dynamic_cast<RcclComm *>(c)) r->abort_comm();
}

void *make_local_world(int size) {
  if (size < 1 || size > LOCAL_MAX) fail(MX_ERR_ARG, "local world size must be in [1, 16]");
  return new LocalWorld(size);
}
Comm *make_local_comm(void *world, int rank, int device) {
  auto *w = static_cast<LocalWorld *>(world);
  if (rank < 0 || rank >= w->size) fail(MX_ERR_ARG, "bad rank for local world");
  return new LocalComm(w, rank, device);
}
void destroy_local_world(void *world) { delete static_cast<LocalWorld *>(world); }
void abort_local_world(void *world) { static_cast<LocalWorld *>(world)->abort_all(); }

// this translation unit's code object, loaded now rather than at the first
// launch of one of its kernels (load_code_objects)
void load_code_comm() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&local_sum_kernel));
  (void)hipGetLastError();
}

void load_code_objects() {
  // the one-time costs of the first pinned, pipelined host-to-device copy
  // (createAIJ from host arrays: mx_abi.hip h2d_pinned), paid at
  // initialisation once per process
  static std::once_flag once;
  std::call_once(once, [] { h2d_warm(); });
  load_code_comm();
  load_code_vec();
  load_code_assembly();
  load_code_spmv();
  load_code_spmv_pair();
  load_code_spmv_cb();
  load_code_ksp();
  load_code_direct();
}

}  // namespace mx
