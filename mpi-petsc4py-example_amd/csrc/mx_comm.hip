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
//   * SelfComm : size 1.
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <mutex>

#include "mx_internal.hpp"

namespace mx {

Comm::~Comm() {}

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
    if (nc) ncclCommDestroy(nc);
    if (stream) (void)hipStreamDestroy(stream);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
  }
  void allreduce_sum(double *dev, int n) override {
    if ((size == 1 && !g_knobs.force_coll) || n <= 0) return;
    NCCLCHECK(ncclAllReduce(dev, dev, (size_t)n, ncclDouble, ncclSum, nc, stream));
  }
  void exchange(const std::vector<Msg> &sends, const std::vector<Msg> &recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return;
    if (!s) s = stream;
    NCCLCHECK(ncclGroupStart());
    for (const Msg &m : sends) NCCLCHECK(ncclSend(m.buf, m.bytes, ncclUint8, m.peer, nc, s));
    for (const Msg &m : recvs) NCCLCHECK(ncclRecv(m.buf, m.bytes, ncclUint8, m.peer, nc, s));
    NCCLCHECK(ncclGroupEnd());
  }
  void alltoall_i64(const int64_t *send, int64_t *recv) override {
    HIPCHECK(hipMemcpyAsync(i64buf.p, send, sizeof(int64_t) * size, hipMemcpyHostToDevice, stream));
    NCCLCHECK(ncclGroupStart());
    for (int q = 0; q < size; ++q) {
      NCCLCHECK(ncclSend(i64buf.p + q, 1, ncclInt64, q, nc, stream));
      NCCLCHECK(ncclRecv(i64buf.p + size + q, 1, ncclInt64, q, nc, stream));
    }
    NCCLCHECK(ncclGroupEnd());
    HIPCHECK(hipMemcpyAsync(recv, i64buf.p + size, sizeof(int64_t) * size, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }
  void allgather_i64(int64_t v, int64_t *all) override {
    HIPCHECK(hipMemcpyAsync(i64buf.p, &v, sizeof(int64_t), hipMemcpyHostToDevice, stream));
    NCCLCHECK(ncclAllGather(i64buf.p, i64buf.p + size, 1, ncclInt64, nc, stream));
    HIPCHECK(hipMemcpyAsync(all, i64buf.p + size, sizeof(int64_t) * size, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }
  void barrier() override {
    HIPCHECK(hipMemsetAsync(i64buf.p, 0, sizeof(int64_t), stream));
    NCCLCHECK(ncclAllReduce(i64buf.p, i64buf.p, 1, ncclInt64, ncclSum, nc, stream));
    HIPCHECK(hipStreamSynchronize(stream));
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
  std::vector<int> tags;        // collective each rank entered (mismatch = error, not a race)
  bool broken = false;          // a rank failed: every barrier throws instead of waiting
  explicit LocalWorld(int s) : size(s), red_ptr(s), posted(s), slots((size_t)s * s), tags(s) {}
  // tag: which collective the caller is in; all ranks must agree
  void barrier(int rank = -1, int tag = 0) {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) fail(MX_ERR_COMM, "local world: another rank failed");
    if (rank >= 0) tags[rank] = tag;
    long g = gen;
    if (++arrived == size) { arrived = 0; gen++; cv.notify_all(); }
    else cv.wait(lk, [&] { return gen != g || broken; });
    if (broken) fail(MX_ERR_COMM, "local world: another rank failed");
    if (rank >= 0)
      for (int q = 0; q < size; ++q)
        if (tags[q] != tag) {
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
    w->barrier();                  // every rank has read every dev
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
    w->barrier();                  // the senders' buffers may be overwritten now
  }

  void alltoall_i64(const int64_t *send, int64_t *recv) override {
    for (int q = 0; q < size; ++q) w->slots[(size_t)rank * size + q] = send[q];
    w->barrier(rank, 3);
    for (int q = 0; q < size; ++q) recv[q] = w->slots[(size_t)q * size + rank];
    w->barrier();
  }
  void allgather_i64(int64_t v, int64_t *all) override {
    w->slots[rank] = v;
    w->barrier(rank, 4);
    for (int q = 0; q < size; ++q) all[q] = w->slots[q];
    w->barrier();
  }
  void barrier() override {
    HIPCHECK(hipStreamSynchronize(stream));
    w->barrier(rank, 5);
  }
};

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

}  // namespace mx
