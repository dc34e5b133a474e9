// mx_abi.hip -- extern "C" entry points of libmxsolve.so (declared in include/mxsolve.h).
// Every call: set the handle's device, run, translate exceptions to an error
// code + thread-local message.  No torch types cross this boundary.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mx_internal.hpp"

struct mx_comm_s { mx::Comm *c; };
struct mx_mat_s { mx::Mat *A; };

namespace mx {

static thread_local std::string g_err;

[[noreturn]] void fail(int code, const std::string &msg) { throw Error(code, msg); }

void hip_check(hipError_t e, const char *what, const char *file, int line) {
  if (e != hipSuccess) {
    char buf[512];
    std::snprintf(buf, sizeof buf, "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    fail(e == hipErrorOutOfMemory ? MX_ERR_MEM : MX_ERR_HIP, buf);
  }
}

template <class F> static int guard(F &&f) {
  try {
    f();
    return MX_OK;
  } catch (const Error &e) {
    g_err = e.what();
    return e.code;
  } catch (const std::bad_alloc &) {
    g_err = "host allocation failed";
    return MX_ERR_MEM;
  } catch (const std::exception &e) {
    g_err = e.what();
    return MX_ERR_INTERNAL;
  }
}

static Comm *C(mx_comm c) {
  if (!c || !c->c) fail(MX_ERR_ARG, "null communicator");
  HIPCHECK(hipSetDevice(c->c->device));
  return c->c;
}
static Mat *M(mx_mat a) {
  if (!a || !a->A) fail(MX_ERR_ARG, "null matrix");
  HIPCHECK(hipSetDevice(a->A->comm->device));
  return a->A;
}

}  // namespace mx

using namespace mx;

extern "C" {

int mx_version(void) { return MX_ABI_VERSION; }

int mx_last_error(char *buf, size_t len) {
  if (buf && len) {
    std::strncpy(buf, g_err.c_str(), len - 1);
    buf[len - 1] = 0;
  }
  return (int)g_err.size();
}

int mx_get_unique_id(void *out, size_t len) { return guard([&] { get_unique_id(out, len); }); }


int mx_comm_create_rccl(int rank, int size, int device, const void *uid, size_t uid_len, mx_comm *out) {
  return guard([&] {
    if (size < 1 || rank < 0 || rank >= size) fail(MX_ERR_ARG, "bad rank/size");
    *out = new mx_comm_s{make_rccl_comm(rank, size, device, uid, uid_len)};
    load_code_objects();
  });
}

int mx_comm_create_shm(int rank, int size, int device, const char *name, int64_t slot_kib, mx_comm *out) {
  return guard([&] {
    if (size < 1 || rank < 0 || rank >= size) fail(MX_ERR_ARG, "bad rank/size");
    if (!name || name[0] != '/') fail(MX_ERR_ARG, "shared-memory name must start with '/'");
    *out = new mx_comm_s{make_shm_comm(rank, size, device, name, slot_kib)};
    load_code_objects();
  });
}

int mx_comm_abort(mx_comm c) { return guard([&] { if (c && c->c) abort_comm_async(c->c); }); }

int mx_comm_create_self(int device, mx_comm *out) {
  return guard([&] {
    *out = new mx_comm_s{make_self_comm(device)};
    load_code_objects();
  });
}

int mx_world_create_local(int size, void **world) { return guard([&] { *world = make_local_world(size); }); }

int mx_comm_create_local(void *world, int rank, int device, mx_comm *out) {
  return guard([&] {
    *out = new mx_comm_s{make_local_comm(world, rank, device)};
    load_code_objects();
  });
}

int mx_world_destroy(void *world) { return guard([&] { destroy_local_world(world); }); }
int mx_world_abort(void *world) { return guard([&] { abort_local_world(world); }); }

int mx_comm_destroy(mx_comm c) {
  return guard([&] {
    if (!c) return;
    if (c->c) { (void)hipSetDevice(c->c->device); delete c->c; }
    delete c;
    scratch_trim();   // cached assembly transients go back to the driver
  });
}

int mx_comm_info(mx_comm c, int *rank, int *size, int *device) {
  return guard([&] {
    Comm *k = C(c);
    if (rank) *rank = k->rank;
    if (size) *size = k->size;
    if (device) *device = k->device;
  });
}

int mx_comm_stream(mx_comm c, void **stream) { return guard([&] { *stream = (void *)C(c)->stream; }); }

int mx_comm_barrier(mx_comm c) { return guard([&] { C(c)->barrier(); }); }

int mx_layout_split(int64_t N, int P, int64_t *ranges) {
  return guard([&] {
    if (P < 1 || N < 0) fail(MX_ERR_ARG, "bad layout");
    const int64_t q = N / P, r = N % P;
    ranges[0] = 0;
    for (int i = 0; i < P; ++i) ranges[i + 1] = ranges[i] + q + (i < r ? 1 : 0);
  });
}

// Host-to-device copy of a caller's (pageable) arrays for createAIJ(csr=...):
// indptr, cols and vals go through ONE pipeline of chunks.  The pages wholly
// inside an array of PIN_MIN bytes or more are page-locked in place
// (hipHostRegister) chunk by chunk, copied, and unregistered once the copy is
// done; registration runs ahead on H2D_REG_THREADS host threads (a chunk of
// fresh numpy pages takes longer to lock than its DMA) while the calling
// thread issues the copies in order.  Chunk sizes ramp from 4 MiB to 64 MiB,
// so the first copy starts after a 4 MiB registration (0.25 ms) rather than a
// 64 MiB one (4 ms); one pipeline over the three arrays avoids a drain and a
// ramp per array (tools/h2d_pin_probe.hip, tools/h2d_lib_probe.py).
// Everything else -- arrays under PIN_MIN, the partial first and last pages
// of a pinned one (never registered, so arrays that share a page never hold
// overlapping registrations), a chunk whose registration fails -- is a plain
// (runtime-staged) copy.  PIN_MIN is 128 MiB: with 1 MiB the GPU suite, which
// assembles many operators from moderate host arrays, twice ended in an
// illegal address during these copies; at 128 MiB
// registration serves the large payloads it pays for.
struct H2dSeg { void *dst; const void *src; size_t bytes; };
constexpr int H2D_REG_THREADS = 4;
constexpr size_t H2D_PIN_MIN = (size_t)128 << 20;
static void h2d_pinned(const std::vector<H2dSeg> &segs, hipStream_t st, size_t pin_min = H2D_PIN_MIN) {
  constexpr size_t CH0 = (size_t)4 << 20, CH = (size_t)64 << 20, PAGE = 4096;
  struct Cut { char *dst; uintptr_t a, b; bool pin; };
  std::vector<Cut> cuts;
  size_t k = 0;    // pinned chunks cut so far (the ramp)
  for (const H2dSeg &g : segs) {
    if (!g.bytes) continue;
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(g.src), s1 = s0 + g.bytes;
    const uintptr_t p0 = (s0 + PAGE - 1) & ~(uintptr_t)(PAGE - 1), p1 = s1 & ~(uintptr_t)(PAGE - 1);
    char *d0 = static_cast<char *>(g.dst);
    if (g.bytes < pin_min || p1 <= p0) { cuts.push_back({d0, s0, s1, false}); continue; }
    if (p0 > s0) cuts.push_back({d0, s0, p0, false});
    for (uintptr_t a = p0; a < p1; ++k) {   // page-aligned chunks: no page registered twice
      const uintptr_t b = std::min<uintptr_t>(p1, a + std::min(CH, CH0 << std::min<size_t>(k, 4)));
      cuts.push_back({d0 + (a - s0), a, b, true});
      a = b;
    }
    if (s1 > p1) cuts.push_back({d0 + (p1 - s0), p1, s1, false});
  }
  struct Chunk { char *dst; uintptr_t a, b; bool pin; std::atomic<int> state{0}; hipEvent_t ev = nullptr; };  // 0 pending, 1 pinned, 2 not pinned
  const size_t n = cuts.size();
  std::vector<Chunk> ch(n);
  size_t npin = 0;
  for (size_t i = 0; i < n; ++i) {
    Chunk &c = ch[i];
    c.dst = cuts[i].dst; c.a = cuts[i].a; c.b = cuts[i].b; c.pin = cuts[i].pin;
    if (!c.pin) c.state.store(2);
    npin += c.pin;
  }
  std::atomic<bool> stop{false};
  std::vector<std::thread> reg;
  const int nt = npin ? (int)std::min<size_t>(H2D_REG_THREADS, n) : 0;
  for (int t = 0; t < nt; ++t)
    reg.emplace_back([&, t] {
      for (size_t i = (size_t)t; i < n && !stop.load(); i += (size_t)nt) {
        if (!ch[i].pin) continue;
        const bool ok = hipHostRegister(reinterpret_cast<void *>(ch[i].a), ch[i].b - ch[i].a, hipHostRegisterDefault) == hipSuccess;
        ch[i].state.store(ok ? 1 : 2, std::memory_order_release);
      }
    });
  auto finish = [&] {
    stop.store(true);
    for (auto &t : reg) t.join();
    (void)hipStreamSynchronize(st);
    for (Chunk &c : ch) {
      if (c.ev) (void)hipEventDestroy(c.ev);
      if (c.state.load() == 1) (void)hipHostUnregister(reinterpret_cast<void *>(c.a));
      c.state.store(0);
    }
    (void)hipGetLastError();   // failed registrations
  };
  try {
    size_t done = 0;   // chunks released
    for (size_t i = 0; i < n; ++i) {
      while (ch[i].state.load(std::memory_order_acquire) == 0) std::this_thread::yield();
      HIPCHECK(hipMemcpyAsync(ch[i].dst, reinterpret_cast<const void *>(ch[i].a), ch[i].b - ch[i].a,
                              hipMemcpyHostToDevice, st));
      if (!ch[i].pin) continue;
      HIPCHECK(hipEventCreateWithFlags(&ch[i].ev, hipEventDisableTiming));
      HIPCHECK(hipEventRecord(ch[i].ev, st));
      // two pinned chunks in flight: release the older ones
      for (; done < i; ++done) {
        if (!ch[done].ev) continue;
        size_t later = 0;
        for (size_t j = done + 1; j <= i; ++j) later += ch[j].ev != nullptr;
        if (later < 2) break;
        HIPCHECK(hipEventSynchronize(ch[done].ev));
        if (ch[done].state.load() == 1) (void)hipHostUnregister(reinterpret_cast<void *>(ch[done].a));
        ch[done].state.store(0);
      }
    }
  } catch (...) {
    finish();
    throw;
  }
  finish();
}

int mx_mat_create_csr(mx_comm c, int64_t Mg, int64_t Ng, int64_t m_local, int64_t n_local,
                      const void *indptr, int indptr_bytes, const void *cols, int col_bytes,
                      const double *vals, int64_t nnz, int insert_mode, int src_is_device, mx_mat *A) {
  return guard([&] {
    Comm *k = C(c);
    const double t0 = wall_ms();
    g_asm_times = AsmTimes{};
    if (Mg < 0 || Ng < 0) fail(MX_ERR_ARG, "negative global size");
    if ((indptr_bytes != 4 && indptr_bytes != 8) || (col_bytes != 4 && col_bytes != 8))
      fail(MX_ERR_ARG, "index width must be 4 or 8 bytes");
    // local row count for the argument checks (the same split assemble() uses)
    int64_t m = m_local;
    if (m < 0) { const int64_t q = Mg / k->size, r = Mg % k->size; m = q + (k->rank < r ? 1 : 0); }
    hipStream_t st = k->stream;
    // 32-bit columns (scipy's default index type) are read as is by the
    // fused assembly passes: a device array directly, a host array after its
    // copy; 64-bit ones are copied / taken as is too
    const bool c32 = col_bytes == 4;
    DBuf<int64_t> ip((size_t)m + 1, kScratch), cl(kScratch);
    DBuf<int32_t> cl32(kScratch);
    if (!src_is_device) { if (c32) cl32.alloc((size_t)(nnz > 0 ? nnz : 1)); else cl.alloc((size_t)(nnz > 0 ? nnz : 1)); }
    DBuf<double> vl((size_t)(src_is_device && nnz > 0 ? 0 : (nnz > 0 ? nnz : 1)), kScratch);
    // host-side copies of the two scalars petsc4py checks
    int64_t first = 0, last = 0;
    if (src_is_device) {
      convert_index(indptr, indptr_bytes, m + 1, ip.p, st);
      HIPCHECK(hipMemcpyAsync(&first, ip.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      HIPCHECK(hipMemcpyAsync(&last, ip.p + m, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
    } else {
      auto rd = [&](int64_t i) -> int64_t {
        return indptr_bytes == 8 ? static_cast<const int64_t *>(indptr)[i] : static_cast<const int32_t *>(indptr)[i];
      };
      first = rd(0);
      last = rd(m);
    }
    if (first != 0) fail(MX_ERR_ARG, "I[0] is " + std::to_string(first) + ", expected 0");
    if (last != nnz) fail(MX_ERR_ARG, "size(J) is " + std::to_string(nnz) + ", expected " + std::to_string(last));
    double t_copy = wall_ms();
    if (!src_is_device) {
      DBuf<char> stage((size_t)(m + 1) * indptr_bytes + 8, kScratch);
      t_copy = wall_ms();   // the copy phase starts once its buffers exist
      g_asm_times.alloc_ms = t_copy - t0;
      std::vector<H2dSeg> segs{{stage.p, indptr, (size_t)(m + 1) * indptr_bytes}};
      if (nnz) {
        segs.push_back({c32 ? (void *)cl32.p : (void *)cl.p, cols, (size_t)nnz * col_bytes});
        segs.push_back({vl.p, vals, sizeof(double) * nnz});
      }
      h2d_pinned(segs, st);
      convert_index(stage.p, indptr_bytes, m + 1, ip.p, st);
      HIPCHECK(hipStreamSynchronize(st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    const double t_h2d = wall_ms();
    AssemblyInput in;
    if (src_is_device) {
      if (c32) in.cols32 = static_cast<const int32_t *>(cols);
      else in.cols = static_cast<const int64_t *>(cols);
    } else {
      in.cols = cl.p; in.cols32 = cl32.p;
    }
    if (!in.cols && !in.cols32) { cl.alloc(1); in.cols = cl.p; }   // nnz == 0 from device
    in.rowptr = ip.p; in.vals = src_is_device && nnz ? vals : vl.p; in.nnz = nnz;
    in.insert_mode = insert_mode;
    *A = new mx_mat_s{assemble(k, Mg, Ng, m_local, n_local, in)};
    g_asm_times.h2d_ms = t_h2d - t_copy;
    g_asm_times.host_bytes = src_is_device ? 0.0 : (double)(m + 1) * indptr_bytes + (double)nnz * (col_bytes + 8);
    g_asm_times.total_ms = wall_ms() - t0;
  });
}

int mx_mat_create_coo(mx_comm c, int64_t Mg, int64_t Ng, int64_t m_local, int64_t n_local,
                      const int64_t *rows, const int64_t *cols, const double *vals, int64_t n,
                      int insert_mode, int src_is_device, mx_mat *A) {
  return guard([&] {
    Comm *k = C(c);
    hipStream_t st = k->stream;
    const size_t cnt = (size_t)(n > 0 ? n : 1);
    DBuf<int64_t> r(cnt, kScratch), cl(cnt, kScratch);
    DBuf<double> v(cnt, kScratch);
    if (n) {
      const hipMemcpyKind kind = src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
      HIPCHECK(hipMemcpyAsync(r.p, rows, sizeof(int64_t) * n, kind, st));
      HIPCHECK(hipMemcpyAsync(cl.p, cols, sizeof(int64_t) * n, kind, st));
      HIPCHECK(hipMemcpyAsync(v.p, vals, sizeof(double) * n, kind, st));
    }
    AssemblyInput in;
    in.coo_rows = r.p; in.cols = cl.p; in.vals = v.p; in.nnz = n; in.insert_mode = insert_mode;
    *A = new mx_mat_s{assemble(k, Mg, Ng, m_local, n_local, in)};
  });
}

int mx_mat_create_stencil(mx_comm c, int kind, int64_t nx, int64_t ny, int64_t nz, mx_mat *A) {
  return guard([&] {
    Comm *k = C(c);
    if (kind < 0 || kind > 3 || nx < 1 || ny < 1 || nz < 1) fail(MX_ERR_ARG, "bad stencil");
    const int64_t Mg = kind == 0 ? nx * ny : nx * ny * nz;
    const int64_t q = Mg / k->size, r = Mg % k->size;
    int64_t row0 = 0;
    for (int i = 0; i < k->rank; ++i) row0 += q + (i < r ? 1 : 0);
    const int64_t m = q + (k->rank < r ? 1 : 0);
    DBuf<int64_t> rp(kScratch), cl(kScratch);
    DBuf<int32_t> cl32(kScratch);
    DBuf<double> vl(kScratch);
    stencil_coo(k, kind, nx, ny, nz, row0, m, rp, cl, cl32, vl);
    AssemblyInput in;
    in.rowptr = rp.p; in.cols = cl.p; in.cols32 = cl32.p; in.vals = vl.p;
    in.nnz = m * (kind == 0 ? 5 : (kind == 2 ? 27 : 7));
    in.insert_mode = MX_INSERT_VALUES;
    *A = new mx_mat_s{assemble(k, Mg, Mg, -1, -1, in)};
  });
}

int mx_mat_get_info(mx_mat a, mx_mat_info *info) {
  return guard([&] {
    Mat *A = M(a);
    std::memset(info, 0, sizeof(*info));
    info->M = A->M; info->N = A->N; info->m = A->m; info->n = A->n;
    info->rstart = A->rstart; info->cstart = A->cstart;
    info->nnz_d = A->nnz_d; info->nnz_o = A->nnz_o; info->nghost = A->nghost;
    info->sell_slots_d = A->sd.slots; info->sell_slots_o = A->so.slots;
    info->nsend_peers = (int)A->halo.send_peer.size();
    info->nrecv_peers = (int)A->halo.recv_peer.size();
    info->nsend = A->halo.nsend; info->nrecv = A->halo.nrecv;
    info->dia_slices = A->sd.dia_slices;
    info->value_codes = A->sd.ntab;
    info->code_bytes = A->sd.code_bytes;
    info->pair_shape = A->sd.ntab > 0 ? A->sd.pair_shape : 0;
    info->pair_units = info->pair_shape ? A->sd.pair_used : 0;
    info->pair_blocks = info->pair_shape ? A->sd.pair_blocks : 0;
    info->pair_block_bytes = info->pair_shape ? 64 * (int64_t)((2 * A->sd.dia_k + 15) / 16 * 16) : 0;
    info->pair_uniform = info->pair_shape && info->pair_blocks > 0 && (A->sd.puni.p || A->sd.puni27.p) ? 1 : 0;
    info->pair_lean = pair_lean_kind(A);
    info->pair_zmarch = info->pair_lean && pair_zm_applies(A) ? 1 : 0;
    // the fp64 row-pair z-march runs only where the launch takes it: one rank,
    // or a product that splits (otherwise the general kernel continues A_o)
    info->pair_f64 = (A->nghost == 0 || matmult_splits(A)) ? pair_f64_kind(A) : 0;
    info->pair_form27 = A->sd.pair_shape == 27 && pair_lean_kind(A)
                            ? (pair_lean_kind(A) == 2 ? (A->sd.pcol27.p ? 2 : 1) : 0) : -1;
    info->pair_code = pair_code_applies(A) && (A->nghost == 0 || matmult_splits(A)) ? 1 : 0;
    info->cb_blocks = (A->nghost == 0 || matmult_splits(A)) ? A->sd.cb_nblk : 0;   // where it runs (cb_applies)
  });
}

int mx_mat_get_split(mx_mat a, int64_t *dptr, int32_t *dcol, double *dval, int64_t *optr,
                     int32_t *ocol, double *oval, int64_t *garray) {
  return guard([&] {
    Mat *A = M(a);
    hipStream_t st = A->comm->stream;
    auto d2h = [&](void *dst, const void *src, size_t bytes) {
      if (dst && bytes) HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    };
    d2h(dptr, A->dptr.p, sizeof(int64_t) * (A->m + 1));
    d2h(optr, A->optr.p, sizeof(int64_t) * (A->m + 1));
    d2h(dcol, A->dcol.p, sizeof(int32_t) * A->nnz_d);
    d2h(dval, A->dval.p, sizeof(double) * A->nnz_d);
    d2h(ocol, A->ocol.p, sizeof(int32_t) * A->nnz_o);
    d2h(oval, A->oval.p, sizeof(double) * A->nnz_o);
    d2h(garray, A->garray.p, sizeof(int64_t) * A->nghost);
    HIPCHECK(hipStreamSynchronize(st));
  });
}

int mx_mat_get_csr(mx_mat a, int64_t *indptr, int64_t *cols, double *vals) {
  return guard([&] {
    Mat *A = M(a);
    const int64_t m = A->m;
    std::vector<int64_t> dp(m + 1), op(m + 1), g(A->garray_h);
    std::vector<int32_t> dc(A->nnz_d), oc(A->nnz_o);
    std::vector<double> dv(A->nnz_d), ov(A->nnz_o);
    hipStream_t st = A->comm->stream;
    HIPCHECK(hipMemcpyAsync(dp.data(), A->dptr.p, sizeof(int64_t) * (m + 1), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(op.data(), A->optr.p, sizeof(int64_t) * (m + 1), hipMemcpyDeviceToHost, st));
    if (A->nnz_d) {
      HIPCHECK(hipMemcpyAsync(dc.data(), A->dcol.p, sizeof(int32_t) * A->nnz_d, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipMemcpyAsync(dv.data(), A->dval.p, sizeof(double) * A->nnz_d, hipMemcpyDeviceToHost, st));
    }
    if (A->nnz_o) {
      HIPCHECK(hipMemcpyAsync(oc.data(), A->ocol.p, sizeof(int32_t) * A->nnz_o, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipMemcpyAsync(ov.data(), A->oval.p, sizeof(double) * A->nnz_o, hipMemcpyDeviceToHost, st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    // MatGetRow_MPIAIJ merge: ghosts left of cstart, diagonal block, ghosts right
    int64_t p = 0;
    indptr[0] = 0;
    for (int64_t i = 0; i < m; ++i) {
      int64_t o = op[i];
      const int64_t oe = op[i + 1];
      for (; o < oe && g[oc[o]] < A->cstart; ++o) { cols[p] = g[oc[o]]; vals[p++] = ov[o]; }
      for (int64_t d = dp[i]; d < dp[i + 1]; ++d) { cols[p] = dc[d] + A->cstart; vals[p++] = dv[d]; }
      for (; o < oe; ++o) { cols[p] = g[oc[o]]; vals[p++] = ov[o]; }
      indptr[i + 1] = p;
    }
  });
}

int mx_mat_mult(mx_mat a, const double *x, double *y) {
  return guard([&] {
    Mat *A = M(a);
    mat_mult(A, x, y);
    HIPCHECK(hipStreamSynchronize(A->comm->stream));
  });
}

int mx_mat_get_diagonal(mx_mat a, double *d) {
  return guard([&] {
    Mat *A = M(a);
    if (A->m) HIPCHECK(hipMemcpyAsync(d, A->diag.p, sizeof(double) * A->m, hipMemcpyDeviceToDevice, A->comm->stream));
    HIPCHECK(hipStreamSynchronize(A->comm->stream));
  });
}

int mx_debug_comm_bench(mx_comm c, mx_mat a, int what, int iters, double *us_per) {
  return guard([&] {
    Comm *cm = C(c);
    hipStream_t st = cm->stream;
    if (iters < 1) fail(MX_ERR_ARG, "iters must be positive");
    if (what == 2 && !a) fail(MX_ERR_ARG, "halo bench needs a matrix");
    if ((int)cm->red_scratch.n < 64) cm->red_scratch.alloc(64);
    DBuf<double> xv;
    if (what == 2) { xv.alloc((size_t)std::max<int64_t>(M(a)->m, 1)); HIPCHECK(hipMemsetAsync(xv.p, 0, sizeof(double) * xv.n, st)); }
    auto once = [&] {
      if (what == 2) halo_begin(M(a), xv.p);
      else cm->allreduce_sum(cm->red_scratch.p, what == 1 ? 3 : 1);
    };
    once();                                  // warm (connections, buffers)
    cm->barrier();
    hipEvent_t e0, e1;
    HIPCHECK(hipEventCreate(&e0));
    HIPCHECK(hipEventCreate(&e1));
    HIPCHECK(hipEventRecord(e0, st));
    for (int k = 0; k < iters; ++k) once();
    HIPCHECK(hipEventRecord(e1, st));
    HIPCHECK(hipEventSynchronize(e1));
    float t = 0.f;
    HIPCHECK(hipEventElapsedTime(&t, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *us_per = 1e3 * (double)t / iters;
  });
}

int mx_mat_bench_mult(mx_mat a, const double *x, double *y, int iters, double *spmv_ms, double *mult_ms) {
  return guard([&] {
    Mat *A = M(a);
    hipStream_t st = A->comm->stream;
    if (iters < 1) fail(MX_ERR_ARG, "iters must be positive");
    std::vector<hipEvent_t> ev(2 * (size_t)iters + 2);
    for (auto &e : ev) HIPCHECK(hipEventCreate(&e));
    mat_mult(A, x, y);  // warm
    HIPCHECK(hipEventRecord(ev[0], st));
    for (int k = 0; k < iters; ++k) {
      HIPCHECK(hipEventRecord(ev[2 + 2 * k], st));
      matmult_overlap(A, x, y, SPMV_PLAIN, Jac{}, nullptr, nullptr);
      HIPCHECK(hipEventRecord(ev[3 + 2 * k], st));
    }
    HIPCHECK(hipEventRecord(ev[1], st));
    HIPCHECK(hipEventSynchronize(ev[1]));
    double s = 0.0;
    for (int k = 0; k < iters; ++k) {
      float t = 0.f;
      HIPCHECK(hipEventElapsedTime(&t, ev[2 + 2 * k], ev[3 + 2 * k]));
      s += t;
    }
    float tot = 0.f;
    HIPCHECK(hipEventElapsedTime(&tot, ev[0], ev[1]));
    for (auto &e : ev) (void)hipEventDestroy(e);
    if (spmv_ms) *spmv_ms = s / iters;
    if (mult_ms) *mult_ms = (double)tot / iters;
  });
}

int mx_mat_bench_mult_cold(mx_mat a, const double *x, double *y, double *flush, int64_t flush_n, int iters,
                           double *spmv_ms, double *mult_ms) {
  return guard([&] {
    Mat *A = M(a);
    hipStream_t st = A->comm->stream;
    if (iters < 1 || !flush || flush_n < 1) fail(MX_ERR_ARG, "cold MatMult: iters and a flush buffer are needed");
    Comm *cm = A->comm;
    if (cm->red_scratch.n < (size_t)RED_BLOCKS + 64) cm->red_scratch.alloc((size_t)RED_BLOCKS + 64);
    hipEvent_t ev[4];
    for (auto &e : ev) HIPCHECK(hipEventCreate(&e));
    std::vector<double> ks, ms;
    for (int k = 0; k < iters; ++k) {
      flush_read(st, flush, flush_n, cm->red_scratch.p);   // the host enqueues the rest while this runs
      HIPCHECK(hipEventRecord(ev[0], st));
      const bool ext = A->comm->size == 1;
      if (ext) g_ext_timing = ExtTiming{ev[2], ev[3], true, false};
      matmult_overlap(A, x, y, SPMV_PLAIN, Jac{}, nullptr, nullptr);
      const bool used = ext && g_ext_timing.used;
      g_ext_timing = ExtTiming{};
      HIPCHECK(hipEventRecord(ev[1], st));
      HIPCHECK(hipEventSynchronize(ev[1]));
      float t = 0.f, u = 0.f;
      HIPCHECK(hipEventElapsedTime(&t, ev[0], ev[1]));
      if (used) HIPCHECK(hipEventElapsedTime(&u, ev[2], ev[3]));
      ms.push_back(t);
      ks.push_back(used ? u : -1.0);
    }
    for (auto &e : ev) (void)hipEventDestroy(e);
    std::sort(ms.begin(), ms.end());
    std::sort(ks.begin(), ks.end());
    if (mult_ms) *mult_ms = ms[ms.size() / 2];
    if (spmv_ms) *spmv_ms = ks[ks.size() / 2];
  });
}

int mx_mat_destroy(mx_mat a) {
  return guard([&] {
    if (!a) return;
    if (a->A) {
      (void)hipSetDevice(a->A->comm->device);
      (void)hipStreamSynchronize(a->A->comm->stream);
      delete a->A;
    }
    delete a;
  });
}

int mx_vec_dot(mx_comm c, int64_t n, const double *x, const double *y, double *out) {
  return guard([&] { *out = host_dot(C(c), n, x, y); });
}
int mx_vec_norm2(mx_comm c, int64_t n, const double *x, double *out) {
  return guard([&] { *out = std::sqrt(host_dot(C(c), n, x, x)); });
}
int mx_vec_axpy(mx_comm c, int64_t n, double a, const double *x, double *y) {
  return guard([&] { Comm *k = C(c); vec_axpy(k->stream, n, a, x, y); HIPCHECK(hipStreamSynchronize(k->stream)); });
}
int mx_vec_aypx(mx_comm c, int64_t n, double a, const double *x, double *y) {
  return guard([&] { Comm *k = C(c); vec_aypx(k->stream, n, a, x, y); HIPCHECK(hipStreamSynchronize(k->stream)); });
}
int mx_vec_pointwise_mult(mx_comm c, int64_t n, const double *x, const double *y, double *w) {
  return guard([&] { Comm *k = C(c); vec_pmult(k->stream, n, x, y, w); HIPCHECK(hipStreamSynchronize(k->stream)); });
}
int mx_vec_scale(mx_comm c, int64_t n, double a, double *x) {
  return guard([&] { Comm *k = C(c); vec_scale(k->stream, n, a, x); HIPCHECK(hipStreamSynchronize(k->stream)); });
}
int mx_vec_set(mx_comm c, int64_t n, double a, double *x) {
  return guard([&] { Comm *k = C(c); vec_set(k->stream, n, a, x); HIPCHECK(hipStreamSynchronize(k->stream)); });
}
int mx_debug_comm_stall(mx_comm c, int stall_us) {
  return guard([&] {
    Comm *k = C(c);
    debug_stall(k->stream, stall_us);
    k->wait_stream(k->stream);
  });
}
int mx_vec_mdot(mx_comm c, int64_t n, const double *x, int nv, const double *const *y, double *out) {
  return guard([&] {
    if (nv < 0 || (nv > 0 && (!y || !out))) fail(MX_ERR_ARG, "VecMDot: bad vector list");
    host_mdot(C(c), n, x, nv, y, out);
  });
}
int mx_vec_maxpy(mx_comm c, int64_t n, double *y, int nv, const double *alpha, const double *const *x) {
  return guard([&] {
    if (nv < 0 || (nv > 0 && (!x || !alpha))) fail(MX_ERR_ARG, "VecMAXPY: bad vector list");
    Comm *k = C(c);
    vec_maxpy(k->stream, n, y, nv, alpha, x);
    HIPCHECK(hipStreamSynchronize(k->stream));
  });
}
int mx_ksp_destroy(mx_mat a) {
  return guard([&] {
    Mat *A = M(a);
    (void)hipSetDevice(A->comm->device);
    HIPCHECK(hipStreamSynchronize(A->comm->stream));
    A->release_ksp();
  });
}
int mx_finalize(void) {
  return guard([&] {
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess) nd = 0;
    for (int d = 0; d < nd; ++d) {
      if (hipSetDevice(d) == hipSuccess) HIPCHECK(hipDeviceSynchronize());
    }
    (void)hipGetLastError();
    scratch_trim();   // the device buffer cache goes back to the driver
  });
}
int mx_vec_rhs_hash(mx_comm c, int64_t i0, int64_t n, double *b) {
  return guard([&] { Comm *k = C(c); vec_rhs_hash(k->stream, i0, n, b); HIPCHECK(hipStreamSynchronize(k->stream)); });
}

void mx_ksp_default_params(mx_ksp_params *p) {
  std::memset(p, 0, sizeof(*p));
  p->ksp_type = MX_KSP_GMRES;   // PETSc's default KSP
  p->pc_type = MX_PC_JACOBI;
  p->norm_type = MX_NORM_DEFAULT;
  p->max_it = 10000;
  p->restart = 30;
  p->rtol = 1e-5;
  p->atol = 1e-50;
  p->dtol = 1e5;
  p->haptol = 1e-30;
  p->breakdowntol = 0.1;
  p->poll_every = 16;
}

int mx_lu_solve_csr(mx_comm c, int64_t n, const int64_t *indptr, const int64_t *cols,
                    const double *vals, const double *b, double *x) {
  return guard([&] { dense_lu_solve(C(c), n, indptr, cols, vals, b, x); });
}

int mx_dev_alloc(int device, size_t bytes, void **ptr) {
  return guard([&] {
    HIPCHECK(hipSetDevice(device));
    *ptr = nullptr;
    if (bytes && dev_malloc(ptr, bytes) != hipSuccess) { *ptr = nullptr; fail(MX_ERR_MEM, "device allocation failed"); }
  });
}

int mx_dev_free(void *ptr) { return guard([&] { dev_free(ptr); }); }

int mx_debug_set(int key, int value) {
  int old = -1;
  switch (key) {
    case 6: old = g_knobs.overlap; g_knobs.overlap = value; break;
    case 7: old = g_knobs.graph; g_knobs.graph = value; break;
    case 8: old = g_knobs.force_coll; g_knobs.force_coll = value; break;
    case 9: old = g_knobs.cg_fuse; g_knobs.cg_fuse = value; break;
    case 13: old = g_knobs.cg_vec; g_knobs.cg_vec = value; break;
    case 21: old = g_knobs.cg_unroll; g_knobs.cg_unroll = value; break;
    case 23: old = g_knobs.vcodes; g_knobs.vcodes = value; break;
    case 27: old = g_knobs.spmv_pairs; g_knobs.spmv_pairs = value; break;
    case 29: old = g_knobs.cg_xbatch; g_knobs.cg_xbatch = value; break;
    case 33: old = g_knobs.comm_timeout_ms; if (value > 0) g_knobs.comm_timeout_ms = value; break;
    case 38: old = g_knobs.pair_lean; g_knobs.pair_lean = value; break;
    case 39: old = g_knobs.pair_zm; g_knobs.pair_zm = value; break;
    case 40: old = g_knobs.pair_zm_bpc; g_knobs.pair_zm_bpc = std::min(std::max(value, 1), 8); break;
    case 41: old = g_knobs.pair_zm_len; g_knobs.pair_zm_len = std::min(std::max(value, 1), 1024); break;
    case 43: old = g_knobs.spmv_fp64_grid; g_knobs.spmv_fp64_grid = std::min(std::max(value, 0), 65536); break;
    case 47: old = g_knobs.comm_wait_ms; g_knobs.comm_wait_ms = std::max(value, 0); break;
    case 48: old = g_knobs.pair_col27; g_knobs.pair_col27 = value; break;
    case 52: old = g_knobs.pair_zmc; g_knobs.pair_zmc = value; break;
    case 53: old = g_knobs.pair_unitv; g_knobs.pair_unitv = value; break;
    case 60: old = g_knobs.pair_zm27p; g_knobs.pair_zm27p = value; break;
    case 70: old = g_knobs.zm27_2line; g_knobs.zm27_2line = value; break;
    case 72: old = g_knobs.asm_fused; g_knobs.asm_fused = value; break;
    case 80: old = g_knobs.cg_pbws; g_knobs.cg_pbws = value; break;
    case 81: old = g_knobs.scratch_cache; g_knobs.scratch_cache = value; if (!value) scratch_trim(); break;
    case 84: old = g_knobs.cb; g_knobs.cb = value; break;
    case 69: old = g_knobs.cg_pbw; g_knobs.cg_pbw = value; break;
    case 68: old = g_knobs.ru_2line; g_knobs.ru_2line = value; break;
    case 61: old = g_knobs.gm_stall_us; g_knobs.gm_stall_us = std::min(std::max(value, 0), 2000000); break;
    case 59: old = g_knobs.pw_sym27; g_knobs.pw_sym27 = value; break;
    default: break;
  }
  return old;
}

int mx_debug_assembly_times(double *out, int n) {
  const AsmTimes &t = g_asm_times;
  const double v[8] = {t.h2d_ms, t.canon_ms, t.split_ms, t.layout_ms, t.halo_ms, t.total_ms, t.host_bytes, t.alloc_ms};
  for (int k = 0; k < n && k < 8; ++k) out[k] = v[k];
  return 0;
}

int mx_debug_dispatch_counts(int64_t *out, int n, int reset) {
  for (int k = 0; k < DSP_COUNT; ++k) {
    const long long v = reset ? g_dispatch[k].exchange(0) : g_dispatch[k].load();
    if (out && k < n) out[k] = v;
  }
  return 0;
}

int mx_debug_stream_read(mx_comm c, const double *x, int64_t n, int width, double *out) {
  return guard([&] {
    Comm *k = C(c);
    debug_stream_read(k->stream, x, n, width, out);
    HIPCHECK(hipStreamSynchronize(k->stream));
  });
}

int mx_ksp_solve(mx_mat a, const mx_ksp_params *p, const double *b, double *x, mx_ksp_result *res,
                 double *history) {
  return guard([&] {
    Mat *A = M(a);
    ksp_solve(A, *p, b, x, *res, history);
  });
}

}  // extern "C"

namespace mx {
// The process's first pipelined copy (threads registering chunks while copies
// run) is ~1 ms slower on 1.47 GB than later ones; the first pinned transfer
// alone costs ~8 ms more.  Paid once at initialisation (load_code_objects) on
// a 32 MiB buffer: four chunks (4, 8, 16, 4 MiB) on the four registration
// threads (tools/h2d_sweep.py, profiles/r06w_h2d_*.txt).
void h2d_warm() {
  constexpr size_t W = (size_t)32 << 20;
  char *h = static_cast<char *>(std::aligned_alloc(4096, W));
  void *d = nullptr;
  hipStream_t st = nullptr;
  if (h && hipMalloc(&d, W) == hipSuccess && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
    std::memset(h, 0, W);
    try {
      h2d_pinned({{d, h, W}}, st, (size_t)1 << 20);   // this buffer is the library's own: registered
    } catch (const Error &) {
    }
  }
  if (st) (void)hipStreamDestroy(st);
  if (d) (void)hipFree(d);
  std::free(h);
  (void)hipGetLastError();
}
}  // namespace mx
