// mx_vec.hip -- Vec kernels, deterministic reductions and scans (gfx950).
//
// Element-wise arithmetic follows PETSc's rounding exactly (SURVEY.md §2 N6;
// oracle/petsc_oracle.c): VecAXPY is a fused multiply-add (BLAS daxpy's
// OpenBLAS Haswell/Zen kernel), VecAYPX / VecPointwiseMult / VecScale round
// each operation (PETSc's own C loops, conda-forge -march=nocona).  The library
// is compiled with -ffp-contract=off so nothing else fuses.
//
// Reductions are two-level and deterministic: every block folds its lanes with
// a fixed xor-butterfly (wave64) plus a fixed 4-wave sum, writes one partial,
// and finish_reduce sums the partials in a fixed order.  Results are therefore
// bitwise reproducible run to run (the order differs from PETSc's BLAS ddot,
// which is itself unspecified).
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include "mx_device.hpp"
#include "mx_internal.hpp"

namespace mx {

// Device buffers of 1 MiB or more go through a small per-device cache.
// Assembly allocates and frees its transients (the generated or copied input,
// widened columns, canonical copies) once per call, and destroying an operator
// frees its arrays: over 14 repeated 27-point share assemblies hipFree of a big
// buffer took 7-97 ms in streaks (160 ms assemblies against a 17 ms median;
// tools/asm_outliers.py, tools/asm_time.py, tools/slow_calls.py).  A freed
// buffer is therefore kept (after a device synchronisation, as hipFree would
// do) in a cache of at most min(1/8 of HBM, 48 GiB), oldest evicted first, and
// the next allocation of a similar size takes it back without a driver call;
// mx_finalize, mx_comm_destroy and knob 81 = 0 give it back to the driver.
// Knob 81 = 2: every block handed out is first filled with 0xA5 bytes, so a
// buffer read before it is written shows up (the GPU suite runs green that
// way, profiles/r06a_gpu_suite_poisoned.log).
//
// Every buffer is plain hipMalloc memory.  Physically contiguous allocations
// (hipExtMallocWithFlags(hipDeviceMallocContiguous), rounds 1-5) were retired
// in round 6: once such a block had been freed and its address range taken by
// another allocation, some kernels still reached the old pages through stale
// translations (a whole workgroup's x writes lost, rows
// of freshly generated columns read as zeros, an illegal address) -- with
// them off, 0 failures where they failed every run.
namespace {
struct BigBlock { void *p; size_t bytes; int device; };
std::mutex g_big_mu;
std::vector<BigBlock> g_big_free;                  // cached, oldest first
std::unordered_map<void *, BigBlock> g_big_live;   // cached-size blocks handed out
size_t g_big_bytes = 0;
constexpr size_t BIG_MIN = (size_t)1 << 20;
// sizes are rounded so that near sizes share blocks: 64 KiB below 64 MiB, 2 MiB above
size_t round_size(size_t b) {
  const size_t r = b < ((size_t)64 << 20) ? ((size_t)64 << 10) : ((size_t)2 << 20);
  return (b + r - 1) / r * r;
}

size_t cache_cap() {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); return 0; }
  return std::min(tot / 8, (size_t)48 << 30);
}

// the smallest cached block of this device that fits within 25% slack
bool cache_take(size_t want, int dev, void **p) {
  std::lock_guard<std::mutex> g(g_big_mu);
  int best = -1;
  for (int i = 0; i < (int)g_big_free.size(); ++i) {
    const BigBlock &b = g_big_free[i];
    if (b.device == dev && b.bytes >= want && b.bytes <= want + want / 4 &&
        (best < 0 || b.bytes < g_big_free[best].bytes))
      best = i;
  }
  if (best < 0) return false;
  const BigBlock b = g_big_free[best];
  g_big_free.erase(g_big_free.begin() + best);
  g_big_bytes -= b.bytes;
  g_big_live[b.p] = b;
  *p = b.p;
  return true;
}

hipError_t big_malloc(void **p, size_t bytes) {
  const bool cache = bytes >= BIG_MIN && g_knobs.scratch_cache;
  const size_t want = cache ? round_size(bytes) : bytes;
  auto poison = [&] {
    if (g_knobs.scratch_cache == 2) { HIPCHECK(hipMemset(*p, 0xA5, want)); HIPCHECK(hipDeviceSynchronize()); }
  };
  int dev = 0;
  if (cache) {
    HIPCHECK(hipGetDevice(&dev));
    if (cache_take(want, dev, p)) { poison(); return hipSuccess; }
  }
  hipError_t e = hipMalloc(p, want);
  if (e != hipSuccess && cache) {   // out of memory: give the cache back, then retry once
    (void)hipGetLastError();
    scratch_trim();
    e = hipMalloc(p, want);
  }
  if (e != hipSuccess) return e;
  if (cache) {
    {
      std::lock_guard<std::mutex> g(g_big_mu);
      g_big_live[*p] = BigBlock{*p, want, dev};
    }
    poison();
  }
  return hipSuccess;
}
}  // namespace

hipError_t dev_malloc(void **p, size_t bytes) { return big_malloc(p, bytes); }
hipError_t scratch_malloc(void **p, size_t bytes) { return big_malloc(p, bytes); }

void dev_free(void *p) {
  if (!p) return;
  BigBlock b{nullptr, 0, 0};
  {
    std::lock_guard<std::mutex> g(g_big_mu);
    auto it = g_big_live.find(p);
    if (it != g_big_live.end()) { b = it->second; g_big_live.erase(it); }
  }
  if (!b.p || !g_knobs.scratch_cache) { (void)hipFree(p); return; }
  // hipFree's implicit device synchronisation, kept: whoever takes the block
  // next must not overlap work still queued on it (any stream) -- on the
  // block's own device, whatever device the calling thread has current (a
  // Python finaliser may run on any thread); the capacity is that device's too
  int cur = b.device;
  (void)hipGetDevice(&cur);
  if (cur != b.device) (void)hipSetDevice(b.device);
  (void)hipDeviceSynchronize();
  const size_t cap = cache_cap();
  if (cur != b.device) (void)hipSetDevice(cur);
  std::lock_guard<std::mutex> g(g_big_mu);
  if (b.bytes > cap) { (void)hipFree(p); return; }
  g_big_free.push_back(b);
  g_big_bytes += b.bytes;
  while (g_big_bytes > cap && !g_big_free.empty()) {
    (void)hipFree(g_big_free.front().p);
    g_big_bytes -= g_big_free.front().bytes;
    g_big_free.erase(g_big_free.begin());
  }
}

void scratch_trim() {
  std::lock_guard<std::mutex> g(g_big_mu);
  for (const BigBlock &b : g_big_free) (void)hipFree(b.p);
  g_big_free.clear();
  g_big_bytes = 0;
}

// one block per value: out[v] = sum_b partials[v][b], fixed order (16 loads
// in flight per thread; the same sums as the plain strided loop)
__global__ void __launch_bounds__(256) finish_kernel(const double *__restrict__ partials,
                                                     int nblocks, double *__restrict__ out,
                                                     const int *done) {
  if (done && *done) return;
  const double t = block_sum_array<16>(partials + (size_t)blockIdx.x * nblocks, nblocks);
  if (threadIdx.x == 0) out[blockIdx.x] = t;
}

void finish_reduce(const double *partials, int nblocks, int nvals, double *out, hipStream_t s,
                   int *done_flag) {
  finish_kernel<<<nvals, 256, 0, s>>>(partials, nblocks, out, done_flag);
  HIPCHECK(hipGetLastError());
}

// ------------------------------------------------------------- dot / norm
__global__ void __launch_bounds__(256) dot_partials_kernel(int64_t n, const double *__restrict__ x,
                                                           const double *__restrict__ y,
                                                           double *__restrict__ partials) {
  double v[1] = {0.0};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) v[0] += x[i] * y[i];
  block_sum_to_partials<1>(v, partials, gridDim.x);
}

double host_dot(Comm *c, int64_t n, const double *x, const double *y) {
  if ((int)c->red_scratch.n < RED_BLOCKS + 64) c->red_scratch.alloc(RED_BLOCKS + 64);
  double *part = c->red_scratch.p, *out = c->red_scratch.p + RED_BLOCKS;
  dot_partials_kernel<<<RED_BLOCKS, 256, 0, c->stream>>>(n, x, y, part);
  HIPCHECK(hipGetLastError());
  finish_reduce(part, RED_BLOCKS, 1, out, c->stream);
  c->allreduce_sum(out, 1);
  double h = 0.0;
  HIPCHECK(hipMemcpyAsync(&h, out, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  return h;
}

// cold-cache helper (mx_mat_bench_mult_cold): stream n doubles in with plain
// loads (L2 and the memory-side cache then hold the flush buffer, clean, and
// none of the operator's data); partials: RED_BLOCKS doubles
void flush_read(hipStream_t s, const double *x, int64_t n, double *partials) {
  dot_partials_kernel<<<RED_BLOCKS, 256, 0, s>>>(n, x, x, partials);
  HIPCHECK(hipGetLastError());
}

// ------------------------------------------------------------- VecMDot / VecMAXPY on arbitrary vectors
constexpr int VGROUP = 8;   // vectors per pass
struct VPtrs { const double *p[VGROUP]; double a[VGROUP]; };

// partials[k][b] for the k < nv vectors of this pass (rows in the fixed
// grid-stride order, the deterministic two-level fold of dot_partials_kernel)
__global__ void __launch_bounds__(256) mdot_ptrs_kernel(int64_t n, const double *__restrict__ x, VPtrs y, int nv,
                                                        double *__restrict__ partials) {
  double v[VGROUP];
#pragma unroll
  for (int k = 0; k < VGROUP; ++k) v[k] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double xi = x[i];
#pragma unroll
    for (int k = 0; k < VGROUP; ++k)
      if (k < nv) v[k] += xi * y.p[k][i];
  }
  block_sum_to_partials<VGROUP>(v, partials, gridDim.x);
}

void host_mdot(Comm *c, int64_t n, const double *x, int nv, const double *const *y, double *out_host) {
  if (nv <= 0) return;
  const size_t need = (size_t)VGROUP * RED_BLOCKS + (size_t)nv + 64;
  if (c->red_scratch.n < need) c->red_scratch.alloc(need);
  double *part = c->red_scratch.p, *out = c->red_scratch.p + (size_t)VGROUP * RED_BLOCKS;
  for (int j0 = 0; j0 < nv; j0 += VGROUP) {
    VPtrs pk{};
    const int k = std::min(VGROUP, nv - j0);
    for (int q = 0; q < VGROUP; ++q) pk.p[q] = y[j0 + std::min(q, k - 1)];
    mdot_ptrs_kernel<<<RED_BLOCKS, 256, 0, c->stream>>>(n, x, pk, k, part);
    HIPCHECK(hipGetLastError());
    finish_reduce(part, RED_BLOCKS, k, out + j0, c->stream);
  }
  c->allreduce_sum(out, nv);
  HIPCHECK(hipMemcpyAsync(out_host, out, sizeof(double) * (size_t)nv, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
}

// VecMAXPY_Seq: the first nv % 4 vectors in one PetscKernelAXPY{,2,3} step,
// then groups of four, u = u + (((a0 x0 + a1 x1) + a2 x2) + a3 x3); a pass
// holds whole groups, so storing u between passes changes no bit
template <int REM>
__global__ void __launch_bounds__(256) maxpy_ptrs_kernel(int64_t n, double *__restrict__ y, VPtrs x, int nv) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double u = y[i];
    if constexpr (REM == 1) u = x.a[0] * x.p[0][i] + u;
    else if constexpr (REM == 2) u = u + (x.a[0] * x.p[0][i] + x.a[1] * x.p[1][i]);
    else if constexpr (REM == 3) u = u + ((x.a[0] * x.p[0][i] + x.a[1] * x.p[1][i]) + x.a[2] * x.p[2][i]);
#pragma unroll
    for (int g = REM; g + 3 < VGROUP; g += 4)
      if (g < nv)
        u = u + (((x.a[g] * x.p[g][i] + x.a[g + 1] * x.p[g + 1][i]) + x.a[g + 2] * x.p[g + 2][i]) + x.a[g + 3] * x.p[g + 3][i]);
    y[i] = u;
  }
}

void vec_maxpy(hipStream_t s, int64_t n, double *y, int nv, const double *alpha, const double *const *x) {
  if (nv <= 0 || n <= 0) return;
  int j0 = 0;
  bool first = true;
  while (j0 < nv) {
    // first pass: the remainder plus whole groups; later passes whole groups
    const int rem = first ? nv % 4 : 0;
    const int cnt = first ? std::min(nv, rem + (rem ? 4 : VGROUP)) : std::min(VGROUP, nv - j0);
    VPtrs pk{};
    for (int q = 0; q < VGROUP; ++q) {
      const int src = j0 + std::min(q, cnt - 1);
      pk.p[q] = x[src];
      pk.a[q] = q < cnt ? alpha[src] : 0.0;
    }
    const unsigned g = grid_for(n, 256, 8192);
    switch (rem) {
      case 1: maxpy_ptrs_kernel<1><<<g, 256, 0, s>>>(n, y, pk, cnt); break;
      case 2: maxpy_ptrs_kernel<2><<<g, 256, 0, s>>>(n, y, pk, cnt); break;
      case 3: maxpy_ptrs_kernel<3><<<g, 256, 0, s>>>(n, y, pk, cnt); break;
      default: maxpy_ptrs_kernel<0><<<g, 256, 0, s>>>(n, y, pk, cnt); break;
    }
    HIPCHECK(hipGetLastError());
    j0 += cnt;
    first = false;
  }
}

// ------------------------------------------------------------- element-wise
__global__ void axpy_kernel(int64_t n, double a, const double *__restrict__ x, double *__restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = fma(a, x[i], y[i]);
}
__global__ void aypx_kernel(int64_t n, double a, const double *__restrict__ x, double *__restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = x[i] + a * y[i];
}
__global__ void xmy_kernel(int64_t n, const double *__restrict__ x, double *__restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = x[i] - y[i];
}
__global__ void pmult_kernel(int64_t n, const double *__restrict__ x, const double *__restrict__ y, double *__restrict__ w) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) w[i] = x[i] * y[i];
}
__global__ void scale_kernel(int64_t n, double a, double *__restrict__ x) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = a * x[i];
}
__global__ void set_kernel(int64_t n, double a, double *__restrict__ x) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = a;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__global__ void rhs_hash_kernel(int64_t i0, int64_t n, double *__restrict__ b) {
  const uint64_t seed = 42ULL * 0x9E3779B97F4A7C15ULL;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    b[i] = (double)(splitmix64((uint64_t)(i0 + i) + seed) >> 11) * 0x1.0p-53;
}

constexpr int EW_BLOCK = 256;
static unsigned ew_grid(int64_t n) { return grid_for(n, EW_BLOCK, 8192); }

void vec_axpy(hipStream_t s, int64_t n, double a, const double *x, double *y) {
  if (a == 0.0 || n == 0) return;   // VecAXPY_Seq returns early for alpha == 0
  axpy_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(n, a, x, y);
  HIPCHECK(hipGetLastError());
}
// VecAYPX_Seq: alpha == 0 -> copy, 1 -> VecAXPY, -1 -> x - y, else x + alpha*y
void vec_aypx(hipStream_t s, int64_t n, double a, const double *x, double *y) {
  if (n == 0) return;
  if (a == 0.0) { HIPCHECK(hipMemcpyAsync(y, x, sizeof(double) * n, hipMemcpyDeviceToDevice, s)); return; }
  if (a == 1.0) { vec_axpy(s, n, 1.0, x, y); return; }
  if (a == -1.0) xmy_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(n, x, y);
  else aypx_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(n, a, x, y);
  HIPCHECK(hipGetLastError());
}
void vec_pmult(hipStream_t s, int64_t n, const double *x, const double *y, double *w) {
  if (n == 0) return;
  pmult_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(n, x, y, w);
  HIPCHECK(hipGetLastError());
}
void vec_scale(hipStream_t s, int64_t n, double a, double *x) {
  if (n == 0) return;
  scale_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(n, a, x);
  HIPCHECK(hipGetLastError());
}
void vec_set(hipStream_t s, int64_t n, double a, double *x) {
  if (n == 0) return;
  set_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(n, a, x);
  HIPCHECK(hipGetLastError());
}
void vec_rhs_hash(hipStream_t s, int64_t i0, int64_t n, double *b) {
  if (n == 0) return;
  rhs_hash_kernel<<<ew_grid(n), EW_BLOCK, 0, s>>>(i0, n, b);
  HIPCHECK(hipGetLastError());
}

// ------------------------------------------------------------- PMC calibration stream
typedef double dbl2v __attribute__((ext_vector_type(2)));
template <int W>
__global__ void __launch_bounds__(256) stream_read_kernel(const double *__restrict__ x, int64_t n,
                                                          double *__restrict__ out) {
  double v[1] = {0.0};
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (W == 16) {
    const dbl2v *x2 = reinterpret_cast<const dbl2v *>(x);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n / 2; i += stride) {
      const dbl2v t = __builtin_nontemporal_load(x2 + i);
      v[0] += t.x + t.y;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      v[0] += __builtin_nontemporal_load(x + i);
  }
  block_sum_to_partials<1>(v, out, gridDim.x);
}

void debug_stream_read(hipStream_t s, const double *x, int64_t n, int width, double *out) {
  if (width == 16) stream_read_kernel<16><<<2048, 256, 0, s>>>(x, n, out);
  else stream_read_kernel<8><<<2048, 256, 0, s>>>(x, n, out);
  HIPCHECK(hipGetLastError());
}

// ------------------------------------------------------------- exclusive scan (int64)
constexpr int SCAN_BLOCK = 256, SCAN_ITEMS = 8, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t *total) {
  __shared__ int64_t wsum[SCAN_BLOCK / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  int64_t woff = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < SCAN_BLOCK / 64; ++k) {
    if (k < wid) woff += wsum[k];
    tot += wsum[k];
  }
  __syncthreads();
  *total = tot;
  return woff + incl - v;
}

__global__ void __launch_bounds__(SCAN_BLOCK) scan_reduce_kernel(const int64_t *__restrict__ in, int64_t n,
                                                                 int64_t *__restrict__ bsum) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) if (base + k < n) s += in[base + k];
  int64_t tot;
  (void)block_exclusive_scan(s, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_BLOCK) scan_apply_kernel(const int64_t *__restrict__ in, int64_t n,
                                                                const int64_t *__restrict__ boff,
                                                                int64_t *__restrict__ out,
                                                                int64_t *__restrict__ total_out) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int64_t loc[SCAN_ITEMS];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) { loc[k] = (base + k < n) ? in[base + k] : 0; s += loc[k]; }
  int64_t tot;
  int64_t off = block_exclusive_scan(s, &tot) + (boff ? boff[blockIdx.x] : 0);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (base + k < n) out[base + k] = off;
    off += loc[k];
  }
  if (total_out && blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_BLOCK - 1) *total_out = off;
}

// out may alias in.  total_host (optional) gets sum(in) (synchronises the stream).
void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, hipStream_t s,
                        int64_t *total_host) {
  DBuf<int64_t> tot(1);
  if (n <= 0) {
    if (total_host) *total_host = 0;
    return;
  }
  int64_t nb = cdiv(n, SCAN_TILE);
  if (nb == 1) {
    scan_apply_kernel<<<1, SCAN_BLOCK, 0, s>>>(in, n, nullptr, out, tot.p);
    HIPCHECK(hipGetLastError());
  } else {
    DBuf<int64_t> bsum((size_t)nb);
    scan_reduce_kernel<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(in, n, bsum.p);
    HIPCHECK(hipGetLastError());
    exclusive_scan_i64(bsum.p, bsum.p, nb, s, nullptr);
    scan_apply_kernel<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(in, n, bsum.p, out, tot.p);
    HIPCHECK(hipGetLastError());
    if (total_host) {
      HIPCHECK(hipMemcpyAsync(total_host, tot.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      return;
    }
    HIPCHECK(hipStreamSynchronize(s));  // bsum is freed on return
    return;
  }
  if (total_host) HIPCHECK(hipMemcpyAsync(total_host, tot.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
}

// ------------------------------------------------------------- failure-detection test hook
// one lane spins for about stall_us microseconds of device time, then exits
// (a bounded wait: the grid always drains), so a host wait with a shorter
// deadline can be exercised without a hung peer
__global__ void stall_kernel(long long cycles) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}

void debug_stall(hipStream_t s, int stall_us) {
  if (stall_us < 0 || stall_us > 10000000) fail(MX_ERR_ARG, "stall must be in [0, 10 s]");
  int khz = 100000;                                   // wall_clock64 rate (100 MHz on gfx9)
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  stall_kernel<<<1, 64, 0, s>>>((long long)stall_us * khz / 1000);
  HIPCHECK(hipGetLastError());
}

// this translation unit's code object, loaded now rather than at the first
// launch of one of its kernels (load_code_objects)
void load_code_vec() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&finish_kernel));
  (void)hipGetLastError();
}

}  // namespace mx
