// colblock_probe.hip -- a two-pass random-pattern SpMV prototype (the
// unstructured AIJ MatMult, test.py:14's matrix family at 2^lg rows x 7).
//
// The one-pass SELL kernel gathers x[c] per entry: uniformly random 8-B reads,
// one L2 miss (a 64-B sector from the memory side) each, and its rate is set
// by those misses (tools/gather_probe: the gathers alone take 94% of it).
// Two passes instead:
//   pass 1 (column blocks): the entries sorted by (column block, row, column);
//     XCD k walks the column blocks k, k + 8, ... so a block's slice of x
//     (2^BS doubles) stays in that XCD's L2 while every CU of it streams the
//     block's values and column ids and writes prod[k] = v * x[c] in that
//     order (sequential);
//   pass 2 (rows): SELL-64 over the products -- y_i = sum of row i's
//     products in ascending column order, read through perm (entry j of the
//     CSR -> its pass-1 position); a slice's entries of one column block are
//     contiguous in pass-1 order, so a wave's 448 reads touch ~2 lines per
//     column block instead of 384 random sectors.
// Every product is rounded once and the sum runs in PETSc's order, so y is
// bitwise the one-pass kernel's (checked here).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/colblock_probe.hip -o tools/colblock_probe
//   tools/colblock_probe [lg] [BS] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(2); } } while (0)
constexpr int K = 7;
typedef double d2v __attribute__((ext_vector_type(2)));
typedef int i2v __attribute__((ext_vector_type(2)));

template <class T> __device__ __forceinline__ T ldnt(const T *p) { return __builtin_nontemporal_load(p); }

// reference: one pass, SELL-64 [slice][j][lane]
__global__ void __launch_bounds__(256) spmv_onepass(int64_t nslices, const int *__restrict__ col,
                                                    const double *__restrict__ val, const double *__restrict__ x,
                                                    double *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  for (int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < nslices; s += (int64_t)gridDim.x * 4) {
    int c[K];
    double v[K], xv[K];
#pragma unroll
    for (int j = 0; j < K; ++j) { c[j] = ldnt(col + (s * K + j) * 64 + lane); v[j] = ldnt(val + (s * K + j) * 64 + lane); }
#pragma unroll
    for (int j = 0; j < K; ++j) xv[j] = x[c[j]];
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) sum = sum + v[j] * xv[j];
    __builtin_nontemporal_store(sum, y + s * 64 + lane);
  }
}

// pass 1: block b of the grid runs on XCD b % 8 (round-robin dispatch);
// the XCD's nper workgroups split each of its column blocks' entry ranges.
// E entries per thread per step (E / 2 16-B value loads in flight)
template <int E>
__global__ void __launch_bounds__(256) pass1(int ncb, const int64_t *__restrict__ bstart, const int *__restrict__ c1,
                                             const double *__restrict__ v1, const double *__restrict__ x,
                                             double *__restrict__ prod) {
  const int xcd = blockIdx.x & 7, wi = blockIdx.x >> 3, nper = gridDim.x >> 3;
  for (int C = xcd; C < ncb; C += 8) {
    const int64_t b0 = bstart[C], b1 = bstart[C + 1], len = b1 - b0;
    const int64_t chunk = ((len + nper - 1) / nper + 1) & ~(int64_t)1;
    const int64_t lo = b0 + chunk * wi, hi = min(b1, lo + chunk);
    int64_t k = lo + 2 * threadIdx.x;
    for (; k + 2 * 256 * (E / 2 - 1) + 1 < hi; k += 512 * (E / 2)) {
      d2v v[E / 2];
      i2v c[E / 2];
#pragma unroll
      for (int e = 0; e < E / 2; ++e) {
        v[e] = ldnt(reinterpret_cast<const d2v *>(v1 + k + 512 * e));
        c[e] = ldnt(reinterpret_cast<const i2v *>(c1 + k + 512 * e));
      }
      double xa[E / 2], xb[E / 2];
#pragma unroll
      for (int e = 0; e < E / 2; ++e) { xa[e] = x[c[e].x]; xb[e] = x[c[e].y]; }
#pragma unroll
      for (int e = 0; e < E / 2; ++e) {
        d2v p;
        p.x = v[e].x * xa[e];
        p.y = v[e].y * xb[e];
        __builtin_nontemporal_store(p, reinterpret_cast<d2v *>(prod + k + 512 * e));
      }
    }
    for (; k < hi; k += 512) {
      prod[k] = ldnt(v1 + k) * x[ldnt(c1 + k)];
      if (k + 1 < hi) prod[k + 1] = ldnt(v1 + k + 1) * x[ldnt(c1 + k + 1)];
    }
  }
}

// pass 2: SELL-64 over perm
__global__ void __launch_bounds__(256) pass2(int64_t nslices, const int *__restrict__ perm,
                                             const double *__restrict__ prod, double *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  for (int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < nslices; s += (int64_t)gridDim.x * 4) {
    int p[K];
#pragma unroll
    for (int j = 0; j < K; ++j) p[j] = ldnt(perm + (s * K + j) * 64 + lane);
    double t[K];
#pragma unroll
    for (int j = 0; j < K; ++j) t[j] = prod[p[j]];
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) sum = sum + t[j];
    __builtin_nontemporal_store(sum, y + s * 64 + lane);
  }
}

template <class F> static double timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char **argv) {
  const int lg = argc > 1 ? std::atoi(argv[1]) : 24;
  const int BS = argc > 2 ? std::atoi(argv[2]) : 19;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 9;
  const int64_t N = (int64_t)1 << lg, ns = N / 64, nnz = N * K;
  const int ncb = (int)((N + ((int64_t)1 << BS) - 1) >> BS);
  // CSR (row-major, sorted columns): entry j = row * K + q
  std::vector<int> cc(nnz);
  std::vector<double> vv(nnz);
  std::mt19937_64 rng(11);
  for (int64_t r = 0; r < N; ++r) {
    int t[K];
    t[0] = (int)r;
    for (int q = 1; q < K; ++q) t[q] = (int)(rng() % (uint64_t)N);
    std::sort(t, t + K);
    for (int q = 0; q < K; ++q) { cc[r * K + q] = t[q]; vv[r * K + q] = -1.0 - (double)(rng() % 1000) / 997.0; }
  }
  // one-pass SELL
  std::vector<int> sc(nnz);
  std::vector<double> sv(nnz);
  for (int64_t s = 0; s < ns; ++s)
    for (int q = 0; q < K; ++q)
      for (int l = 0; l < 64; ++l) { sc[(s * K + q) * 64 + l] = cc[(s * 64 + l) * K + q]; sv[(s * K + q) * 64 + l] = vv[(s * 64 + l) * K + q]; }
  // pass-1 order: by (column block, row, column) -- a counting sort by block keeps row-major order within a block
  std::vector<int64_t> bstart(ncb + 1, 0);
  for (int64_t j = 0; j < nnz; ++j) bstart[(cc[j] >> BS) + 1]++;
  for (int C = 0; C < ncb; ++C) bstart[C + 1] += bstart[C];
  std::vector<int64_t> fill(bstart.begin(), bstart.end() - 1);
  std::vector<int> c1(nnz), perm_csr(nnz);
  std::vector<double> v1(nnz);
  for (int64_t j = 0; j < nnz; ++j) {
    const int64_t k = fill[cc[j] >> BS]++;
    c1[k] = cc[j]; v1[k] = vv[j]; perm_csr[j] = (int)k;
  }
  std::vector<int> perm(nnz);   // SELL layout of perm
  for (int64_t s = 0; s < ns; ++s)
    for (int q = 0; q < K; ++q)
      for (int l = 0; l < 64; ++l) perm[(s * K + q) * 64 + l] = perm_csr[(s * 64 + l) * K + q];
  int *d_sc, *d_c1, *d_perm;
  double *d_sv, *d_v1, *d_x, *d_y, *d_y2, *d_prod;
  int64_t *d_b;
  CK(hipMalloc(&d_sc, 4 * nnz)); CK(hipMalloc(&d_c1, 4 * nnz)); CK(hipMalloc(&d_perm, 4 * nnz));
  CK(hipMalloc(&d_sv, 8 * nnz)); CK(hipMalloc(&d_v1, 8 * nnz)); CK(hipMalloc(&d_prod, 8 * nnz));
  CK(hipMalloc(&d_x, 8 * N)); CK(hipMalloc(&d_y, 8 * N)); CK(hipMalloc(&d_y2, 8 * N));
  CK(hipMalloc(&d_b, 8 * (ncb + 1)));
  CK(hipMemcpy(d_sc, sc.data(), 4 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sv, sv.data(), 8 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_c1, c1.data(), 4 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_v1, v1.data(), 8 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_perm, perm.data(), 4 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_b, bstart.data(), 8 * (ncb + 1), hipMemcpyHostToDevice));
  std::vector<double> hx(N);
  std::mt19937_64 r2(5);
  for (auto &e : hx) e = (double)(r2() >> 11) * 0x1.0p-53 - 0.5;
  CK(hipMemcpy(d_x, hx.data(), 8 * N, hipMemcpyHostToDevice));
  const double sector = 12.0 * nnz + 8.0 * N + 64.0 * (K - 1) * N;
  std::printf("N = 2^%d x %d, column blocks of 2^%d doubles (%d blocks), sector model %.2f GB\n", lg, K, BS, ncb, sector / 1e9);
  const double t1 = timeit([&] { spmv_onepass<<<8192, 256>>>(ns, d_sc, d_sv, d_x, d_y); }, reps);
  std::printf("one pass                 %8.1f us  sector frac %.3f\n", t1 * 1e3, sector / t1 / 1e6 / 8000);
  const double t2 = timeit([&] { pass2<<<8192, 256>>>(ns, d_perm, d_prod, d_y2); }, reps);
  std::printf("pass2 alone              %8.1f us  (%.0f GB/s on perm + y)\n", t2 * 1e3, (4.0 * nnz + 8.0 * N) / t2 / 1e6);
  for (int g : {512, 768, 1024, 1536}) {
    const double a2 = timeit([&] { pass1<2><<<g, 256>>>(ncb, d_b, d_c1, d_v1, d_x, d_prod); }, reps);
    const double a4 = timeit([&] { pass1<4><<<g, 256>>>(ncb, d_b, d_c1, d_v1, d_x, d_prod); }, reps);
    const double a8 = timeit([&] { pass1<8><<<g, 256>>>(ncb, d_b, d_c1, d_v1, d_x, d_prod); }, reps);
    const double ab = timeit([&] { pass1<4><<<g, 256>>>(ncb, d_b, d_c1, d_v1, d_x, d_prod); pass2<<<8192, 256>>>(ns, d_perm, d_prod, d_y2); }, reps);
    std::printf("grid %5d: pass1 E=2 %7.1f  E=4 %7.1f  E=8 %7.1f us (E=4: %.0f GB/s on 20 B/nnz)  E=4 + pass2 %7.1f us  sector frac %.3f\n",
                g, a2 * 1e3, a4 * 1e3, a8 * 1e3, 20.0 * nnz / a4 / 1e6, ab * 1e3, sector / ab / 1e6 / 8000);
  }
  std::vector<double> y1(N), y2(N);
  CK(hipMemcpy(y1.data(), d_y, 8 * N, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y2.data(), d_y2, 8 * N, hipMemcpyDeviceToHost));
  std::printf("bitwise equal: %s\n", std::memcmp(y1.data(), y2.data(), 8 * N) == 0 ? "yes" : "NO");
  return 0;
}
