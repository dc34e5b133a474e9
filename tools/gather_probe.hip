// gather_probe.hip -- what bounds the random-pattern SpMV (y = A x, N rows, K
// entries per row, one diagonal + K-1 uniformly random columns; SELL-64 with
// entry j of a slice's 64 rows at [slice][j][lane]).  Variants (template
// flags): nt loads for the matrix streams and y stores (NTM), nt loads for the
// x gathers (NTX), slices per wave in flight (U = 1 or 2), and two ceilings:
// the same kernel gathering x[row] (sequential: the streams alone) and the
// gathers alone (values not read).  Device time per launch from HIP events,
// median of `reps`; bytes on the streamed model (12 B per slot + 16 B per
// row) and the sector model (+ 64 B per off-diagonal gather).
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/gather_probe
//   tools/gather_probe [log2 N] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(2); } } while (0)
constexpr int K = 7;

template <bool NT, class T> __device__ __forceinline__ T ld(const T *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// MODE 0: SpMV; 1: gather x[row] instead (streams only); 2: gathers only (v = 1)
template <bool NTM, bool NTX, int U, int MODE>
__global__ void __launch_bounds__(256) spmv_probe(int64_t nslices, const int *__restrict__ col,
                                                  const double *__restrict__ val, const double *__restrict__ x,
                                                  double *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  for (int64_t s0 = w0 * U; s0 < nslices; s0 += nw * U) {
    int c[U][K];
    double v[U][K], xv[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t s = s0 + u < nslices ? s0 + u : s0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        c[u][j] = MODE == 1 ? (int)(s * 64 + lane) : ld<NTM>(col + (s * K + j) * 64 + lane);
        v[u][j] = MODE == 2 ? 1.0 : ld<NTM>(val + (s * K + j) * 64 + lane);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < K; ++j) xv[u][j] = ld<NTX>(x + c[u][j]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double sum = 0.0;
#pragma unroll
      for (int j = 0; j < K; ++j) sum = sum + v[u][j] * xv[u][j];
      if (s0 + u < nslices) {
        if constexpr (NTM) __builtin_nontemporal_store(sum, y + (s0 + u) * 64 + lane);
        else y[(s0 + u) * 64 + lane] = sum;
      }
    }
  }
}

template <bool NTM, bool NTX, int U, int MODE>
static double run(const char *name, int64_t ns, const int *c, const double *v, const double *x, double *y, int grid,
                  int reps, double stream_b, double sector_b) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(a));
    spmv_probe<NTM, NTX, U, MODE><<<grid, 256>>>(ns, c, v, x, y);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double ms = t[t.size() / 2];
  std::printf("%-34s grid %6d  %8.1f us  streamed %6.0f GB/s (%.3f)  sector %6.0f GB/s (%.3f)\n", name, grid, ms * 1e3,
              stream_b / ms / 1e6, stream_b / ms / 1e6 / 8000, sector_b / ms / 1e6, sector_b / ms / 1e6 / 8000);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms;
}

int main(int argc, char **argv) {
  const int lg = argc > 1 ? std::atoi(argv[1]) : 24;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 9;
  const int64_t N = (int64_t)1 << lg, ns = N / 64;
  std::vector<int> hc((size_t)N * K);
  std::vector<double> hv((size_t)N * K);
  std::mt19937_64 rng(11);
  for (int64_t s = 0; s < ns; ++s)
    for (int l = 0; l < 64; ++l) {
      const int64_t row = s * 64 + l;
      int cc[K];
      cc[0] = (int)row;
      for (int j = 1; j < K; ++j) cc[j] = (int)(rng() % (uint64_t)N);
      std::sort(cc, cc + K);
      for (int j = 0; j < K; ++j) {
        hc[(s * K + j) * 64 + l] = cc[j];
        hv[(s * K + j) * 64 + l] = -1.0 - (double)(rng() % 1000) / 1000.0;
      }
    }
  int *c;
  double *v, *x, *y;
  CK(hipMalloc(&c, sizeof(int) * N * K));
  CK(hipMalloc(&v, sizeof(double) * N * K));
  CK(hipMalloc(&x, sizeof(double) * N));
  CK(hipMalloc(&y, sizeof(double) * N));
  CK(hipMemcpy(c, hc.data(), sizeof(int) * N * K, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), sizeof(double) * N * K, hipMemcpyHostToDevice));
  std::vector<double> hx(N, 1.0);
  CK(hipMemcpy(x, hx.data(), sizeof(double) * N, hipMemcpyHostToDevice));
  const double stream_b = 12.0 * K * N + 16.0 * N, sector_b = 12.0 * K * N + 8.0 * N + 64.0 * (K - 1) * N;
  std::printf("N = 2^%d rows x %d (x %.0f MB), streamed model %.2f GB, sector model %.2f GB\n", lg, K, 8.0 * N / 1e6,
              stream_b / 1e9, sector_b / 1e9);
  int dev;
  CK(hipGetDevice(&dev));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  for (int g : {cus * 4, cus * 8, 8192, 32768}) {
    run<false, false, 1, 0>("spmv plain", ns, c, v, x, y, g, reps, stream_b, sector_b);
    run<true, false, 1, 0>("spmv nt matrix", ns, c, v, x, y, g, reps, stream_b, sector_b);
    run<true, true, 1, 0>("spmv nt matrix + nt x", ns, c, v, x, y, g, reps, stream_b, sector_b);
    run<true, false, 2, 0>("spmv nt matrix, 2 slices/wave", ns, c, v, x, y, g, reps, stream_b, sector_b);
    run<false, false, 2, 0>("spmv plain, 2 slices/wave", ns, c, v, x, y, g, reps, stream_b, sector_b);
  }
  const int g = 8192;
  run<true, false, 1, 1>("ceiling: streams only (x[row])", ns, c, v, x, y, g, reps, stream_b, stream_b);
  run<false, false, 1, 1>("ceiling: streams only, plain", ns, c, v, x, y, g, reps, stream_b, stream_b);
  run<true, false, 1, 2>("ceiling: gathers only (+cols)", ns, c, v, x, y, g, reps, stream_b, sector_b);
  run<true, true, 1, 2>("ceiling: gathers only, nt x", ns, c, v, x, y, g, reps, stream_b, sector_b);
  return 0;
}
