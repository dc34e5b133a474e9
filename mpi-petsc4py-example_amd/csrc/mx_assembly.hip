// mx_assembly.hip -- device-side AIJ assembly (gfx950).
//
// Replaces what PETSc does behind PETSc.Mat().createAIJ(csr=...) + assemble()
// (petsc_funcs.py:6-7, test.py:24-28): MatMPIAIJSetPreallocationCSR ->
// MatSetValues(INSERT) row by row -> MatAssemblyEnd -> MatSetUpMultiply_MPIAIJ
// (SURVEY.md §2 N1-N3).  Semantics restated in oracle/petsc_oracle.c
// (canon_row, build_block):
//   * per row, columns end up sorted; negative columns are ignored;
//   * a repeated column keeps the LAST value (INSERT) or the values added in
//     input order (ADD: first stored, later ones added);
//   * explicit zeros are kept; column >= N is an out-of-range error;
//   * the row block splits into A_d (columns owned by this rank, stored as
//     local column ids) and A_o (other columns, renumbered into [0, nghost) in
//     ascending global order = garray).
//
// Device pipeline (all on the communicator's stream):
//   [COO: row histogram -> scan -> scatter with the input position kept]
//   canonicalise rows: W-lane segments (W = 8..64) bitonic-sort (col, pos)
//     pairs in registers with xor shuffles, then a segmented last-wins /
//     ordered-fold dedupe with ballot compaction; rows longer than 64 go to a
//     block-per-row LDS bitonic sort (<= 2048 entries), longer ones to a
//     global chunk-sort + merge-pass sort (canon_huge_rows);
//   split + ghost bitmap (atomicOr) -> scans -> bitmap popcount-scan gives
//     garray and the A_o renumbering without any sort;
//   SELL-64 copies of A_d and A_o for the SpMV;
//   halo plan: garray owners from the column layout, one count all-to-all,
//     requested indices sent to their owners, contiguous send ranges detected.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <unordered_map>

#include "mx_internal.hpp"

namespace mx {

constexpr int64_t KEY_DROP = LLONG_MAX;
constexpr int LONG_ROW_MAX = 2048;

// ---------------------------------------------------------------- helpers
__global__ void cvt_i32_i64_kernel(const int32_t *__restrict__ s, int64_t n, int64_t *__restrict__ d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
}

void convert_index(const void *src, int bytes, int64_t n, int64_t *dst, hipStream_t s) {
  if (n <= 0) return;
  if (bytes == 8) {
    HIPCHECK(hipMemcpyAsync(dst, src, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, s));
  } else if (bytes == 4) {
    cvt_i32_i64_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>(static_cast<const int32_t *>(src), n, dst);
    HIPCHECK(hipGetLastError());
  } else {
    fail(MX_ERR_ARG, "index width must be 4 or 8 bytes");
  }
}

// grid-stride (a capped grid): one atomicMax per workgroup -- a workgroup per
// 256 rows put 65,536 atomics on one word (0.75 ms for 2^24 rows)
__global__ void row_len_max_kernel(int64_t m, const int64_t *__restrict__ rowptr,
                                   unsigned long long *__restrict__ out, int *__restrict__ err) {
  unsigned long long mx = 0;
  bool bad = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const int64_t len = rowptr[i + 1] - rowptr[i];
    if (len < 0) bad = true;
    else mx = (unsigned long long)len > mx ? (unsigned long long)len : mx;
  }
  if (bad) atomicOr(err, 4);
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(mx, o, 64);
    mx = t > mx ? t : mx;
  }
  __shared__ unsigned long long sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = sh[0];
    for (int k = 1; k < 4; ++k) mx = sh[k] > mx ? sh[k] : mx;
    if (mx) atomicMax(out, mx);   // one atomic per block
  }
}

// ---------------------------------------------------------------- COO bucketing
__global__ void coo_count_kernel(int64_t n, const int64_t *__restrict__ rows,
                                 const int64_t *__restrict__ cols, int64_t rstart, int64_t m,
                                 unsigned long long *__restrict__ cnt, int *__restrict__ err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    int64_t r = rows[k];
    if (r < 0 || cols[k] < 0) continue;                 // MatSetValues ignores negative indices
    if (r < rstart || r >= rstart + m) { atomicOr(err, 8); continue; }
    atomicAdd(&cnt[r - rstart], 1ULL);
  }
}

__global__ void coo_scatter_kernel(int64_t n, const int64_t *__restrict__ rows,
                                   const int64_t *__restrict__ cols, const double *__restrict__ vals,
                                   int64_t rstart, int64_t m, const int64_t *__restrict__ rowptr,
                                   unsigned long long *__restrict__ cursor, int64_t *__restrict__ gcol,
                                   double *__restrict__ gval, int64_t *__restrict__ gpos) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    int64_t r = rows[k];
    if (r < 0 || cols[k] < 0 || r < rstart || r >= rstart + m) continue;
    int64_t i = r - rstart;
    int64_t slot = rowptr[i] + (int64_t)atomicAdd(&cursor[i], 1ULL);
    gcol[slot] = cols[k]; gval[slot] = vals[k]; gpos[slot] = k;   // k restores input order
  }
}

// ---------------------------------------------------------------- off-process stash
// MatSetValues on rows owned elsewhere go to PETSc's stash and are applied by
// their owner at MatAssemblyEnd.  Here every COO entry is tagged with the
// owner of its row, entries are stably partitioned by owner, one count
// all-to-all and one grouped send/recv move them, and the owner appends the
// received entries after its own (local first, then by source rank: a
// deterministic version of PETSc's arrival order).
struct CooEntry { int64_t row, col; double val; };

__global__ void coo_owner_kernel(int64_t n, const int64_t *__restrict__ rows, const int64_t *__restrict__ cols,
                                 const int64_t *__restrict__ ranges, int P, int64_t M, int *__restrict__ owner,
                                 unsigned long long *__restrict__ cnt, int *__restrict__ err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const int64_t r = rows[k];
    int o = -1;
    if (r >= 0 && cols[k] >= 0) {
      if (r >= M) { atomicOr(err, 16); }
      else {
        int lo = 0, hi = P - 1;
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (ranges[mid] <= r) lo = mid; else hi = mid - 1; }
        o = lo;
        atomicAdd(&cnt[o], 1ULL);
      }
    }
    owner[k] = o;
  }
}

__global__ void coo_flag_kernel(int64_t n, const int *__restrict__ owner, int q, int64_t *__restrict__ flag) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) flag[k] = owner[k] == q;
}

__global__ void coo_pack_kernel(int64_t n, const int *__restrict__ owner, int q, const int64_t *__restrict__ pos,
                                const int64_t *__restrict__ rows, const int64_t *__restrict__ cols,
                                const double *__restrict__ vals, CooEntry *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
    if (owner[k] == q) out[pos[k]] = CooEntry{rows[k], cols[k], vals[k]};
}

__global__ void coo_unpack_kernel(int64_t n, const CooEntry *__restrict__ in, int64_t *__restrict__ rows,
                                  int64_t *__restrict__ cols, double *__restrict__ vals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const CooEntry e = in[k];
    rows[k] = e.row; cols[k] = e.col; vals[k] = e.val;
  }
}

// Returns the number of entries now held by this rank (all rows local).
static int64_t coo_redistribute(Comm *c, const std::vector<int64_t> &rr, int64_t M, const int64_t *rows,
                                const int64_t *cols, const double *vals, int64_t n, DBuf<int64_t> &orows,
                                DBuf<int64_t> &ocols, DBuf<double> &ovals) {
  const int P = c->size;
  hipStream_t st = c->stream;
  DBuf<int64_t> ranges((size_t)P + 1);
  HIPCHECK(hipMemcpyAsync(ranges.p, rr.data(), sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, st));
  DBuf<int> owner((size_t)std::max<int64_t>(n, 1), kScratch), err(1);
  DBuf<unsigned long long> cnt((size_t)P);
  HIPCHECK(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long) * P, st));
  HIPCHECK(hipMemsetAsync(err.p, 0, sizeof(int), st));
  if (n) {
    coo_owner_kernel<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, rows, cols, ranges.p, P, M, owner.p, cnt.p, err.p);
    HIPCHECK(hipGetLastError());
  }
  std::vector<unsigned long long> cs(P);
  int herr = 0;
  HIPCHECK(hipMemcpyAsync(cs.data(), cnt.p, sizeof(unsigned long long) * P, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  int gerr = 0;
  {
    std::vector<int64_t> all(P);
    c->allgather_i64(herr, all.data());
    for (int64_t e : all) gerr |= (int)e;
  }
  if (gerr & 16) fail(MX_ERR_OUTOFRANGE, "Row too large: max " + std::to_string(M - 1));
  std::vector<int64_t> send(P), recv(P);
  for (int q = 0; q < P; ++q) send[q] = (int64_t)cs[q];
  c->alltoall_i64(send.data(), recv.data());
  // stable partition by owner into one buffer, owner segments in rank order
  std::vector<int64_t> soff(P + 1, 0);
  for (int q = 0; q < P; ++q) soff[q + 1] = soff[q] + send[q];
  DBuf<CooEntry> sbuf((size_t)std::max<int64_t>(soff[P], 1));
  DBuf<int64_t> pos((size_t)std::max<int64_t>(n, 1), kScratch);
  for (int q = 0; q < P; ++q) {
    if (!send[q]) continue;
    coo_flag_kernel<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, owner.p, q, pos.p);
    exclusive_scan_i64(pos.p, pos.p, n, st, nullptr);
    coo_pack_kernel<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, owner.p, q, pos.p, rows, cols, vals, sbuf.p + soff[q]);
    HIPCHECK(hipGetLastError());
  }
  // received entries: own segment first, then the other ranks in order
  int64_t total = send[c->rank];
  std::vector<int64_t> roff(P, 0);
  for (int q = 0; q < P; ++q) {
    if (q == c->rank) continue;
    roff[q] = total;
    total += recv[q];
  }
  DBuf<CooEntry> rbuf((size_t)std::max<int64_t>(total, 1));
  if (send[c->rank])
    HIPCHECK(hipMemcpyAsync(rbuf.p, sbuf.p + soff[c->rank], sizeof(CooEntry) * send[c->rank], hipMemcpyDeviceToDevice, st));
  std::vector<Msg> sends, recvs;
  for (int q = 0; q < P; ++q) {
    if (q == c->rank) continue;
    if (send[q]) sends.push_back({q, sbuf.p + soff[q], sizeof(CooEntry) * (size_t)send[q]});
    if (recv[q]) recvs.push_back({q, rbuf.p + roff[q], sizeof(CooEntry) * (size_t)recv[q]});
  }
  c->exchange(sends, recvs);
  orows.alloc((size_t)std::max<int64_t>(total, 1));
  ocols.alloc((size_t)std::max<int64_t>(total, 1));
  ovals.alloc((size_t)std::max<int64_t>(total, 1));
  if (total) {
    coo_unpack_kernel<<<grid_for(total, 256, 8192), 256, 0, st>>>(total, rbuf.p, orows.p, ocols.p, ovals.p);
    HIPCHECK(hipGetLastError());
  }
  HIPCHECK(hipStreamSynchronize(st));
  return total;
}

// ---------------------------------------------------------------- row canonicalisation
// One W-lane segment per row (W | 64).  Keys (col, pos) are unique per row
// except the dropped/padding lanes, which all carry (KEY_DROP, KEY_DROP).
// canon_seg: the row's entries (lane l: entry l) sorted and deduplicated in
// registers; returns keep (this lane holds a canonical entry: column c and,
// with VALS, its value -- INSERT: the last of its run, ADD: the run folded in
// input order).  The kept lanes are in ascending column order.
// canon_load: lane l's input entry (column, input position, value), or the
// drop key; canon_sorted: canon_seg on loaded entries (the fused count / fill
// passes load several rows' entries first, then sort each).
template <bool VALS, typename CT = int64_t>
__device__ __forceinline__ void canon_load(int l, bool active, int64_t start, int64_t len,
                                           const CT *__restrict__ col, const double *__restrict__ val,
                                           const int64_t *__restrict__ pos, int64_t N, int *__restrict__ err,
                                           int64_t &c, int64_t &p, double &v) {
  p = KEY_DROP;
  v = 0.0;
  c = KEY_DROP;
  if (active && l < len) {
    const int64_t cc = (int64_t)col[start + l];   // int32 columns sign-extend: -1 stays a drop
    if (cc >= 0) {
      if (err && cc >= N) atomicOr(err, 1);
      c = cc;
      p = pos ? pos[start + l] : (int64_t)l;
      if (VALS) v = val[start + l];
    }
  }
}

template <int W, bool VALS>
__device__ __forceinline__ bool canon_sorted(int lane, int l, int add, int64_t &c, int64_t p, double v, double &out);

template <int W, bool VALS>
__device__ __forceinline__ bool canon_seg(int lane, int l, bool active, int64_t start, int64_t len,
                                          const int64_t *__restrict__ col, const double *__restrict__ val,
                                          const int64_t *__restrict__ pos, int64_t N, int add, int *__restrict__ err,
                                          int64_t &c, double &out) {
  int64_t p;
  double v;
  canon_load<VALS>(l, active, start, len, col, val, pos, N, err, c, p, v);
  return canon_sorted<W, VALS>(lane, l, add, c, p, v, out);
}

template <int W, bool VALS>
__device__ __forceinline__ bool canon_sorted(int lane, int l, int add, int64_t &c, int64_t p, double v, double &out) {
  // Already canonical (every kept column above the previous kept column of
  // its row, in input order -- scipy's canonical CSR, the stencil generator):
  // the sort would only move the dropped lanes to the end, which the ballot
  // compaction of the callers does anyway, and there is nothing to dedupe.
  // Decided per wave, so most waves of such inputs skip the bitonic network.
  const int gbase0 = lane - l;
  const unsigned long long vb = __ballot(c != KEY_DROP);
  const unsigned long long below_v = vb & ((l == 0) ? 0ULL : (((1ULL << l) - 1ULL) << gbase0));
  const int pl = below_v ? 63 - __clzll(below_v) : lane;
  const int64_t cprev = __shfl(c, pl, 64);
  const bool sorted = !__any(c != KEY_DROP && below_v != 0 && cprev >= c);
  // bitonic sort of (c, p) ascending inside each W-lane segment
  if (!sorted) {
#pragma unroll
    for (int k = 2; k <= W; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        int64_t c2 = __shfl_xor(c, j, 64);
        int64_t p2 = __shfl_xor(p, j, 64);
        double v2 = VALS ? __shfl_xor(v, j, 64) : 0.0;
        const bool up = (l & k) == 0;
        const bool lower = (l & j) == 0;
        const bool mine_less = (c < c2) || (c == c2 && p < p2);
        const bool keep = (lower == up) ? mine_less : !mine_less;
        if (!keep) { c = c2; p = p2; if (VALS) v = v2; }
      }
    }
  }
  const bool valid = c != KEY_DROP;
  const int64_t c_next = __shfl(c, (lane + 1) & 63, 64);
  const int64_t c_prev = __shfl(c, (lane + 63) & 63, 64);
  bool keep;
  out = v;
  if (!add) {
    keep = valid && (l == W - 1 || c_next != c);       // INSERT: last occurrence wins
  } else {
    keep = valid && (l == 0 || c_prev != c);           // ADD: run head folds its run in order
    if (VALS) {
      bool run = true;
#pragma unroll
      for (int t = 1; t < W; ++t) {
        const double vt = __shfl(v, (lane + t) & 63, 64);
        const int64_t ct = __shfl(c, (lane + t) & 63, 64);
        run = run && (l + t < W) && (ct == c);
        if (run) out = out + vt;
      }
    }
  }
  return keep;
}

template <int W>
__global__ void __launch_bounds__(256) canon_rows_wave_kernel(
    int64_t m, const int64_t *__restrict__ rowptr, const int64_t *__restrict__ col,
    const double *__restrict__ val, const int64_t *__restrict__ pos, int64_t N, int add,
    int64_t *__restrict__ ccol, double *__restrict__ cval, int64_t *__restrict__ cnt_out,
    int64_t *__restrict__ long_rows, unsigned long long *__restrict__ nlong, int *__restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int l = lane % W;
  const int64_t row = (int64_t)blockIdx.x * (256 / W) + threadIdx.x / W;
  const bool rvalid = row < m;
  const int64_t start = rvalid ? rowptr[row] : 0;
  const int64_t len = rvalid ? rowptr[row + 1] - start : 0;
  const bool too_long = len > W;
  if (rvalid && too_long && l == 0) long_rows[atomicAdd(nlong, 1ULL)] = row;
  const bool active = rvalid && !too_long;
  int64_t c;
  double out;
  const bool keep = canon_seg<W, true>(lane, l, active, start, len, col, val, pos, N, add, err, c, out);
  const unsigned long long ball = __ballot(keep);
  const int gbase = lane - l;
  const unsigned long long gmask =
      (W == 64) ? ball : ((ball >> gbase) & ((1ULL << (W == 64 ? 0 : W)) - 1ULL));
  const int idx = __popcll(gmask & ((l == 0) ? 0ULL : ((1ULL << l) - 1ULL)));
  if (active) {
    if (keep) { ccol[start + idx] = c; cval[start + idx] = out; }
    if (l == 0) cnt_out[row] = __popcll(gmask);
  }
}

// Canonicalisation fused with the MPIAIJ split, for inputs whose rows are all
// at most 64 entries (every configuration; longer rows take the separate
// passes above and below): a count pass sorts / deduplicates each row in
// registers and writes its A_d / A_o counts (and the ghost bitmap) straight
// into the split's row pointers, then -- after the scans -- a fill pass
// repeats the same register canonicalisation with the values and stores the
// split arrays.  No canonical copy of the input goes through HBM (round 4:
// canonicalise 14.4 GB + split count 3.6 + split fill 12.6 for a 27-point
// share; fused: 3.6 + 12.6).
constexpr int CANON_R = 4, CANON_FR = 1;

template <int W>
__device__ __forceinline__ unsigned long long seg_bits_w(unsigned long long ball, int gbase) {
  return W == 64 ? ball : ((ball >> gbase) & ((1ULL << (W == 64 ? 0 : W)) - 1ULL));
}

template <int W, typename CT>
__global__ void __launch_bounds__(256) canon_count_kernel(int64_t m, const int64_t *__restrict__ rowptr,
                                                          const CT *__restrict__ col,
                                                          const int64_t *__restrict__ pos, int64_t N, int add,
                                                          int64_t cstart, int64_t cend, int64_t *__restrict__ cnt_d,
                                                          int64_t *__restrict__ cnt_o, unsigned *__restrict__ bitmap,
                                                          int *__restrict__ err) {
  // CANON_R rows per W-lane segment, every row's loads issued before the
  // first row is sorted (one row per segment left each wave waiting on two
  // dependent loads at a time: 2.35 ms for a 27-point share, round 5)
  const int lane = threadIdx.x & 63, l = lane % W, gbase = lane - l;
  const int64_t row0 = (int64_t)blockIdx.x * (256 / W) * CANON_R + threadIdx.x / W;
  int64_t start[CANON_R], len[CANON_R], c[CANON_R], p[CANON_R];
  double v[CANON_R];
#pragma unroll
  for (int r = 0; r < CANON_R; ++r) {
    const int64_t row = row0 + (int64_t)r * (256 / W);
    start[r] = row < m ? rowptr[row] : 0;
    len[r] = row < m ? rowptr[row + 1] - start[r] : 0;
  }
#pragma unroll
  for (int r = 0; r < CANON_R; ++r)
    canon_load<false, CT>(l, row0 + (int64_t)r * (256 / W) < m, start[r], len[r], col, nullptr, pos, N, err, c[r], p[r], v[r]);
#pragma unroll
  for (int r = 0; r < CANON_R; ++r) {
    const int64_t row = row0 + (int64_t)r * (256 / W);
    double out;
    const bool keep = canon_sorted<W, false>(lane, l, add, c[r], p[r], v[r], out);
    const bool isd = keep && c[r] >= cstart && c[r] < cend, iso = keep && !isd;
    if (iso) atomicOr(&bitmap[c[r] >> 5], 1u << (c[r] & 31));
    const int nd = __popcll(seg_bits_w<W>(__ballot(isd), gbase)), no = __popcll(seg_bits_w<W>(__ballot(iso), gbase));
    if (row < m && l == 0) { cnt_d[row] = nd; cnt_o[row] = no; }
  }
}

// (one row per segment: four, as in the count pass, measured 5.65 ms against
// 4.4 for a 27-point share -- 99 VGPRs, half the waves)
template <int W, typename CT>
__global__ void __launch_bounds__(256) canon_fill_kernel(
    int64_t m, const int64_t *__restrict__ rowptr, const CT *__restrict__ col, const double *__restrict__ val,
    const int64_t *__restrict__ pos, int64_t N, int add, int64_t cstart, int64_t cend, int64_t rstart,
    const int64_t *__restrict__ dptr, const int64_t *__restrict__ optr, int32_t *__restrict__ dcol,
    double *__restrict__ dval, int32_t *__restrict__ ocol, double *__restrict__ oval, double *__restrict__ diag,
    const unsigned *__restrict__ bitmap, const int64_t *__restrict__ wbase) {
  const int lane = threadIdx.x & 63, l = lane % W, gbase = lane - l;
  const int64_t row0 = (int64_t)blockIdx.x * (256 / W) * CANON_FR + threadIdx.x / W;
  int64_t start[CANON_FR], len[CANON_FR], c[CANON_FR], p[CANON_FR], dp[CANON_FR], op[CANON_FR];
  double v[CANON_FR];
#pragma unroll
  for (int r = 0; r < CANON_FR; ++r) {   // the row's split offsets too: no load after the sort
    const int64_t row = row0 + (int64_t)r * (256 / W);
    start[r] = row < m ? rowptr[row] : 0;
    len[r] = row < m ? rowptr[row + 1] - start[r] : 0;
    dp[r] = row < m ? dptr[row] : 0;
    op[r] = row < m ? optr[row] : 0;
  }
#pragma unroll
  for (int r = 0; r < CANON_FR; ++r)
    canon_load<true, CT>(l, row0 + (int64_t)r * (256 / W) < m, start[r], len[r], col, val, pos, N, nullptr, c[r], p[r], v[r]);
#pragma unroll
  for (int r = 0; r < CANON_FR; ++r) {
    const int64_t row = row0 + (int64_t)r * (256 / W);
    const bool rv = row < m;
    double out;
    const bool keep = canon_sorted<W, true>(lane, l, add, c[r], p[r], v[r], out);
    const int64_t cr = c[r];
    const bool isd = keep && cr >= cstart && cr < cend, iso = keep && !isd;
    const unsigned long long below = l == 0 ? 0ULL : ((1ULL << l) - 1ULL);
    const unsigned long long bd = seg_bits_w<W>(__ballot(isd), gbase), bo = seg_bits_w<W>(__ballot(iso), gbase);
    const unsigned long long bg = seg_bits_w<W>(__ballot(isd && cr == rstart + row), gbase);
    if (isd) {
      const int64_t t = dp[r] + __popcll(bd & below);
      dcol[t] = (int32_t)(cr - cstart);
      dval[t] = out;
      if (cr == rstart + row) diag[row] = out;
    } else if (iso) {
      const int64_t w = cr >> 5;
      const unsigned bit = (unsigned)(cr & 31);
      const int64_t t = op[r] + __popcll(bo & below);
      ocol[t] = (int32_t)(wbase[w] + __popc(bitmap[w] & ((1u << bit) - 1u)));
      oval[t] = out;
    }
    if (rv && l == 0 && !bg) diag[row] = 0.0;
  }
}

// Rows longer than 64 entries: one block per row, LDS bitonic sort, then a
// sequential (exactly ordered) dedupe by one thread.
__global__ void __launch_bounds__(256) canon_rows_block_kernel(
    const int64_t *__restrict__ rows_list, const int64_t *__restrict__ rowptr,
    const int64_t *__restrict__ col, const double *__restrict__ val,
    const int64_t *__restrict__ pos, int64_t N, int add, int64_t *__restrict__ ccol,
    double *__restrict__ cval, int64_t *__restrict__ cnt_out, int *__restrict__ err,
    int64_t *__restrict__ huge_rows, unsigned long long *__restrict__ nhuge) {
  __shared__ int64_t kc[LONG_ROW_MAX];
  __shared__ int64_t kp[LONG_ROW_MAX];
  __shared__ double kv[LONG_ROW_MAX];
  const int64_t row = rows_list[blockIdx.x];
  const int64_t start = rowptr[row];
  const int64_t len = rowptr[row + 1] - start;
  if (len > LONG_ROW_MAX) {                 // canon_huge_row below
    if (threadIdx.x == 0) huge_rows[atomicAdd(nhuge, 1ULL)] = row;
    return;
  }
  int npad = 1;
  while (npad < len) npad <<= 1;
  for (int i = threadIdx.x; i < npad; i += 256) {
    int64_t c = KEY_DROP, p = KEY_DROP;
    double v = 0.0;
    if (i < len) {
      int64_t cc = col[start + i];
      if (cc >= 0) {
        if (cc >= N) atomicOr(err, 1);
        c = cc; p = pos ? pos[start + i] : (int64_t)i; v = val[start + i];
      }
    }
    kc[i] = c; kp[i] = p; kv[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= npad; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npad; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const bool greater = (kc[i] > kc[ixj]) || (kc[i] == kc[ixj] && kp[i] > kp[ixj]);
          if (greater == up) {
            int64_t tc = kc[i]; kc[i] = kc[ixj]; kc[ixj] = tc;
            int64_t tp = kp[i]; kp[i] = kp[ixj]; kp[ixj] = tp;
            double tv = kv[i]; kv[i] = kv[ixj]; kv[ixj] = tv;
          }
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    int64_t k = 0;
    for (int64_t i = 0; i < len && kc[i] != KEY_DROP; ++i) {
      if (k > 0 && ccol[start + k - 1] == kc[i]) {
        if (add) cval[start + k - 1] = cval[start + k - 1] + kv[i];
        else cval[start + k - 1] = kv[i];
      } else {
        ccol[start + k] = kc[i]; cval[start + k] = kv[i]; ++k;
      }
    }
    cnt_out[row] = k;
  }
}

// Rows longer than LONG_ROW_MAX: sorted in global scratch by the whole GPU --
// LDS bitonic sorts of 2048-entry chunks, then merge passes that double the
// run length (each entry finds its output slot by a binary search in the
// partner run; ties go to the left run, so the merge is stable), then the
// same sequential ordered dedupe.  (col, pos) keys are unique apart from the
// dropped entries, which all sort last.
struct SortKey { int64_t c, p; double v; };
__device__ __forceinline__ bool key_less(const SortKey &a, const SortKey &b) {
  return a.c < b.c || (a.c == b.c && a.p < b.p);
}

__global__ void __launch_bounds__(256) huge_chunk_sort_kernel(
    int64_t start, int64_t len, const int64_t *__restrict__ col, const double *__restrict__ val,
    const int64_t *__restrict__ pos, int64_t N, SortKey *__restrict__ out, int *__restrict__ err) {
  __shared__ int64_t kc[LONG_ROW_MAX];
  __shared__ int64_t kp[LONG_ROW_MAX];
  __shared__ double kv[LONG_ROW_MAX];
  const int64_t c0 = (int64_t)blockIdx.x * LONG_ROW_MAX;
  const int cl = (int)min((int64_t)LONG_ROW_MAX, len - c0);
  int npad = 1;
  while (npad < cl) npad <<= 1;
  for (int i = threadIdx.x; i < npad; i += 256) {
    int64_t c = KEY_DROP, p = KEY_DROP;
    double v = 0.0;
    if (i < cl) {
      const int64_t cc = col[start + c0 + i];
      if (cc >= 0) {
        if (cc >= N) atomicOr(err, 1);
        c = cc; p = pos ? pos[start + c0 + i] : c0 + i; v = val[start + c0 + i];
      }
    }
    kc[i] = c; kp[i] = p; kv[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= npad; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npad; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const bool greater = (kc[i] > kc[ixj]) || (kc[i] == kc[ixj] && kp[i] > kp[ixj]);
          if (greater == up) {
            int64_t tc = kc[i]; kc[i] = kc[ixj]; kc[ixj] = tc;
            int64_t tp = kp[i]; kp[i] = kp[ixj]; kp[ixj] = tp;
            double tv = kv[i]; kv[i] = kv[ixj]; kv[ixj] = tv;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < cl; i += 256) out[c0 + i] = SortKey{kc[i], kp[i], kv[i]};
}

__global__ void huge_merge_kernel(int64_t len, int64_t run, const SortKey *__restrict__ in,
                                  SortKey *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += stride) {
    const int64_t r = i / run, lo = (r >> 1) * 2 * run;
    const int64_t mid = min(lo + run, len), hi = min(lo + 2 * run, len);
    const SortKey k = in[i];
    int64_t a, b, rank = 0;
    if ((r & 1) == 0) {           // left run: count partner entries < k
      a = mid; b = hi;
      while (a < b) { const int64_t h = (a + b) >> 1; if (key_less(in[h], k)) a = h + 1; else b = h; }
      rank = a - mid;
      out[lo + (i - lo) + rank] = k;
    } else {                      // right run: count partner entries <= k
      a = lo; b = mid;
      while (a < b) { const int64_t h = (a + b) >> 1; if (!key_less(k, in[h])) a = h + 1; else b = h; }
      rank = a - lo;
      out[lo + (i - mid) + rank] = k;
    }
  }
}

__global__ void huge_dedupe_kernel(int64_t row, int64_t start, int64_t len, int add,
                                   const SortKey *__restrict__ in, int64_t *__restrict__ ccol,
                                   double *__restrict__ cval, int64_t *__restrict__ cnt_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t k = 0;
  for (int64_t i = 0; i < len && in[i].c != KEY_DROP; ++i) {
    if (k > 0 && ccol[start + k - 1] == in[i].c) {
      if (add) cval[start + k - 1] = cval[start + k - 1] + in[i].v;
      else cval[start + k - 1] = in[i].v;
    } else {
      ccol[start + k] = in[i].c; cval[start + k] = in[i].v; ++k;
    }
  }
  cnt_out[row] = k;
}

static void canon_huge_rows(const std::vector<int64_t> &rows, const int64_t *rowptr, const int64_t *col,
                            const double *val, const int64_t *pos, int64_t N, int add, int64_t *ccol,
                            double *cval, int64_t *cnt_out, int *err, hipStream_t st) {
  for (int64_t row : rows) {
    int64_t se[2];
    HIPCHECK(hipMemcpy(se, rowptr + row, sizeof(se), hipMemcpyDeviceToHost));
    const int64_t start = se[0], len = se[1] - se[0];
    DBuf<SortKey> a((size_t)len), b((size_t)len);
    huge_chunk_sort_kernel<<<(unsigned)cdiv(len, LONG_ROW_MAX), 256, 0, st>>>(start, len, col, val, pos, N, a.p, err);
    HIPCHECK(hipGetLastError());
    for (int64_t run = LONG_ROW_MAX; run < len; run *= 2) {
      huge_merge_kernel<<<grid_for(len, 256, 8192), 256, 0, st>>>(len, run, a.p, b.p);
      HIPCHECK(hipGetLastError());
      std::swap(a, b);
    }
    huge_dedupe_kernel<<<1, 64, 0, st>>>(row, start, len, add, a.p, ccol, cval, cnt_out);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(st));
  }
}

// ---------------------------------------------------------------- split
// W-lane segment per row (the canonicalisation's width): lane l reads entry
// base + l of its row, chunks of W entries, so a wave's loads are contiguous
// runs of the canonical arrays instead of 64 row walks ~W entries apart (the
// thread-per-row kernels they replace took 33 ms of a 27-point share's
// 100 ms assembly, round 5).  A row's diagonal / ghost
// entries keep their order: each lane's destination is its segment's running
// count plus the ballot prefix below it.
template <int W>
__device__ __forceinline__ unsigned long long seg_bits(unsigned long long ball, int gbase) {
  return W == 64 ? ball : ((ball >> gbase) & ((1ULL << (W == 64 ? 0 : W)) - 1ULL));
}

template <int W>
__global__ void __launch_bounds__(256) split_count_seg_kernel(int64_t m, const int64_t *__restrict__ rowptr,
                                                              const int64_t *__restrict__ cnt,
                                                              const int64_t *__restrict__ ccol, int64_t cstart,
                                                              int64_t cend, int64_t *__restrict__ cnt_d,
                                                              int64_t *__restrict__ cnt_o, unsigned *__restrict__ bitmap) {
  const int lane = threadIdx.x & 63, l = lane % W, gbase = lane - l;
  const int64_t row = (int64_t)blockIdx.x * (256 / W) + threadIdx.x / W;
  const bool rv = row < m;
  const int64_t s = rv ? rowptr[row] : 0, n = rv ? cnt[row] : 0;
  int64_t d = 0;
  int64_t nmax = n;   // wave-uniform trip count
  for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, (int64_t)__shfl_xor(nmax, o, 64));
  for (int64_t b = 0; b < nmax; b += W) {
    const bool in = b + l < n;
    const int64_t c = in ? ccol[s + b + l] : 0;
    const bool isd = in && c >= cstart && c < cend;
    if (in && !isd) atomicOr(&bitmap[c >> 5], 1u << (c & 31));
    d += __popcll(seg_bits<W>(__ballot(isd), gbase));
  }
  if (rv && l == 0) { cnt_d[row] = d; cnt_o[row] = n - d; }
}

template <int W>
__global__ void __launch_bounds__(256) fill_split_seg_kernel(
    int64_t m, const int64_t *__restrict__ rowptr, const int64_t *__restrict__ cnt, const int64_t *__restrict__ ccol,
    const double *__restrict__ cval, int64_t cstart, int64_t cend, int64_t rstart, const int64_t *__restrict__ dptr,
    const int64_t *__restrict__ optr, int32_t *__restrict__ dcol, double *__restrict__ dval, int32_t *__restrict__ ocol,
    double *__restrict__ oval, double *__restrict__ diag, const unsigned *__restrict__ bitmap,
    const int64_t *__restrict__ wbase) {
  const int lane = threadIdx.x & 63, l = lane % W, gbase = lane - l;
  const int64_t row = (int64_t)blockIdx.x * (256 / W) + threadIdx.x / W;
  const bool rv = row < m;
  const int64_t s = rv ? rowptr[row] : 0, n = rv ? cnt[row] : 0;
  int64_t pd = rv ? dptr[row] : 0, po = rv ? optr[row] : 0;
  const int64_t grow = rstart + row;
  const unsigned long long below = l == 0 ? 0ULL : ((1ULL << l) - 1ULL);
  int64_t nmax = n;
  for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, (int64_t)__shfl_xor(nmax, o, 64));
  bool have_diag = false;
  for (int64_t b = 0; b < nmax; b += W) {
    const bool in = b + l < n;
    const int64_t c = in ? ccol[s + b + l] : 0;
    const double v = in ? cval[s + b + l] : 0.0;
    const bool isd = in && c >= cstart && c < cend;
    const bool iso = in && !isd;
    const unsigned long long bd = seg_bits<W>(__ballot(isd), gbase), bo = seg_bits<W>(__ballot(iso), gbase);
    const unsigned long long bg = seg_bits<W>(__ballot(isd && c == grow), gbase);
    if (isd) {
      const int64_t t = pd + __popcll(bd & below);
      dcol[t] = (int32_t)(c - cstart);
      dval[t] = v;
      if (c == grow) diag[row] = v;
    } else if (iso) {
      const int64_t w = c >> 5;
      const unsigned bit = (unsigned)(c & 31);
      const int64_t t = po + __popcll(bo & below);
      ocol[t] = (int32_t)(wbase[w] + __popc(bitmap[w] & ((1u << bit) - 1u)));
      oval[t] = v;
    }
    pd += __popcll(bd);
    po += __popcll(bo);
    have_diag = have_diag || bg != 0;
  }
  if (rv && l == 0 && !have_diag) diag[row] = 0.0;
}

__global__ void popc_kernel(int64_t nw, const unsigned *__restrict__ bitmap, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) out[w] = __popc(bitmap[w]);
}

__global__ void garray_kernel(int64_t nw, const unsigned *__restrict__ bitmap,
                              const int64_t *__restrict__ wbase, int64_t *__restrict__ garray) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    unsigned b = bitmap[w];
    int64_t k = wbase[w];
    while (b) {
      int bit = __ffs(b) - 1;
      garray[k++] = (w << 5) + bit;
      b &= b - 1;
    }
  }
}

// ---------------------------------------------------------------- SELL-64
// One wave per slice: longest row (SELL width) and, for the diagonal block,
// the distinct column offsets d = col - row in ascending order (enumerated by
// repeated wave-min over each lane's sorted row).  Picks the aligned-offset
// format when 8 k + 4 < 12 w bytes per row.  The slice's columns are staged
// in LDS by contiguous loads first: the walk's k dependent steps then wait on
// LDS, not on a global load each (3.25 ms for a 27-point share when every
// step went to memory, round 5).  A slice with more entries than the stage
// walks global memory.
constexpr int SELL_STAGE = 2048;

__global__ void __launch_bounds__(64) slice_format_kernel(int64_t m, const int64_t *__restrict__ ptr,
                                                          const int32_t *__restrict__ col, int64_t nslices,
                                                          int allow_dia, int32_t *__restrict__ width,
                                                          int64_t *__restrict__ slots, int32_t *__restrict__ doff) {
  __shared__ int32_t lc[SELL_STAGE];
  const int64_t s = blockIdx.x;
  if (s >= nslices) return;   // block-uniform
  const int lane = threadIdx.x;
  const int64_t row = s * SLICE + lane;
  int64_t a = 0, b = 0;
  if (row < m) { a = ptr[row]; b = ptr[row + 1]; }
  int len = (int)(b - a);
  int w = len;
  for (int o = 32; o > 0; o >>= 1) w = max(w, __shfl_xor(w, o, 64));
  int k = 0;
  if (allow_dia && w > 0) {
    const int64_t r0 = s * SLICE, r1 = min(m, r0 + SLICE);
    const int64_t a0 = ptr[r0], cnt = ptr[r1] - a0;
    const bool staged = cnt <= SELL_STAGE;   // block-uniform
    if (staged) {
      for (int64_t e = lane; e < cnt; e += 64) lc[e] = col[a0 + e];
      __syncthreads();
    }
    int64_t cur = a;
    while (true) {
      int my = INT_MAX;
      if (cur < b) my = (int)((staged ? lc[cur - a0] : col[cur]) - row);
      int mn = my;
      for (int o = 32; o > 0; o >>= 1) mn = min(mn, __shfl_xor(mn, o, 64));
      if (mn == INT_MAX) break;
      if (k == DIA_MAX) { k = DIA_MAX + 1; break; }
      if (lane == 0) doff[s * DIA_MAX + k] = mn;
      ++k;
      if (my == mn) ++cur;
    }
  }
  const bool dia = allow_dia && w > 0 && k <= DIA_MAX && (8 * k + 4 < 12 * w);
  if (lane == 0) {
    width[s] = dia ? -k : w;
    slots[s] = (int64_t)(dia ? k : w) * SLICE;
  }
}

__device__ __forceinline__ int64_t sell_slot(int64_t base, int j, int w, int lane, bool paired) {
  if (!paired) return base + (int64_t)j * SLICE + lane;
  return base + ((j >> 1) < (w >> 1) ? (int64_t)(j >> 1) * 2 * SLICE + 2 * lane + (j & 1)
                                     : (int64_t)(w >> 1) * 2 * SLICE + lane);
}

// SELL fill, one wave per slice, with the slice's canonical entries staged in LDS: a
// slice's 64 rows are one contiguous range of the CSR arrays, so the wave
// reads it with contiguous loads and each lane then walks its row in LDS
// (the global row walks touched 64 lines per load, lanes ~K entries apart:
// 8.1 ms for a 27-point share, round 5).  One wave per block; a slice with
// more entries than the staging buffer takes the global walk.  Aligned-offset
// slices are filled by sell_fill_dia_kernel (they return at once here).

template <bool PAIRED>
__global__ void __launch_bounds__(64) sell_fill_lds_kernel(int64_t m, const int64_t *__restrict__ ptr,
                                                           const int32_t *__restrict__ ccol,
                                                           const double *__restrict__ cval, int64_t nslices,
                                                           const int64_t *__restrict__ sptr,
                                                           const int32_t *__restrict__ width,
                                                           const int32_t *__restrict__ doff, int32_t *__restrict__ scol,
                                                           double *__restrict__ sval, uint32_t *__restrict__ mask,
                                                           uint8_t *__restrict__ mask8) {
  __shared__ int32_t lc[SELL_STAGE];
  __shared__ double lv[SELL_STAGE];
  const int64_t s = blockIdx.x;
  if (s >= nslices) return;
  const int wr = width[s];
  if (wr < 0) return;                 // aligned-offset slice: sell_fill_dia_kernel
  const int lane = threadIdx.x;
  const int64_t row = s * SLICE + lane;
  const int64_t r0 = s * SLICE, r1 = min(m, r0 + SLICE);
  const int64_t a0 = ptr[r0], cnt = ptr[r1] - a0;
  const int64_t base = sptr[s];
  const int64_t rs = row < m ? ptr[row] : a0;
  const int len = row < m ? (int)(ptr[row + 1] - rs) : 0;
  const bool staged = cnt <= SELL_STAGE;   // block-uniform
  if (staged) {
    for (int64_t e = lane; e < cnt; e += 64) { lc[e] = ccol[a0 + e]; lv[e] = cval[a0 + e]; }
    __syncthreads();
  }
  const int32_t *__restrict__ rc = staged ? lc + (rs - a0) : ccol + rs;
  const double *__restrict__ rvv = staged ? lv + (rs - a0) : cval + rs;
  const int w = wr;
  for (int j = 0; j < w; ++j) {
    const bool in = j < len;
    const int64_t t = sell_slot(base, j, w, lane, PAIRED);
    scol[t] = in ? rc[j] : -1;
    sval[t] = in ? rvv[j] : 0.0;
  }
}

// ---------------------------------------------------------------- offset patterns
// The aligned-offset slices of a stencil share a handful of offset lists.
// SpMV reads a slice's list right after its width, on the dependent path to
// the gathers; one list per slice (128 B each) missed in the caches on every
// slice, a shared table stays resident.  Slices are grouped by a hash of the
// list, and every slice is checked against its group's list (any mismatch
// keeps the per-slice lists).
__global__ void dia_hash_kernel(int64_t ns, const int32_t *__restrict__ width, const int32_t *__restrict__ doff,
                                unsigned long long *__restrict__ h) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns) return;
  const int w = width[s];
  unsigned long long x = 0xcbf29ce484222325ULL ^ (unsigned long long)(uint32_t)w;
  if (w < 0)
    for (int j = 0; j < -w; ++j) x = (x ^ (unsigned long long)(uint32_t)doff[s * DIA_MAX + j]) * 0x100000001b3ULL;
  h[s] = w < 0 ? x : 0ULL;
}

__global__ void dia_pattern_gather_kernel(int npat, const int64_t *__restrict__ rep, const int32_t *__restrict__ doff,
                                          int32_t *__restrict__ ptab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)npat * DIA_MAX) return;
  ptab[i] = doff[rep[i / DIA_MAX] * DIA_MAX + i % DIA_MAX];
}

__global__ void dia_pattern_check_kernel(int64_t ns, const int32_t *__restrict__ width, const int32_t *__restrict__ doff,
                                         const int32_t *__restrict__ dpat, const int32_t *__restrict__ ptab,
                                         int *__restrict__ bad) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns || width[s] >= 0) return;
  for (int j = 0; j < -width[s]; ++j)
    if (doff[s * DIA_MAX + j] != ptab[(int64_t)dpat[s] * DIA_MAX + j]) *bad = 1;
}

// bit DPAT_INB of dpat[s]: every gather of the slice (rows 64 s .. 64 s + 63,
// present or not) lies inside the operand, so SpMV takes the unguarded body
// without scanning the offsets
__global__ void dia_inb_kernel(int64_t ns, int64_t ncols, const int32_t *__restrict__ width,
                               const int32_t *__restrict__ ptab, int32_t *__restrict__ dpat) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns || width[s] >= 0) return;
  const int32_t *off = ptab + (int64_t)dpat[s] * DIA_MAX;
  int omin = off[0], omax = off[0];
  for (int j = 1; j < -width[s]; ++j) { omin = min(omin, off[j]); omax = max(omax, off[j]); }
  const int64_t srow = s * SLICE;
  if (srow + omin >= 0 && srow + (SLICE - 1) + omax < ncols) dpat[s] |= DPAT_INB;
}

static void share_offset_patterns(Sell &S, const std::vector<int32_t> &wh, int64_t ncols, hipStream_t st) {
  const int64_t ns = S.nslices;
  S.dpat.alloc((size_t)ns);
  std::vector<int32_t> pat((size_t)ns);
  for (int64_t s = 0; s < ns; ++s) pat[s] = (int32_t)s;        // fallback: one list per slice
  S.npat = ns;
  {
    DBuf<unsigned long long> hd((size_t)ns);
    dia_hash_kernel<<<(unsigned)cdiv(ns, 256), 256, 0, st>>>(ns, S.width.p, S.doff.p, hd.p);
    HIPCHECK(hipGetLastError());
    std::vector<unsigned long long> hh((size_t)ns);
    HIPCHECK(hipMemcpyAsync(hh.data(), hd.p, sizeof(unsigned long long) * ns, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    std::unordered_map<unsigned long long, int32_t> id;
    std::vector<int64_t> rep;
    std::vector<int32_t> p2((size_t)ns, 0);
    unsigned long long last = 0;
    int32_t last_id = -1;
    for (int64_t s = 0; s < ns; ++s) {
      if (wh[s] >= 0) continue;
      if (last_id >= 0 && hh[s] == last) { p2[s] = last_id; continue; }
      auto it = id.find(hh[s]);
      if (it == id.end()) {
        it = id.emplace(hh[s], (int32_t)rep.size()).first;
        rep.push_back(s);
      }
      p2[s] = last_id = it->second;
      last = hh[s];
    }
    if ((int64_t)rep.size() * 4 < ns) {
      const int npat = (int)rep.size();
      DBuf<int64_t> rd((size_t)npat);
      DBuf<int32_t> ptab((size_t)npat * DIA_MAX);
      DBuf<int> bad(1);
      HIPCHECK(hipMemcpyAsync(rd.p, rep.data(), sizeof(int64_t) * npat, hipMemcpyHostToDevice, st));
      HIPCHECK(hipMemcpyAsync(S.dpat.p, p2.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice, st));
      HIPCHECK(hipMemsetAsync(bad.p, 0, sizeof(int), st));
      dia_pattern_gather_kernel<<<(unsigned)cdiv((int64_t)npat * DIA_MAX, 256), 256, 0, st>>>(npat, rd.p, S.doff.p,
                                                                                                ptab.p);
      dia_pattern_check_kernel<<<(unsigned)cdiv(ns, 256), 256, 0, st>>>(ns, S.width.p, S.doff.p, S.dpat.p, ptab.p,
                                                                        bad.p);
      HIPCHECK(hipGetLastError());
      int hb = 0;
      HIPCHECK(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (!hb) {
        // the dominant pattern of the dominant width (row-pair layout, below)
        std::vector<int64_t> cnt((size_t)npat, 0);
        for (int64_t q = 0; q < ns; ++q)
          if (wh[q] == -S.dia_k) cnt[p2[q]]++;
        const int star = (int)(std::max_element(cnt.begin(), cnt.end()) - cnt.begin());
        if (cnt[star] > 0) {
          S.pat_star = star;
          S.pat_star_off.resize((size_t)S.dia_k);
          HIPCHECK(hipMemcpyAsync(S.pat_star_off.data(), ptab.p + (size_t)star * DIA_MAX, sizeof(int32_t) * S.dia_k,
                                  hipMemcpyDeviceToHost, st));
          HIPCHECK(hipStreamSynchronize(st));
        }
        S.pat_len.resize((size_t)npat);
        for (int q = 0; q < npat; ++q) S.pat_len[(size_t)q] = -wh[(size_t)rep[(size_t)q]];
        S.pat_host.resize((size_t)npat * DIA_MAX);
        HIPCHECK(hipMemcpyAsync(S.pat_host.data(), ptab.p, sizeof(int32_t) * S.pat_host.size(), hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        S.doff = std::move(ptab);
        S.npat = npat;
        dia_inb_kernel<<<(unsigned)cdiv(ns, 256), 256, 0, st>>>(ns, ncols, S.width.p, S.doff.p, S.dpat.p);
        HIPCHECK(hipGetLastError());
        return;
      }
    }
  }
  HIPCHECK(hipMemcpyAsync(S.dpat.p, pat.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice, st));
  dia_inb_kernel<<<(unsigned)cdiv(ns, 256), 256, 0, st>>>(ns, ncols, S.width.p, S.doff.p, S.dpat.p);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));
}

// ---------------------------------------------------------------- value codes
// A stencil or FEM block with few distinct coefficients streams one byte per
// slot instead of eight: the distinct values (bit patterns) are collected in
// an open-addressing table, and when there are at most VCODE_MAX of them every
// slot stores its value's index.  SpMV reads the table from LDS, so the
// product uses the very same doubles (bitwise results unchanged).
constexpr int VDICT_SLOTS = 4096;
constexpr unsigned long long VDICT_EMPTY = 0x7ff8dead5eed1e55ULL;   // a NaN payload; never a key

__device__ __forceinline__ unsigned vdict_hash(unsigned long long k) {
  return (unsigned)((k * 0x9E3779B97F4A7C15ULL) >> 52);   // 12 bits
}

// one wave per slice, the slots a row stores (absent aligned-offset slots
// and padding skipped).  st[0] = distinct values inserted, st[1] = overflow
// (too many, or a value with the empty pattern).  A plain read that sees
// EMPTY falls through to the CAS, which returns the slot's real content; keys
// never leave a slot.
__device__ __forceinline__ bool vdict_insert(unsigned long long *tab, int *st, unsigned long long k) {
  if (k == VDICT_EMPTY) return false;
  unsigned h = vdict_hash(k);
  for (int probe = 0; probe < 64; ++probe) {
    unsigned long long c = tab[h];
    if (c == VDICT_EMPTY) {
      c = atomicCAS(tab + h, VDICT_EMPTY, k);
      if (c == VDICT_EMPTY) return atomicAdd(st, 1) < VCODE_ABSENT;
    }
    if (c == k) return true;
    h = (h + 1) & (VDICT_SLOTS - 1);
  }
  return false;
}

__device__ __forceinline__ bool slot_stored(int wr, uint32_t mk, const int32_t *__restrict__ col, int64_t t, int j) {
  return wr < 0 ? ((mk >> j) & 1u) != 0 : col[t] >= 0;
}

// The aligned-offset slices' fill (paired slot order), one slice per 256-thread
// block: the slice's CSR entries are read in order by contiguous loads, each
// placed in an LDS image of the slice's k x 64 slots by its row (a search of
// the slice's row starts) and its offset's rank in the slice's ascending list
// (a search of doff), with the row's presence bit; then the image is written
// out as 16-byte slot pairs, absent slots 0.0.  The same slots and masks as a
// per-row walk (every entry's offset is in the list, which slice_format_kernel
// enumerated from these rows), without a wave walking 64 rows ~k entries apart
// (6.4 ms for a 27-point share at 6 waves per CU, round 5).  With tab set it
// also collects the value dictionary (vdict_insert_kernel's table, which then
// skips these slices): the slice's stored values go through an LDS set first,
// a plain read before any CAS, so a value the slice repeats costs one LDS
// read, and only the slice's distinct values reach the global table.
__global__ void __launch_bounds__(256) sell_fill_dia_kernel(int64_t m, const int64_t *__restrict__ ptr,
                                                            const int32_t *__restrict__ ccol,
                                                            const double *__restrict__ cval, int64_t nslices,
                                                            const int64_t *__restrict__ sptr,
                                                            const int32_t *__restrict__ width,
                                                            const int32_t *__restrict__ doff, double *__restrict__ sval,
                                                            uint32_t *__restrict__ mask, uint8_t *__restrict__ mask8,
                                                            unsigned long long *tab, int *vst) {
  constexpr int VS_N = 64;
  __shared__ double img[DIA_MAX * SLICE];
  __shared__ unsigned long long vs[VS_N];
  __shared__ int32_t rs[SLICE + 1], dl[DIA_MAX];
  __shared__ uint32_t mk[SLICE];
  const int64_t s = blockIdx.x;
  if (s >= nslices) return;
  const int wr = width[s];
  if (wr >= 0) return;                // block-uniform: a SELL slice
  const int k = -wr, t = threadIdx.x;
  const int64_t r0 = s * SLICE, r1 = min(m, r0 + SLICE);
  const int nr = (int)(r1 - r0);
  const int64_t a0 = ptr[r0];
  if (t <= SLICE) rs[t] = (int32_t)(ptr[r0 + min(t, nr)] - a0);
  if (t < SLICE) mk[t] = 0u;
  if (t < k) dl[t] = doff[s * DIA_MAX + t];
  if (t < VS_N) vs[t] = VDICT_EMPTY;
  __syncthreads();
  const int cnt = rs[SLICE];
  for (int e = t; e < cnt; e += 256) {
    const int32_t c = ccol[a0 + e];
    const double v = cval[a0 + e];
    int lo = 0, hi = nr - 1;                      // the last row starting at or before e
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (rs[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const int off = (int)((int64_t)c - (r0 + lo));
    int jl = 0, jh = k - 1;                       // off's rank in the ascending list
    while (jl < jh) {
      const int mid = (jl + jh) >> 1;
      if (dl[mid] < off) jl = mid + 1; else jh = mid;
    }
    img[jl * SLICE + lo] = v;
    atomicOr(&mk[lo], 1u << jl);
  }
  __syncthreads();
  if (tab && !*(volatile int *)(vst + 1)) {       // block-uniform
    for (int q = t; q < k * SLICE; q += 256) {
      const int j = q / SLICE, l = q % SLICE;
      if (!((mk[l] >> j) & 1u)) continue;
      const unsigned long long key = (unsigned long long)__double_as_longlong(img[q]);
      if (key == VDICT_EMPTY) { vst[1] = 1; continue; }
      unsigned h = vdict_hash(key) & (VS_N - 1);
      bool done = false;
      for (int probe = 0; probe < VS_N && !done; ++probe) {
        unsigned long long c = vs[h];
        if (c == VDICT_EMPTY) c = atomicCAS(&vs[h], VDICT_EMPTY, key);
        done = c == VDICT_EMPTY || c == key;
        h = (h + 1) & (VS_N - 1);
      }
      if (!done && !vdict_insert(tab, vst, key)) vst[1] = 1;   // the LDS set full: straight to the table
    }
    __syncthreads();
    if (t < VS_N && vs[t] != VDICT_EMPTY && !vdict_insert(tab, vst, vs[t])) vst[1] = 1;
  }
  const int64_t base = sptr[s];
  const int np = k >> 1;
  for (int q = t; q < np * SLICE; q += 256) {     // slot pairs (2 jp, 2 jp + 1) of row l
    const int jp = q / SLICE, l = q % SLICE, j = 2 * jp;
    const uint32_t b = mk[l];
    const double v0 = (b >> j) & 1u ? img[j * SLICE + l] : 0.0;
    const double v1 = (b >> (j + 1)) & 1u ? img[(j + 1) * SLICE + l] : 0.0;
    *reinterpret_cast<double2 *>(sval + base + (int64_t)jp * 2 * SLICE + 2 * l) = make_double2(v0, v1);
  }
  if (k & 1) {                                    // the odd last slot, one per row
    const int j = k - 1;
    for (int l = t; l < SLICE; l += 256) sval[base + (int64_t)np * 2 * SLICE + l] = (mk[l] >> j) & 1u ? img[j * SLICE + l] : 0.0;
  }
  if (t < SLICE) {                                // rows past m: 0, as their slots
    if (mask8) mask8[r0 + t] = (uint8_t)mk[t];
    else mask[r0 + t] = mk[t];
  }
}

// (skip_dia: the aligned-offset slices' values were collected by sell_fill_dia_kernel)
__global__ void vdict_insert_kernel(int64_t ns, const int64_t *__restrict__ sptr, const int32_t *__restrict__ width,
                                    const int32_t *__restrict__ col, const double *__restrict__ sval,
                                    const uint32_t *__restrict__ mask, const uint8_t *__restrict__ mask8,
                                    unsigned long long *tab, int *st, int skip_dia) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= ns || *(volatile int *)(st + 1)) return;
  const int lane = threadIdx.x & 63;
  const int wr = width[s];
  if (skip_dia && wr < 0) return;
  const int w = wr < 0 ? -wr : wr;
  const int64_t row = s * SLICE + lane;
  const uint32_t mk = wr >= 0 ? 0u : (mask8 ? (uint32_t)mask8[row] : mask[row]);
  unsigned long long last = VDICT_EMPTY;
  for (int j = 0; j < w; ++j) {
    const int64_t t = sell_slot(sptr[s], j, w, lane, true);
    const bool stored = slot_stored(wr, mk, col, t, j);
    const unsigned long long k = stored ? (unsigned long long)__double_as_longlong(sval[t]) : VDICT_EMPTY;
    // a stencil slot holds one value across the wave: lane 0 alone inserts it
    const unsigned long long k0 = __shfl(k, 0, 64);
    const bool uniform = __all(k == k0 || !stored);
    if (!stored || k == last || (uniform && lane != 0 && k0 != VDICT_EMPTY)) continue;
    last = k;
    if (!vdict_insert(tab, st, k)) { st[1] = 1; return; }
  }
}

__global__ void code_bytes_kernel(int64_t ns, const int32_t *__restrict__ width, int64_t *__restrict__ cb) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns) return;
  const int w = width[s] < 0 ? -width[s] : width[s];
  cb[s] = (int64_t)((w + 7) / 8) * CODE_BATCH;
}

// ---------------------------------------------------------------- row pairs
// Units of 128 rows (slices 2u, 2u+1) whose both slices are aligned-offset
// slices with an offset pattern contained in the dominant one are stored a
// second time as row pairs: lane l owns rows 128 u + 2 l and + 1, its codes
// are [K codes of row 0][K codes of row 1] in the dominant pattern's slot
// order, padded to PB bytes; a slot whose offset the row does not store is
// VCODE_ABSENT.  SpMV loads x as 16-byte pairs -- one load per run of the
// pattern instead of one per offset and row (mx_spmv.hip, pair body) --
// through buffer loads that read 0 outside the operand, so the boundary
// units of a stencil (first/last planes, lines, and the planes next to
// another rank's rows, whose A_o entries the boundary kernel adds) are pair
// units too.  Shapes (sorted offsets):
//   5:  a, -1, 0, 1, b          (2D 5-point)
//   7:  a, b, -1, 0, 1, c, d    (3D 7-point)
//   27: nine runs c-1, c, c+1   (3D 27-point)
// with every singleton and run centre even (16-byte aligned pairs).
static int pair_shape_of(const std::vector<int32_t> &o) {
  const int k = (int)o.size();
  auto even = [](int32_t v) { return (v & 1) == 0; };
  auto tri = [&](int j) { return o[j + 1] == o[j] + 1 && o[j + 2] == o[j] + 2 && even(o[j + 1]); };
  if (k == 5 && tri(1) && o[2] == 0 && even(o[0]) && even(o[4]) && o[0] < o[1] - 1 && o[4] > o[3] + 1) return 5;
  if (k == 7 && tri(2) && o[3] == 0 && even(o[0]) && even(o[1]) && even(o[5]) && even(o[6]) &&
      o[1] < o[2] - 1 && o[5] > o[4] + 1)
    return 7;
  if (k == 27) {
    for (int t = 0; t < 9; ++t)
      if (!tri(3 * t)) return 0;
    return o[13] == 0 ? 27 : 0;
  }
  return 0;
}

constexpr int pair_bytes(int k) { return (2 * k + 15) / 16 * 16; }

// Value codes and row-pair codes in one pass, one 128-thread block per unit
// (slices 2u and 2u + 1, a wave each).  Each wave writes its slice's code
// words (lane = row, 8 slots per 8-byte word; absent slots of aligned-offset
// rows and slots past the width get VCODE_ABSENT, whose table entry is 0.0)
// and keeps an aligned-offset slice's codes in LDS.  A pair unit then gathers
// its lanes' 2K codes from there by a per-pattern slot map built on the host
// (dominant slot j -> the slot of the slice's own pattern, and whether the
// pattern's offsets all belong to the dominant one), writes them as 8-byte
// words and sets DPAT_PAIR on slice 2u.  Round 4's pair fill scanned the
// patterns and probed the value table per slot with single-byte stores
// (16.3 ms for a 27-point share); round 5's separate pass read each code
// back with a byte load (1.7 ms).  pcode = nullptr: code words only.
__global__ void __launch_bounds__(128) code_pair_fill_kernel(
    int64_t m, int64_t ns, const int64_t *__restrict__ sptr, const int32_t *__restrict__ width,
    const int32_t *__restrict__ col, const double *__restrict__ sval, const int64_t *__restrict__ cptr,
    const unsigned long long *__restrict__ keys, int ntab, const uint32_t *__restrict__ mask, const uint8_t *__restrict__ mask8, uint8_t *__restrict__ code,
    int64_t nunits, int k, int32_t *__restrict__ dpat, const int8_t *__restrict__ pmap,
    const uint8_t *__restrict__ pok, uint8_t *__restrict__ pcode) {
  __shared__ uint8_t lcode[2][DIA_MAX][SLICE];
  __shared__ unsigned long long kl[VCODE_MAX];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t u = blockIdx.x, s = 2 * u + wv;
  for (int i = threadIdx.x; i < ntab; i += 128) kl[i] = keys[i];
  __syncthreads();
  // a value's code: its rank among the sorted keys (S.vtab's order), 0 if absent
  auto code_of = [&](double v) -> unsigned long long {
    const unsigned long long key = (unsigned long long)__double_as_longlong(v);
    int lo = 0, hi = ntab;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (kl[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo < ntab && kl[lo] == key ? (unsigned long long)lo : 0ULL;
  };
  if (s < ns) {
    const int wr = width[s];
    const int w = wr < 0 ? -wr : wr;
    const int64_t base = sptr[s];
    const int64_t row = s * SLICE + lane;
    const uint32_t mk = wr >= 0 ? 0u : (mask8 ? (uint32_t)mask8[row] : mask[row]);
    for (int b = 0; b < (w + 7) / 8; ++b) {
      unsigned long long word = 0;
      for (int q = 0; q < 8; q += 2) {
        const int j = 8 * b + q;
        unsigned long long c[2] = {VCODE_ABSENT, VCODE_ABSENT};
        if (wr < 0 && j + 1 < w) {                 // an aligned-offset slot pair: one 16-byte load
          const double2 v2 = *reinterpret_cast<const double2 *>(sval + sell_slot(base, j, w, lane, true));
          if ((mk >> j) & 1u) c[0] = code_of(v2.x);
          if ((mk >> (j + 1)) & 1u) c[1] = code_of(v2.y);
        } else {
          for (int h = 0; h < 2; ++h) {
            const int64_t t = j + h < w ? sell_slot(base, j + h, w, lane, true) : 0;
            if (j + h < w && slot_stored(wr, mk, col, t, j + h)) c[h] = code_of(sval[t]);
          }
        }
        for (int h = 0; h < 2; ++h) {
          if (wr < 0 && j + h < w) lcode[wv][j + h][lane] = (uint8_t)c[h];
          word |= c[h] << (8 * (q + h));
        }
      }
      reinterpret_cast<unsigned long long *>(code + cptr[s] + (int64_t)b * CODE_BATCH)[lane] = word;
    }
  }
  if (!pcode || u >= nunits) return;   // block-uniform
  __syncthreads();
  const int64_t s0 = 2 * u, s1 = s0 + 1;
  if (u * 128 + 127 >= m || width[s0] >= 0 || width[s1] >= 0) return;   // block-uniform
  const int p0 = dpat[s0] & DPAT_ID, p1 = dpat[s1] & DPAT_ID;
  if (!pok[p0] || !pok[p1]) return;
  const int hs = lane < 32 ? 0 : 1;
  const int8_t *__restrict__ mp = pmap + (int64_t)(hs ? p1 : p0) * DIA_MAX;
  const int pb = pair_bytes(k);
  unsigned long long *dst = reinterpret_cast<unsigned long long *>(pcode + (u * 64 + lane) * pb);
  for (int w = wv; w < pb / 8; w += 2) {
    unsigned long long word = 0;
    for (int t = 0; t < 8; ++t) {
      const int idx = 8 * w + t;
      unsigned long long c = VCODE_ABSENT;
      if (idx < 2 * k) {
        const int h = idx >= k ? 1 : 0;
        const int q = mp[idx - h * k];
        if (q >= 0) c = lcode[hs][q][(2 * lane + h) & 63];
      }
      word |= c << (8 * t);
    }
    dst[w] = word;
  }
  if (threadIdx.x == 0) dpat[s0] |= DPAT_PAIR;
}

// fp64 row pairs (Sell::pval / pflag): one wave per unit, the pair_fill_kernel
// slot mapping with values instead of codes; the unit's presence ballots give
// its select-free flags (build_pair_uniform's rule), and a unit that is not
// select-free (or not a pair unit) clears *clean
__global__ void pair_fill_f64_kernel(int64_t m, int64_t nunits, int k, int ps, int32_t star,
                                     const int64_t *__restrict__ sptr, const int32_t *__restrict__ width,
                                     const int32_t *__restrict__ dpat, const int32_t *__restrict__ doff,
                                     const double *__restrict__ sval, const uint32_t *__restrict__ mask,
                                     const uint8_t *__restrict__ mask8, double *__restrict__ pval,
                                     int32_t *__restrict__ pflag, int *__restrict__ clean) {
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= nunits) return;
  const int lane = threadIdx.x & 63;
  const int32_t *__restrict__ so = doff + (int64_t)star * DIA_MAX;
  auto slot_of = [&](int64_t sl, int j) -> int {
    const int32_t *__restrict__ po = doff + (int64_t)(dpat[sl] & DPAT_ID) * DIA_MAX;
    for (int q = 0; q < -width[sl]; ++q)
      if (po[q] == so[j]) return q;
    return -1;
  };
  auto ok = [&](int64_t sl) {
    if (width[sl] >= 0) return false;
    const int32_t *__restrict__ po = doff + (int64_t)(dpat[sl] & DPAT_ID) * DIA_MAX;
    for (int q = 0; q < -width[sl]; ++q) {
      bool in = false;
      for (int j = 0; j < k; ++j) in = in || po[q] == so[j];
      if (!in) return false;
    }
    return true;
  };
  if (u * 128 + 127 >= m || !ok(2 * u) || !ok(2 * u + 1)) {   // wave-uniform
    if (lane == 0) *clean = 0;
    return;
  }
  unsigned long long pm[2][8];
  for (int j = 0; j < k; ++j) {
    double v[2];
    bool pr[2];
    for (int h = 0; h < 2; ++h) {
      const int64_t row = u * 128 + 2 * lane + h;
      const int64_t sl = row >> 6;
      const int li = (int)(row & 63);
      const uint32_t mk = mask8 ? (uint32_t)mask8[row] : mask[row];
      const int q = slot_of(sl, j);
      pr[h] = q >= 0 && ((mk >> q) & 1u);
      v[h] = pr[h] ? sval[sell_slot(sptr[sl], q, -width[sl], li, true)] : 0.0;
    }
    reinterpret_cast<double2 *>(pval)[(u * k + j) * 64 + lane] = make_double2(v[0], v[1]);
    pm[0][j] = __ballot(pr[0]);
    pm[1][j] = __ballot(pr[1]);
  }
  if (lane != 0) return;
  const unsigned long long F = ~0ull;
  const int NR = ps == 5 ? 3 : 5;
  uint32_t f = 0;
  bool cl = true;
  for (int r = 0; r < NR && cl; ++r) {
    const bool tri = ps == 5 ? r == 1 : r == 2;
    const int j = ps == 5 ? (r == 0 ? 0 : r == 1 ? 1 : 4) : (r < 2 ? r : r == 2 ? 2 : r + 2);
    if (!tri) {
      if (pm[0][j] == 0 && pm[1][j] == 0) f |= PBLK_RUN0 << r;
      else if (pm[0][j] != F || pm[1][j] != F) cl = false;
      continue;
    }
    const unsigned long long m0 = pm[0][j], m1 = pm[0][j + 1], m2 = pm[0][j + 2];
    const unsigned long long n0 = pm[1][j], n1 = pm[1][j + 1], n2 = pm[1][j + 2];
    if ((m0 | m1 | m2 | n0 | n1 | n2) == 0) { f |= (PBLK_RUN0 << r) | PBLK_ELO | PBLK_EHI; continue; }
    if (m1 != F || m2 != F || n0 != F || n1 != F) cl = false;
    else if (m0 != F && m0 != (F & ~1ull)) cl = false;
    else if (n2 != F && n2 != (F >> 1)) cl = false;
    if (m0 != F) f |= PBLK_ELO;
    if (n2 != F) f |= PBLK_EHI;
  }
  pflag[u] = (int32_t)f;
  if (!cl) *clean = 0;
}

__global__ void pair_f64_ghost_kernel(int64_t nunits, int64_t nslices, const int32_t *__restrict__ wid_o,
                                      int32_t *__restrict__ pflag) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits) return;
  uint32_t f = 0;
  if (wid_o[2 * u]) f |= PBLK_GHOST_LO;
  if (2 * u + 1 < nslices && wid_o[2 * u + 1]) f |= PBLK_GHOST_HI;
  if (f) pflag[u] = (int32_t)((uint32_t)pflag[u] | f);
}

// fp64 row-pair layout for uncoded 5/7-point diagonal blocks (wid_o: the A_o
// widths per slice on a multi-rank matrix -- units with ghost entries are
// flagged, the SpMV then splits and the boundary kernel finishes them)
static void build_pair_f64(Sell &S, int64_t m, int64_t ncols, const int32_t *wid_o, hipStream_t st) {
  S.pval.reset();
  S.pflag.reset();
  S.pair_f64 = 0;
  if (!g_knobs.pair_f64 || S.ntab > 0 || S.pat_star < 0 || m % 128 != 0 || m > (int64_t(1) << 27) ||
      ncols > (int64_t(1) << 27) || S.nslices * 64 != m)
    return;
  const int ps = pair_shape_of(S.pat_star_off);
  if ((ps != 5 && ps != 7) || S.dia_k != ps) return;
  const int64_t nu = m / 128;
  S.pval.alloc((size_t)nu * ps * 128);
  S.pflag.alloc((size_t)nu);
  DBuf<int> clean(1);
  const int one = 1;
  HIPCHECK(hipMemcpyAsync(clean.p, &one, sizeof(int), hipMemcpyHostToDevice, st));
  pair_fill_f64_kernel<<<(unsigned)cdiv(nu, 4), 256, 0, st>>>(m, nu, ps, ps, S.pat_star, S.sptr.p, S.width.p, S.dpat.p,
                                                              S.doff.p, S.val.p, S.mask.p, S.mask8.p, S.pval.p,
                                                              S.pflag.p, clean.p);
  HIPCHECK(hipGetLastError());
  int hc = 0;
  HIPCHECK(hipMemcpyAsync(&hc, clean.p, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  if (!hc) { S.pval.reset(); S.pflag.reset(); return; }
  if (wid_o) {      // the ghost flags go into the flag word as into pblk (pair units only here)
    pair_f64_ghost_kernel<<<(unsigned)cdiv(nu, 256), 256, 0, st>>>(nu, S.nslices, wid_o, S.pflag.p);
    HIPCHECK(hipGetLastError());
  }
  S.pair_f64 = ps;
}

__global__ void pair_count_kernel(int64_t nunits, const int32_t *__restrict__ dpat, unsigned long long *__restrict__ cnt) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool p = u < nunits && (dpat[2 * u] & DPAT_PAIR);
  const unsigned long long b = __ballot(p);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(cnt, (unsigned long long)__popcll(b));
}

// pblk flags of the pair units whose slices hold off-diagonal (A_o) entries:
// SpMV stores their diagonal-block sums and the boundary kernel finishes them
__global__ void pair_ghost_flags_kernel(int64_t nunits, int64_t nslices, const int32_t *__restrict__ dpat,
                                        const int32_t *__restrict__ wid_o, int32_t *__restrict__ pblk,
                                        int *__restrict__ any) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits || !(dpat[2 * u] & DPAT_PAIR)) return;
  uint32_t f = 0;
  if (wid_o[2 * u]) f |= PBLK_GHOST_LO;
  if (2 * u + 1 < nslices && wid_o[2 * u + 1]) f |= PBLK_GHOST_HI;
  if (f) {
    pblk[u] = (int32_t)((uint32_t)pblk[u] | f);
    *any = 1;
  }
}

// Code-block dictionary of the row-pair layout.  A unit's code block (64
// lanes x pair_bytes) depends only on which slots of its 128 rows are present
// and on their value codes, so a stencil block has a few dozen distinct blocks
// (the x-line position of the unit, the y/z boundary class, the coefficient
// class) however many units it has.  Distinct blocks are found by a 64-bit
// hash per unit (host map), copied to a dictionary, and every unit is then
// compared byte for byte with its dictionary block on the device; a hash
// collision, or more distinct blocks than fit comfortably in L2, keeps one
// block per unit.  SpMV then reads 4 bytes per 128 rows plus L2-resident
// dictionary lines instead of pair_bytes per row pair from HBM.
__global__ void pair_hash_kernel(int64_t nunits, int pb, const int32_t *__restrict__ dpat,
                                 const uint8_t *__restrict__ pcode, unsigned long long *__restrict__ h) {
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= nunits) return;
  const int lane = threadIdx.x & 63;
  if (!(dpat[2 * u] & DPAT_PAIR)) {                 // wave-uniform: no code block
    if (lane == 0) h[u] = 0;
    return;
  }
  const unsigned long long *w = reinterpret_cast<const unsigned long long *>(pcode + (u * 64 + lane) * pb);
  unsigned long long a = 0x9E3779B97F4A7C15ull * (unsigned long long)(lane + 1);
  for (int q = 0; q < pb / 8; ++q) {
    a ^= w[q] + 0x632BE59BD9B4E019ull * (unsigned long long)(q + 1);
    a ^= a >> 31; a *= 0xBF58476D1CE4E5B9ull; a ^= a >> 29; a *= 0x94D049BB133111EBull; a ^= a >> 32;
  }
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if (lane == 0) h[u] = a | 1ull;
}

__global__ void pair_gather_kernel(int64_t nblocks, int pb, const int64_t *__restrict__ rep,
                                   const uint8_t *__restrict__ pcode, uint8_t *__restrict__ dict) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nblocks) return;
  const int lane = threadIdx.x & 63;
  const unsigned long long *src = reinterpret_cast<const unsigned long long *>(pcode + (rep[b] * 64 + lane) * pb);
  unsigned long long *dst = reinterpret_cast<unsigned long long *>(dict + (b * 64 + lane) * pb);
  for (int q = 0; q < pb / 8; ++q) dst[q] = src[q];
}

__global__ void pair_verify_kernel(int64_t nunits, int pb, const int32_t *__restrict__ dpat,
                                   const uint8_t *__restrict__ pcode, const int32_t *__restrict__ blk,
                                   const uint8_t *__restrict__ dict, int *__restrict__ bad) {
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= nunits) return;
  const int lane = threadIdx.x & 63;
  if (!(dpat[2 * u] & DPAT_PAIR)) return;
  const unsigned long long *a = reinterpret_cast<const unsigned long long *>(pcode + (u * 64 + lane) * pb);
  const unsigned long long *d = reinterpret_cast<const unsigned long long *>(dict + ((int64_t)blk[u] * 64 + lane) * pb);
  bool same = true;
  for (int q = 0; q < pb / 8; ++q) same = same && a[q] == d[q];
  if (!same) bad[lane] = 1;
}

constexpr int64_t PAIR_DICT_MAX_BYTES = 2 << 20;   // 2 MiB: well inside one XCD's 4 MB L2

static void dedupe_pair_blocks(Sell &S, hipStream_t st) {
  const int64_t nu = S.nunits;
  const int pb = pair_bytes(S.dia_k);
  S.pair_blocks = 0;
  std::vector<int32_t> blk((size_t)std::max<int64_t>(nu, 1));
  for (int64_t u = 0; u < nu; ++u) blk[(size_t)u] = (int32_t)u;
  S.pblk.alloc(blk.size());
  auto identity = [&] {
    for (int64_t u = 0; u < nu; ++u) blk[(size_t)u] = (int32_t)u;
    HIPCHECK(hipMemcpyAsync(S.pblk.p, blk.data(), sizeof(int32_t) * blk.size(), hipMemcpyHostToDevice, st));
    HIPCHECK(hipStreamSynchronize(st));
  };
  if (nu == 0 || !g_knobs.pdict || nu > INT32_MAX) { identity(); return; }
  DBuf<unsigned long long> hd((size_t)nu);
  pair_hash_kernel<<<(unsigned)cdiv(nu, 4), 256, 0, st>>>(nu, pb, S.dpat.p, S.pcode.p, hd.p);
  HIPCHECK(hipGetLastError());
  std::vector<unsigned long long> hh((size_t)nu);
  HIPCHECK(hipMemcpyAsync(hh.data(), hd.p, sizeof(unsigned long long) * (size_t)nu, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  const int64_t max_blocks = PAIR_DICT_MAX_BYTES / (64 * pb);
  std::unordered_map<unsigned long long, int32_t> ids;
  std::vector<int64_t> rep;
  for (int64_t u = 0; u < nu; ++u) {
    // knob 30 = 2 (tests): every unit hashes alike, so the byte comparison
    // below must reject the dictionary
    const unsigned long long k = g_knobs.pdict == 2 && hh[(size_t)u] ? 1ull : hh[(size_t)u];
    if (!k) { blk[(size_t)u] = 0; continue; }       // not a pair unit: never read
    auto it = ids.find(k);
    if (it == ids.end()) {
      if ((int64_t)rep.size() >= max_blocks) { identity(); return; }
      it = ids.emplace(k, (int32_t)rep.size()).first;
      rep.push_back(u);
    }
    blk[(size_t)u] = it->second;
  }
  const int64_t nb = (int64_t)rep.size();
  if (nb == 0 || (4 * nb > nu && g_knobs.pdict != 2)) { identity(); return; }   // too few repeats to pay for the indirection
  DBuf<int64_t> repd((size_t)nb);
  DBuf<uint8_t> dict((size_t)nb * 64 * pb);
  DBuf<int> bad(64);
  HIPCHECK(hipMemcpyAsync(repd.p, rep.data(), sizeof(int64_t) * (size_t)nb, hipMemcpyHostToDevice, st));
  HIPCHECK(hipMemcpyAsync(S.pblk.p, blk.data(), sizeof(int32_t) * blk.size(), hipMemcpyHostToDevice, st));
  HIPCHECK(hipMemsetAsync(bad.p, 0, 64 * sizeof(int), st));
  pair_gather_kernel<<<(unsigned)cdiv(nb, 4), 256, 0, st>>>(nb, pb, repd.p, S.pcode.p, dict.p);
  HIPCHECK(hipGetLastError());
  pair_verify_kernel<<<(unsigned)cdiv(nu, 4), 256, 0, st>>>(nu, pb, S.dpat.p, S.pcode.p, S.pblk.p, dict.p, bad.p);
  HIPCHECK(hipGetLastError());
  std::vector<int> bh(64);
  HIPCHECK(hipMemcpyAsync(bh.data(), bad.p, 64 * sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  for (int v : bh)
    if (v) { identity(); return; }                  // hash collision: keep every block
  S.pcode = std::move(dict);
  S.pair_blocks = nb;
}

// select-free flags of each pair unit's dictionary block (build_pair_uniform)
__global__ void pair_clean_flags_kernel(int64_t nunits, const int32_t *__restrict__ dpat, const int32_t *__restrict__ bfl,
                                        int32_t *__restrict__ pblk) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits || !(dpat[2 * u] & DPAT_PAIR)) return;
  pblk[u] = (int32_t)((uint32_t)pblk[u] | (uint32_t)bfl[(uint32_t)pblk[u] & PBLK_ID]);
}

// Select-free ("clean") rule of one 5/7-point row-pair block given its
// slot-row presence masks pm[0 .. 2K): every absent slot's operand can be made
// exactly 0.0 by an out-of-range read -- a run whose slot-rows are empty for
// both rows, or the tri run's edge value when only lane 0 row 0 lacks -1 /
// lane 63 row 1 lacks +1 -- so no presence select is needed.  f: the flags
// (PBLK_RUN0 << r, PBLK_ELO / EHI) the z-march kernels read from pblk.
static bool pair_block_clean(int ps, int K, const unsigned long long *pm, uint32_t &f) {
  const unsigned long long F = ~0ull;
  f = 0;
  const int NR = ps == 5 ? 3 : 5;
  for (int r = 0; r < NR; ++r) {
    const bool tri = ps == 5 ? r == 1 : r == 2;
    const int j = ps == 5 ? (r == 0 ? 0 : r == 1 ? 1 : 4) : (r < 2 ? r : r == 2 ? 2 : r + 2);
    if (!tri) {
      const unsigned long long a = pm[j], c = pm[K + j];
      if (a == 0 && c == 0) f |= PBLK_RUN0 << r;
      else if (a != F || c != F) return false;
      continue;
    }
    const unsigned long long m0 = pm[j], m1 = pm[j + 1], m2 = pm[j + 2];
    const unsigned long long n0 = pm[K + j], n1 = pm[K + j + 1], n2 = pm[K + j + 2];
    if ((m0 | m1 | m2 | n0 | n1 | n2) == 0) { f |= (PBLK_RUN0 << r) | PBLK_ELO | PBLK_EHI; continue; }
    if (m1 != F || m2 != F || n0 != F || n1 != F) return false;
    if (m0 != F && m0 != (F & ~1ull)) return false;
    if (n2 != F && n2 != (F >> 1)) return false;
    if (m0 != F) f |= PBLK_ELO;
    if (n2 != F) f |= PBLK_EHI;
  }
  return true;
}

// Uniform-slot form of the code-block dictionary (Sell::puni), 5/7-point
// shapes: kept only when, in every block, each slot-row's present codes are
// one code (constant-coefficient stencils: a few dozen boundary classes).
static void build_pair_uniform(Sell &S, const std::vector<double> &vt, hipStream_t st) {
  S.puni.reset();
  S.pair_clean = false;
  const int K = S.dia_k;
  if (S.pair_blocks <= 0 || (S.pair_shape != 5 && S.pair_shape != 7) || K != S.pair_shape || 2 * K > 16) return;
  const int pb = pair_bytes(K);
  const int64_t nb = S.pair_blocks;
  std::vector<uint8_t> d((size_t)nb * 64 * pb);
  HIPCHECK(hipMemcpyAsync(d.data(), S.pcode.p, d.size(), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  std::vector<PairUni> u((size_t)nb);
  for (int64_t b = 0; b < nb; ++b) {
    PairUni &B = u[(size_t)b];
    std::memset(&B, 0, sizeof(B));
    for (int q = 0; q < 2 * K; ++q) {
      int code = -1;
      for (int lane = 0; lane < 64; ++lane) {
        const int c = d[((size_t)b * 64 + lane) * pb + q];
        if (c == VCODE_ABSENT) continue;
        if (code >= 0 && c != code) return;       // two values in one slot-row: not uniform
        code = c;
        B.pm[q] |= 1ull << lane;
      }
      if (code >= 0) B.v[q] = vt[(size_t)code];
    }
    for (int lane = 0; lane < 64; ++lane) {
      uint32_t w = 0;
      for (int q = 0; q < 2 * K; ++q) w |= (uint32_t)((B.pm[q] >> lane) & 1ull) << q;
      B.lane[lane] = w;
    }
  }
  S.puni.alloc((size_t)nb);
  HIPCHECK(hipMemcpyAsync(S.puni.p, u.data(), sizeof(PairUni) * u.size(), hipMemcpyHostToDevice, st));
  // select-free form (mx_spmv_pair.hip): every absent slot's operand can be
  // made exactly 0.0 by an out-of-range read -- a run whose slot-rows are
  // empty for both rows, or the tri run's edge value when only lane 0 row 0
  // lacks -1 / lane 63 row 1 lacks +1 -- so no presence select is needed
  std::vector<int32_t> fl((size_t)nb, 0);
  bool clean = true;
  for (int64_t b = 0; b < nb && clean; ++b) {
    uint32_t f = 0;
    clean = pair_block_clean(S.pair_shape, K, u[(size_t)b].pm, f);
    fl[(size_t)b] = (int32_t)f;
  }
  S.pair_clean = clean && S.nunits > 0;
  if (S.pair_clean) {
    DBuf<int32_t> fd((size_t)nb);
    HIPCHECK(hipMemcpyAsync(fd.p, fl.data(), sizeof(int32_t) * fl.size(), hipMemcpyHostToDevice, st));
    pair_clean_flags_kernel<<<(unsigned)cdiv(S.nunits, 256), 256, 0, st>>>(S.nunits, S.dpat.p, fd.p, S.pblk.p);
    HIPCHECK(hipGetLastError());
  }
  HIPCHECK(hipStreamSynchronize(st));
}

// Select-free flags of a non-uniform code dictionary (Sell::pair_code_clean):
// the coded z-march (mx_spmv_pair.hip spmv_pair_zmc_kernel) reads each unit's
// code block and looks its values up in LDS, an absent slot's code giving the
// table's 0.0 and its operand made 0.0 by the same out-of-range reads as the
// uniform form, so it needs these flags in pblk and no presence select.
static void build_pair_code_clean(Sell &S, hipStream_t st) {
  S.pair_code_clean = false;
  const int K = S.dia_k;
  if (S.puni.p || S.pair_blocks <= 0 || (S.pair_shape != 5 && S.pair_shape != 7) || K != S.pair_shape || 2 * K > 16)
    return;
  const int pb = pair_bytes(K);
  const int64_t nb = S.pair_blocks;
  std::vector<uint8_t> d((size_t)nb * 64 * pb);
  HIPCHECK(hipMemcpyAsync(d.data(), S.pcode.p, d.size(), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  std::vector<int32_t> fl((size_t)nb, 0);
  for (int64_t b = 0; b < nb; ++b) {
    unsigned long long pm[16] = {};
    for (int q = 0; q < 2 * K; ++q)
      for (int lane = 0; lane < 64; ++lane)
        if (d[((size_t)b * 64 + lane) * pb + q] != VCODE_ABSENT) pm[q] |= 1ull << lane;
    uint32_t f = 0;
    if (!pair_block_clean(S.pair_shape, K, pm, f)) return;
    fl[(size_t)b] = (int32_t)f;
  }
  if (S.nunits <= 0) return;
  DBuf<int32_t> fd((size_t)nb);
  HIPCHECK(hipMemcpyAsync(fd.p, fl.data(), sizeof(int32_t) * fl.size(), hipMemcpyHostToDevice, st));
  pair_clean_flags_kernel<<<(unsigned)cdiv(S.nunits, 256), 256, 0, st>>>(S.nunits, S.dpat.p, fd.p, S.pblk.p);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));
  S.pair_code_clean = true;
}

// 27-point uniform-slot dictionary (Sell::puni27): kept when every block's
// 54 slot-rows are uniform; each block also gets its select-free flags (runs
// empty for both rows, and the x-line edges, which the nine runs of a
// regular grid share).
static void build_pair_uniform27(Sell &S, const std::vector<double> &vt, hipStream_t st) {
  S.puni27.reset();
  S.pair_clean27 = false;
  S.pair_unit27 = false;
  const int K = 27;
  if (S.pair_blocks <= 0 || S.pair_shape != 27 || S.dia_k != 27) return;
  const int pb = pair_bytes(K);
  const int64_t nb = S.pair_blocks;
  std::vector<uint8_t> d((size_t)nb * 64 * pb);
  HIPCHECK(hipMemcpyAsync(d.data(), S.pcode.p, d.size(), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  std::vector<PairUni27> u((size_t)nb);
  const unsigned long long F = ~0ull;
  bool all_clean = true;
  for (int64_t b = 0; b < nb; ++b) {
    PairUni27 &B = u[(size_t)b];
    std::memset(&B, 0, sizeof(B));
    for (int q = 0; q < 2 * K; ++q) {
      int code = -1;
      for (int lane = 0; lane < 64; ++lane) {
        const int c = d[((size_t)b * 64 + lane) * pb + q];
        if (c == VCODE_ABSENT) continue;
        if (code >= 0 && c != code) return;         // two values in one slot-row: not uniform
        code = c;
        B.pm[q] |= 1ull << lane;
      }
      if (code >= 0) B.v[q] = vt[(size_t)code];
    }
    // one value per slot for both rows (the lean kernel reads 27, not 54):
    // the rows of a regular-grid block share their stencil values; a block
    // whose rows differ keeps the general kernel
    for (int j = 0; j < K; ++j) {
      if (B.pm[j] && B.pm[K + j] && std::memcmp(&B.v[j], &B.v[K + j], sizeof(double)) != 0) return;
      if (!B.pm[j]) B.v[j] = B.v[K + j];
      B.v[K + j] = B.v[j];
    }
    for (int lane = 0; lane < 64; ++lane) {
      unsigned long long w = 0;
      for (int j = 0; j < 2 * K; ++j) w |= ((B.pm[j] >> lane) & 1ull) << j;
      B.lane[lane] = w;
    }
    uint32_t f = 0;
    int elo = -1, ehi = -1;                         // every non-empty run must agree
    bool clean = true;
    for (int r = 0; r < 9 && clean; ++r) {
      const int j = 3 * r;
      const unsigned long long m0 = B.pm[j], m1 = B.pm[j + 1], m2 = B.pm[j + 2];
      const unsigned long long n0 = B.pm[K + j], n1 = B.pm[K + j + 1], n2 = B.pm[K + j + 2];
      if ((m0 | m1 | m2 | n0 | n1 | n2) == 0) { f |= 1u << r; continue; }
      if (m1 != F || m2 != F || n0 != F || n1 != F) { clean = false; break; }
      if (m0 != F && m0 != (F & ~1ull)) { clean = false; break; }
      if (n2 != F && n2 != (F >> 1)) { clean = false; break; }
      const int lo = m0 != F, hi = n2 != F;
      if ((elo >= 0 && elo != lo) || (ehi >= 0 && ehi != hi)) { clean = false; break; }
      elo = lo;
      ehi = hi;
    }
    if (elo == 1) f |= U27_ELO;
    if (ehi == 1) f |= U27_EHI;
    B.flags = f;
    B.clean = clean ? 1u : 0u;
    all_clean = all_clean && clean;
  }
  // slot values -1 / 0 / +1 off the diagonal (slot 13): exact products
  bool unit = true;
  for (int64_t b = 0; b < nb && unit; ++b)
    for (int j = 0; j < K && unit; ++j)
      if (j != 13 && u[(size_t)b].v[j] != -1.0 && u[(size_t)b].v[j] != 0.0 && u[(size_t)b].v[j] != 1.0) unit = false;
  S.puni27.alloc((size_t)nb);
  HIPCHECK(hipMemcpyAsync(S.puni27.p, u.data(), sizeof(PairUni27) * u.size(), hipMemcpyHostToDevice, st));
  HIPCHECK(hipStreamSynchronize(st));
  S.pair_clean27 = all_clean;
  S.pair_unit27 = unit;
}

// Column words of a clean 27-point layout (Sell::pcol27), when the units'
// empty runs and x-line edges follow the plane / column rule exactly: unit u =
// (plane z, column c) must have empty runs = z-boundary runs (z = 0: runs 0-2,
// z = NZ - 1: runs 6-8) | the column's y-boundary runs (dy = -1: runs 0, 3, 6;
// dy = +1: 2, 5, 8) and the column's ELO / EHI.  Otherwise none is built.
static void build_pair_col27(Sell &S, int64_t m, hipStream_t st) {
  S.pcol27.reset();
  S.pair_2l27 = false;
  S.pair_4l27 = false;
  S.pair_sym27 = false;
  if (!S.puni27.p || !S.pair_clean27 || !S.pair_all || S.pat_star_off.size() < 27) return;
  const int64_t D = S.pat_star_off[22];                   // run 7's centre: +D
  if (D <= 0 || D % 128 != 0 || m % D != 0 || m > (int64_t(1) << 27)) return;
  const int64_t P = D / 128, NZ = m / D;
  const int64_t nb = S.pair_blocks;
  std::vector<PairUni27> blk((size_t)nb);
  std::vector<int32_t> pb((size_t)S.nunits);
  HIPCHECK(hipMemcpyAsync(blk.data(), S.puni27.p, sizeof(PairUni27) * nb, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(pb.data(), S.pblk.p, sizeof(int32_t) * S.nunits, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  std::vector<int32_t> cw((size_t)P, -1);
  const uint32_t RUNS = 0x1ffu, EDGES = U27_ELO | U27_EHI;
  for (int64_t u = 0; u < S.nunits; ++u) {
    const int64_t z = u / P, c = u % P;
    const uint32_t f = blk[(size_t)(pb[(size_t)u] & (int32_t)PBLK_ID)].flags;
    const uint32_t zb = (z == 0 ? 0x007u : 0u) | (z == NZ - 1 ? 0x1c0u : 0u);
    // the y status from the plane's own runs (dz = 0: runs 3 / 5, never z-boundary runs)
    uint32_t w = (f & EDGES) | ((f & (1u << 3)) ? U27C_YLO : 0u) | ((f & (1u << 5)) ? U27C_YHI : 0u);
    const uint32_t ys = ((w & U27C_YLO) ? 0x049u : 0u) | ((w & U27C_YHI) ? 0x124u : 0u);
    if ((f & RUNS) != (zb | ys)) return;                   // an empty run off the rule
    if (cw[(size_t)c] >= 0 && (uint32_t)cw[(size_t)c] != w) return;   // the column disagrees with itself
    cw[(size_t)c] = (int32_t)w;
  }
  // line groups for the G-line z-march (Sell::pair_2l27 / pair_4l27): in each
  // group of G lines the columns at one x share their edge words, and only
  // the first line may have a dy = -1 boundary, only the last a dy = +1 one
  auto groups = [&](int64_t G) {
    const int64_t nl = S.pat_star_off[16];               // run 5's centre: +n
    bool ok = nl > 0 && nl % 128 == 0 && D % nl == 0 && (D / nl) % G == 0;
    const int64_t PL = ok ? nl / 128 : 1;
    for (int64_t c = 0; ok && c < P; ++c) {
      const int64_t k = (c / PL) % G, c0 = c - k * PL;   // line k of its group; the group's first column
      const uint32_t wa = (uint32_t)cw[(size_t)c], w0 = (uint32_t)cw[(size_t)c0];
      if ((wa & EDGES) != (w0 & EDGES) || (k > 0 && (wa & U27C_YLO)) || (k < G - 1 && (wa & U27C_YHI))) ok = false;
    }
    return ok;
  };
  S.pair_2l27 = groups(2);
  S.pair_4l27 = groups(4);
  S.pcol27.alloc((size_t)P);
  HIPCHECK(hipMemcpyAsync(S.pcol27.p, cw.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, st));
  HIPCHECK(hipStreamSynchronize(st));
  // symmetry (Sell::pair_sym27): one value per off-diagonal slot over every
  // block's present slots, and that value equal to the mirrored slot's
  double V[27];
  bool have[27] = {};
  bool sym = true;
  for (int64_t b = 0; b < nb && sym; ++b)
    for (int j = 0; j < 27 && sym; ++j) {
      if (j == 13 || !(blk[(size_t)b].pm[j] | blk[(size_t)b].pm[27 + j])) continue;
      const double v = blk[(size_t)b].v[j];
      if (!have[j]) { V[j] = v; have[j] = true; }
      else if (std::memcmp(&V[j], &v, sizeof(double)) != 0) sym = false;
    }
  for (int j = 0; j < 27 && sym; ++j)
    if (j != 13 && have[j] != have[26 - j]) sym = false;
    else if (j != 13 && have[j] && std::memcmp(&V[j], &V[26 - j], sizeof(double)) != 0) sym = false;
  S.pair_sym27 = sym;
}

// The value dictionary's open-addressing table, set up before the diagonal
// block's SELL fill, which collects the aligned-offset slices' values into it
struct VDict {
  DBuf<unsigned long long> tab;
  DBuf<int> stat;
  bool dia_done = false;   // sell_fill_dia_kernel inserted the aligned-offset slices' values
  void init(hipStream_t st) {
    tab.alloc(VDICT_SLOTS);
    stat.alloc(2);
    const std::vector<unsigned long long> th(VDICT_SLOTS, VDICT_EMPTY);
    HIPCHECK(hipMemcpyAsync(tab.p, th.data(), sizeof(unsigned long long) * VDICT_SLOTS, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemsetAsync(stat.p, 0, 2 * sizeof(int), st));
    HIPCHECK(hipStreamSynchronize(st));   // th is freed on return
  }
};

static void build_value_codes(Sell &S, const int32_t *wid_o, int64_t m, int64_t ncols, hipStream_t st, VDict &vd) {
  S.ntab = 0;
  if (S.slots == 0 || !g_knobs.vcodes || !vd.tab.p) return;
  DBuf<unsigned long long> &tab = vd.tab;
  DBuf<int> &stat = vd.stat;
  std::vector<unsigned long long> th(VDICT_SLOTS, VDICT_EMPTY);
  if (!vd.dia_done || S.dia_slices < S.nslices)
    vdict_insert_kernel<<<(unsigned)cdiv(S.nslices, 4), 256, 0, st>>>(S.nslices, S.sptr.p, S.width.p, S.col.p, S.val.p,
                                                                    S.mask.p, S.mask8.p, tab.p, stat.p, vd.dia_done ? 1 : 0);
  HIPCHECK(hipGetLastError());
  int sh[2];
  HIPCHECK(hipMemcpyAsync(sh, stat.p, sizeof(sh), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  if (sh[1] || sh[0] > VCODE_ABSENT || sh[0] == 0) return;
  HIPCHECK(hipMemcpyAsync(th.data(), tab.p, sizeof(unsigned long long) * VDICT_SLOTS, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  std::vector<unsigned long long> keys;
  for (unsigned long long k : th)
    if (k != VDICT_EMPTY) keys.push_back(k);
  std::sort(keys.begin(), keys.end());
  std::vector<double> vt(VCODE_MAX, 0.0);
  for (size_t i = 0; i < keys.size(); ++i) std::memcpy(&vt[i], &keys[i], sizeof(double));
  const int64_t ns = S.nslices;
  S.cptr.alloc((size_t)ns);
  code_bytes_kernel<<<(unsigned)cdiv(ns, 256), 256, 0, st>>>(ns, S.width.p, S.cptr.p);
  HIPCHECK(hipGetLastError());
  exclusive_scan_i64(S.cptr.p, S.cptr.p, ns, st, &S.code_bytes);
  S.code.alloc((size_t)std::max<int64_t>(S.code_bytes, 8));
  S.vtab.alloc(VCODE_MAX);
  HIPCHECK(hipMemcpyAsync(S.vtab.p, vt.data(), sizeof(double) * vt.size(), hipMemcpyHostToDevice, st));
  {
    // jacobi_setup_kernel's dinv = d == 0 ? 1 : 1 / d, per code (IEEE division,
    // the same correctly rounded quotient on the host); absent -> 1
    std::vector<double> dt(VCODE_MAX, 1.0);
    for (size_t i = 0; i < keys.size(); ++i) dt[i] = vt[i] == 0.0 ? 1.0 : 1.0 / vt[i];
    S.dtab.alloc(VCODE_MAX);
    HIPCHECK(hipMemcpyAsync(S.dtab.p, dt.data(), sizeof(double) * dt.size(), hipMemcpyHostToDevice, st));
  }
  // row pairs read the operand through buffer loads with 32-bit byte offsets
  S.pair_shape = g_knobs.spmv_pairs && S.pat_star >= 0 && m < PAIR_MAX_ROWS && ncols < PAIR_MAX_ROWS
                     ? pair_shape_of(S.pat_star_off) : 0;
  DBuf<int8_t> pmd;
  DBuf<uint8_t> pkd;
  if (S.pair_shape) {
    S.nunits = ns / 2;
    S.pcode.alloc((size_t)std::max<int64_t>(S.nunits, 1) * 64 * pair_bytes(S.dia_k));
    if (S.nunits) {
      // per pattern: where each dominant slot sits in it, and whether its
      // offsets are all dominant ones (code_pair_fill_kernel)
      const int64_t np = S.npat;
      if ((int64_t)S.pat_len.size() != np) fail(MX_ERR_INTERNAL, "row pairs without shared offset patterns");
      std::vector<int8_t> pm((size_t)np * DIA_MAX, -1);
      std::vector<uint8_t> pk((size_t)np, 0);
      const int32_t *so = S.pat_host.data() + (size_t)S.pat_star * DIA_MAX;
      for (int64_t p = 0; p < np; ++p) {
        const int32_t *po = S.pat_host.data() + (size_t)p * DIA_MAX;
        const int len = S.pat_len[(size_t)p];
        bool ok = true;
        for (int q = 0; q < len; ++q) {
          int at = -1;
          for (int j = 0; j < S.dia_k; ++j)
            if (so[j] == po[q]) at = j;
          if (at < 0) ok = false;
          else pm[(size_t)p * DIA_MAX + at] = (int8_t)q;
        }
        pk[(size_t)p] = ok ? 1 : 0;
      }
      pmd.alloc(pm.size());
      pkd.alloc(pk.size());
      HIPCHECK(hipMemcpyAsync(pmd.p, pm.data(), pm.size(), hipMemcpyHostToDevice, st));
      HIPCHECK(hipMemcpyAsync(pkd.p, pk.data(), pk.size(), hipMemcpyHostToDevice, st));
      HIPCHECK(hipStreamSynchronize(st));   // pm / pk are freed at the end of this block
    }
  }
  code_pair_fill_kernel<<<(unsigned)cdiv(ns, 2), 128, 0, st>>>(
      m, ns, S.sptr.p, S.width.p, S.col.p, S.val.p, S.cptr.p,
      reinterpret_cast<const unsigned long long *>(S.vtab.p), (int)keys.size(), S.mask.p, S.mask8.p, S.code.p,
      S.pair_shape ? S.nunits : 0, S.dia_k, S.dpat.p, pmd.p, pkd.p, S.pair_shape && S.nunits ? S.pcode.p : nullptr);
  HIPCHECK(hipGetLastError());
  if (S.pair_shape) {
    HIPCHECK(hipGetLastError());
    {
      DBuf<unsigned long long> cnt(1);
      HIPCHECK(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long), st));
      pair_count_kernel<<<(unsigned)cdiv(std::max<int64_t>(S.nunits, 1), 256), 256, 0, st>>>(S.nunits, S.dpat.p, cnt.p);
      HIPCHECK(hipGetLastError());
      unsigned long long hc = 0;
      HIPCHECK(hipMemcpyAsync(&hc, cnt.p, sizeof(hc), hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      S.pair_used = (int64_t)hc;
    }
    dedupe_pair_blocks(S, st);
    build_pair_uniform(S, vt, st);
    build_pair_code_clean(S, st);
    build_pair_uniform27(S, vt, st);
    S.pair_ghosts = false;
    if (wid_o && S.nunits) {
      DBuf<int> any(1);
      HIPCHECK(hipMemsetAsync(any.p, 0, sizeof(int), st));
      pair_ghost_flags_kernel<<<(unsigned)cdiv(S.nunits, 256), 256, 0, st>>>(S.nunits, ns, S.dpat.p, wid_o, S.pblk.p,
                                                                             any.p);
      HIPCHECK(hipGetLastError());
      int ha = 0;
      HIPCHECK(hipMemcpyAsync(&ha, any.p, sizeof(int), hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      S.pair_ghosts = ha != 0;
    }
    // every full unit a pair unit: SpMV reads no per-unit pattern word
    S.pair_all = S.pair_used == m / 128;
    if (g_knobs.pair_col27) build_pair_col27(S, m, st);
  }
  HIPCHECK(hipStreamSynchronize(st));   // the host tables are freed on return
  S.ntab = (int)keys.size();
}

static void build_sell(Sell &S, int64_t m, int64_t ncols, const int64_t *ptr, const int32_t *col,
                       const double *val, hipStream_t st, bool allow_dia, VDict *vd = nullptr) {
  S.nslices = cdiv(m, SLICE);
  const int64_t ns = S.nslices;
  S.width.alloc((size_t)std::max<int64_t>(ns, 1));
  S.sptr.alloc((size_t)std::max<int64_t>(ns, 1));
  S.doff.alloc((size_t)std::max<int64_t>(allow_dia ? ns * DIA_MAX : 1, 1));
  if (ns == 0) { S.slots = 0; S.mask.alloc(1); return; }
  if (!allow_dia) {   // an off-diagonal block with no entries (one rank): every width 0, nothing to fill
    int64_t nnz = 0;
    HIPCHECK(hipMemcpyAsync(&nnz, ptr + m, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (nnz == 0) {
      HIPCHECK(hipMemsetAsync(S.width.p, 0, sizeof(int32_t) * ns, st));
      HIPCHECK(hipMemsetAsync(S.sptr.p, 0, sizeof(int64_t) * ns, st));
      S.slots = 0;
      S.mask.alloc(1);
      S.col.alloc(1);
      S.val.alloc(1);
      S.dpat.alloc(1);
      return;
    }
  }
  slice_format_kernel<<<(unsigned)ns, 64, 0, st>>>(m, ptr, col, ns, allow_dia ? 1 : 0, S.width.p,
                                                              S.sptr.p, S.doff.p);
  HIPCHECK(hipGetLastError());
  std::vector<int32_t> wh;
  if (allow_dia) {
    wh.resize((size_t)ns);
    HIPCHECK(hipMemcpyAsync(wh.data(), S.width.p, sizeof(int32_t) * ns, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    S.dia_slices = 0;
    int64_t hist[DIA_MAX + 1] = {0};
    for (int32_t w : wh)
      if (w < 0) { S.dia_slices++; hist[-w]++; }
    S.dia_k = 0;
    int kmax = 0;
    for (int k = 1; k <= DIA_MAX; ++k) {
      if (hist[k] > hist[S.dia_k]) S.dia_k = k;
      if (hist[k]) kmax = k;
    }
    // presence masks: one byte per row when every aligned-offset slice has <= 8 offsets
    if (S.dia_slices && kmax <= 8 && g_knobs.mask8) S.mask8.alloc((size_t)ns * SLICE);
    else if (S.dia_slices) S.mask.alloc((size_t)ns * SLICE);
  }
  if (!S.mask.p) S.mask.alloc(1);
  exclusive_scan_i64(S.sptr.p, S.sptr.p, ns, st, &S.slots);
  // aligned-offset slices keep no columns (their offsets are in doff): a
  // diagonal block made only of such slices needs no column array
  S.col.alloc((size_t)std::max<int64_t>(S.dia_slices < ns ? S.slots : 0, 1));
  S.val.alloc((size_t)std::max<int64_t>(S.slots, 1));
  if (S.dia_slices < ns)
    sell_fill_lds_kernel<true><<<(unsigned)ns, 64, 0, st>>>(m, ptr, col, val, ns, S.sptr.p, S.width.p, S.doff.p, S.col.p,
                                                            S.val.p, S.mask.p, S.mask8.p);
  if (S.dia_slices)
    sell_fill_dia_kernel<<<(unsigned)ns, 256, 0, st>>>(m, ptr, col, val, ns, S.sptr.p, S.width.p, S.doff.p, S.val.p,
                                                       S.mask.p, S.mask8.p, vd ? vd->tab.p : nullptr,
                                                       vd ? vd->stat.p : nullptr);
  if (vd && S.dia_slices) vd->dia_done = true;
  HIPCHECK(hipGetLastError());
  if (S.dia_slices) share_offset_patterns(S, wh, ncols, st);
  else S.dpat.alloc(1);
}

// ---------------------------------------------------------------- halo plan
static void build_halo(Mat *A) {
  Comm *c = A->comm;
  const int P = c->size;
  Halo &H = A->halo;
  std::vector<int64_t> want(P, 0), give(P, 0);
  // ghosts grouped by owning rank of the COLUMN layout (garray is sorted)
  std::vector<int64_t> off(P + 1, 0);
  {
    int q = 0;
    for (int64_t k = 0; k < A->nghost; ++k) {
      const int64_t g = A->garray_h[k];
      while (g >= A->cranges[q + 1]) ++q;
      want[q]++;
    }
    for (int q2 = 0; q2 < P; ++q2) off[q2 + 1] = off[q2] + want[q2];
  }
  if (want[c->rank] != 0) fail(MX_ERR_INTERNAL, "ghost owned by self");
  c->alltoall_i64(want.data(), give.data());
  std::vector<int32_t> req_h((size_t)std::max<int64_t>(A->nghost, 1));
  for (int q = 0; q < P; ++q)
    for (int64_t k = off[q]; k < off[q + 1]; ++k) req_h[k] = (int32_t)(A->garray_h[k] - A->cranges[q]);
  H.nrecv = A->nghost;
  H.nsend = 0;
  for (int q = 0; q < P; ++q) {
    if (want[q]) { H.recv_peer.push_back(q); H.recv_off.push_back(off[q]); H.recv_cnt.push_back(want[q]); }
    if (give[q]) { H.send_peer.push_back(q); H.send_off.push_back(H.nsend); H.send_cnt.push_back(give[q]); H.nsend += give[q]; }
  }
  DBuf<int32_t> req((size_t)std::max<int64_t>(A->nghost, 1));
  H.send_idx.alloc((size_t)std::max<int64_t>(H.nsend, 1));
  H.send_buf.alloc((size_t)std::max<int64_t>(H.nsend, 1));
  H.lvec.alloc((size_t)std::max<int64_t>(A->nghost, 1));
  if (A->nghost) HIPCHECK(hipMemcpyAsync(req.p, req_h.data(), sizeof(int32_t) * A->nghost, hipMemcpyHostToDevice, c->stream));
  std::vector<Msg> sends, recvs;
  for (size_t i = 0; i < H.recv_peer.size(); ++i)
    sends.push_back({H.recv_peer[i], req.p + H.recv_off[i], sizeof(int32_t) * (size_t)H.recv_cnt[i]});
  for (size_t i = 0; i < H.send_peer.size(); ++i)
    recvs.push_back({H.send_peer[i], H.send_idx.p + H.send_off[i], sizeof(int32_t) * (size_t)H.send_cnt[i]});
  c->exchange(sends, recvs);
  std::vector<int32_t> sidx((size_t)std::max<int64_t>(H.nsend, 1));
  if (H.nsend) HIPCHECK(hipMemcpyAsync(sidx.data(), H.send_idx.p, sizeof(int32_t) * H.nsend, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  H.need_pack = false;
  for (size_t i = 0; i < H.send_peer.size(); ++i) {
    const int32_t *s = sidx.data() + H.send_off[i];
    bool contig = true;
    for (int64_t k = 1; k < H.send_cnt[i]; ++k) if (s[k] != s[0] + k) { contig = false; break; }
    H.send_contig_start.push_back(contig ? s[0] : -1);
    if (!contig) H.need_pack = true;
  }
}

// ---------------------------------------------------------------- driver
static void layout(Comm *c, int64_t G, int64_t local, std::vector<int64_t> &ranges) {
  const int P = c->size;
  ranges.assign(P + 1, 0);
  if (local < 0) {
    const int64_t q = G / P, r = G % P;
    for (int i = 0; i < P; ++i) ranges[i + 1] = ranges[i] + q + (i < r ? 1 : 0);
  } else {
    std::vector<int64_t> all(P);
    c->allgather_i64(local, all.data());
    for (int i = 0; i < P; ++i) ranges[i + 1] = ranges[i] + all[i];
    if (ranges[P] != G)
      fail(MX_ERR_ARG, "Sum of local lengths " + std::to_string(ranges[P]) +
                           " does not equal global length " + std::to_string(G));
  }
}

thread_local AsmTimes g_asm_times;
double wall_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Mat *assemble(Comm *c, int64_t M, int64_t N, int64_t m_local, int64_t n_local,
              const AssemblyInput &in) {
  hipStream_t st = c->stream;
  const double t_start = wall_ms();
  std::unique_ptr<Mat> A(new Mat());
  A->comm = c;
  A->M = M; A->N = N;
  layout(c, M, m_local, A->rranges);
  layout(c, N, n_local, A->cranges);
  A->rstart = A->rranges[c->rank];
  A->m = A->rranges[c->rank + 1] - A->rstart;
  A->cstart = A->cranges[c->rank];
  A->cend = A->cranges[c->rank + 1];
  A->n = A->cend - A->cstart;
  const int64_t m = A->m;
  int64_t nnz = in.nnz;

  DBuf<int> err(1);
  HIPCHECK(hipMemsetAsync(err.p, 0, sizeof(int), st));

  // ---- group entries by row
  DBuf<int64_t> rowptr_own(kScratch), gcol(kScratch), gpos(kScratch);
  DBuf<double> gval(kScratch);
  const int64_t *rowptr = in.rowptr;
  const int64_t *col = in.cols;
  const int32_t *col32 = in.cols ? nullptr : in.cols32;   // read as is by the fused passes
  DBuf<int64_t> col_wide(kScratch);
  if (col32 && in.coo_rows) fail(MX_ERR_INTERNAL, "32-bit columns with COO input");
  const double *val = in.vals;
  const int64_t *pos = nullptr;
  DBuf<int64_t> rd_rows(kScratch), rd_cols(kScratch);
  DBuf<double> rd_vals(kScratch);
  AssemblyInput cin = in;
  if (in.coo_rows && c->size > 1) {   // off-process rows: stash exchange first
    cin.nnz = coo_redistribute(c, A->rranges, M, in.coo_rows, in.cols, in.vals, in.nnz, rd_rows, rd_cols, rd_vals);
    cin.coo_rows = rd_rows.p; cin.cols = rd_cols.p; cin.vals = rd_vals.p;
    nnz = cin.nnz;
  }
  if (cin.coo_rows) {
    const AssemblyInput &in = cin;
    DBuf<unsigned long long> cnt((size_t)m + 1, kScratch);
    HIPCHECK(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long) * (m + 1), st));
    if (nnz) {
      coo_count_kernel<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(nnz, in.coo_rows, in.cols, A->rstart, m, cnt.p, err.p);
      HIPCHECK(hipGetLastError());
    }
    rowptr_own.alloc((size_t)m + 1);
    int64_t total = 0;
    exclusive_scan_i64(reinterpret_cast<int64_t *>(cnt.p), rowptr_own.p, m + 1, st, &total);
    int herr = 0;
    HIPCHECK(hipMemcpy(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost));
    if (herr & 8) fail(MX_ERR_OUTOFRANGE, "Row out of range for this rank");
    HIPCHECK(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long) * (m + 1), st));
    gcol.alloc((size_t)std::max<int64_t>(total, 1));
    gval.alloc((size_t)std::max<int64_t>(total, 1));
    gpos.alloc((size_t)std::max<int64_t>(total, 1));
    if (nnz) {
      coo_scatter_kernel<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(nnz, in.coo_rows, in.cols, in.vals, A->rstart, m,
                                                                   rowptr_own.p, cnt.p, gcol.p, gval.p, gpos.p);
      HIPCHECK(hipGetLastError());
    }
    rowptr = rowptr_own.p; col = gcol.p; val = gval.p; pos = gpos.p;
  }


  // ---- longest row picks the segment width
  DBuf<unsigned long long> lmax(2);
  HIPCHECK(hipMemsetAsync(lmax.p, 0, sizeof(unsigned long long) * 2, st));
  if (m) {
    row_len_max_kernel<<<grid_for(m, 256, 2048), 256, 0, st>>>(m, rowptr, lmax.p, err.p);
    HIPCHECK(hipGetLastError());
  }
  unsigned long long Lh = 0;
  HIPCHECK(hipMemcpyAsync(&Lh, lmax.p, sizeof(Lh), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  int64_t tot_in = 0;
  if (m) HIPCHECK(hipMemcpy(&tot_in, rowptr + m, sizeof(int64_t), hipMemcpyDeviceToHost));

  const bool multi = c->size > 1;
  const int64_t nw = multi ? cdiv(N, 32) : 0;
  DBuf<unsigned> bitmap((size_t)std::max<int64_t>(nw, 1), kScratch);
  DBuf<int64_t> wbase((size_t)std::max<int64_t>(nw, 1), kScratch);
  if (nw) HIPCHECK(hipMemsetAsync(bitmap.p, 0, sizeof(unsigned) * nw, st));
  A->dptr.alloc((size_t)m + 1);
  A->optr.alloc((size_t)m + 1);
  HIPCHECK(hipMemsetAsync(A->dptr.p, 0, sizeof(int64_t) * (m + 1), st));
  HIPCHECK(hipMemsetAsync(A->optr.p, 0, sizeof(int64_t) * (m + 1), st));
  const int add = in.insert_mode == MX_ADD_VALUES;
  // segment width: the longest row's
  const int SW = Lh <= 8 ? 8 : Lh <= 16 ? 16 : Lh <= 32 ? 32 : 64;
  const unsigned sgrid = (unsigned)cdiv(std::max<int64_t>(m, 1), 256 / SW);
  const unsigned cgrid = (unsigned)cdiv(std::max<int64_t>(m, 1), 256 / SW * CANON_R);    // the fused count pass
  const unsigned fgrid = (unsigned)cdiv(std::max<int64_t>(m, 1), 256 / SW * CANON_FR);   // the fused fill pass
  const bool fused = Lh <= 64 && g_knobs.asm_fused;
  if (col32 && !fused) {   // the separate passes (and long rows) take 64-bit columns
    col_wide.alloc((size_t)std::max<int64_t>(tot_in, 1));
    if (tot_in) convert_index(col32, 4, tot_in, col_wide.p, st);
    col = col_wide.p;
    col32 = nullptr;
  }
  auto check_err = [&] {
    int herr = 0;
    HIPCHECK(hipMemcpyAsync(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (herr & 4) fail(MX_ERR_ARG, "row pointer array is not nondecreasing");
    if (herr & 1) fail(MX_ERR_OUTOFRANGE, "Column too large: max " + std::to_string(N - 1));
  };
  DBuf<int64_t> ccol(kScratch), cnt_out(kScratch);
  DBuf<double> cval(kScratch);
  double t_canon;
  if (fused) {
    // ---- canonicalise + split counts in one register pass (canon_count_kernel)
    // (no device synchronisation before it: round 5's in-process 8-rank
    // assemblies that read a few rows of columns as zeros were reading
    // through stale translations of freed contiguous allocations, retired in
    // round 6 -- mx_vec.hip; tools/asm_race.py 0 of 320)
    if (m) {
#define CCNT(WW) if (col32) canon_count_kernel<WW, int32_t><<<cgrid, 256, 0, st>>>(m, rowptr, col32, pos, N, add, A->cstart, A->cend, A->dptr.p, A->optr.p, bitmap.p, err.p); \
                 else canon_count_kernel<WW, int64_t><<<cgrid, 256, 0, st>>>(m, rowptr, col, pos, N, add, A->cstart, A->cend, A->dptr.p, A->optr.p, bitmap.p, err.p)
      switch (SW) { case 8: CCNT(8); break; case 16: CCNT(16); break; case 32: CCNT(32); break; default: CCNT(64); }
#undef CCNT
      HIPCHECK(hipGetLastError());
    }
    check_err();
    t_canon = wall_ms();
  } else {
    // ---- canonicalise rows
    ccol.alloc((size_t)std::max<int64_t>(tot_in, 1));
    cval.alloc((size_t)std::max<int64_t>(tot_in, 1));
    cnt_out.alloc((size_t)m + 1);
    DBuf<int64_t> long_rows((size_t)m + 1, kScratch);
    if (m) {
#define CANON(WW) canon_rows_wave_kernel<WW><<<sgrid, 256, 0, st>>>(m, rowptr, col, val, pos, N, add, ccol.p, cval.p, cnt_out.p, long_rows.p, &lmax.p[1], err.p)
      switch (SW) { case 8: CANON(8); break; case 16: CANON(16); break; case 32: CANON(32); break; default: CANON(64); }
#undef CANON
      HIPCHECK(hipGetLastError());
      if (Lh > 64) {
        unsigned long long nl = 0;
        HIPCHECK(hipMemcpyAsync(&nl, &lmax.p[1], sizeof(nl), hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        if (nl) {
          DBuf<int64_t> huge((size_t)nl);
          HIPCHECK(hipMemsetAsync(&lmax.p[0], 0, sizeof(unsigned long long), st));   // reused: huge-row count
          canon_rows_block_kernel<<<(unsigned)nl, 256, 0, st>>>(long_rows.p, rowptr, col, val, pos, N, add, ccol.p,
                                                                cval.p, cnt_out.p, err.p, huge.p, &lmax.p[0]);
          HIPCHECK(hipGetLastError());
          if (Lh > LONG_ROW_MAX) {
            unsigned long long nh = 0;
            HIPCHECK(hipMemcpyAsync(&nh, &lmax.p[0], sizeof(nh), hipMemcpyDeviceToHost, st));
            HIPCHECK(hipStreamSynchronize(st));
            std::vector<int64_t> hrows((size_t)nh);
            if (nh) HIPCHECK(hipMemcpy(hrows.data(), huge.p, sizeof(int64_t) * nh, hipMemcpyDeviceToHost));
            std::sort(hrows.begin(), hrows.end());
            canon_huge_rows(hrows, rowptr, col, val, pos, N, add, ccol.p, cval.p, cnt_out.p, err.p, st);
          }
        }
      }
    }
    check_err();
    t_canon = wall_ms();
    // ---- split counts + ghost bitmap
    if (m) {
#define SPLITC(WW) split_count_seg_kernel<WW><<<sgrid, 256, 0, st>>>(m, rowptr, cnt_out.p, ccol.p, A->cstart, A->cend, A->dptr.p, A->optr.p, bitmap.p)
      switch (SW) { case 8: SPLITC(8); break; case 16: SPLITC(16); break; case 32: SPLITC(32); break; default: SPLITC(64); }
#undef SPLITC
      HIPCHECK(hipGetLastError());
    }
  }
  // ---- split: row pointers, garray (bitmap popcount scan), A_d / A_o
  exclusive_scan_i64(A->dptr.p, A->dptr.p, m + 1, st, &A->nnz_d);
  exclusive_scan_i64(A->optr.p, A->optr.p, m + 1, st, &A->nnz_o);
  if (!multi && A->nnz_o) fail(MX_ERR_INTERNAL, "off-diagonal entries on one rank");
  A->nghost = 0;
  if (nw) {
    popc_kernel<<<grid_for(nw, 256, 8192), 256, 0, st>>>(nw, bitmap.p, wbase.p);
    HIPCHECK(hipGetLastError());
    exclusive_scan_i64(wbase.p, wbase.p, nw, st, &A->nghost);
  }
  A->garray.alloc((size_t)std::max<int64_t>(A->nghost, 1));
  if (A->nghost) {
    garray_kernel<<<grid_for(nw, 256, 8192), 256, 0, st>>>(nw, bitmap.p, wbase.p, A->garray.p);
    HIPCHECK(hipGetLastError());
  }
  A->dcol.alloc((size_t)std::max<int64_t>(A->nnz_d, 1));
  A->dval.alloc((size_t)std::max<int64_t>(A->nnz_d, 1));
  A->ocol.alloc((size_t)std::max<int64_t>(A->nnz_o, 1));
  A->oval.alloc((size_t)std::max<int64_t>(A->nnz_o, 1));
  A->diag.alloc((size_t)std::max<int64_t>(m, 1));
  if (m) {
    if (fused) {
#define CFILL_T(WW, T, CP) canon_fill_kernel<WW, T><<<fgrid, 256, 0, st>>>(m, rowptr, CP, val, pos, N, add, A->cstart, A->cend, A->rstart, A->dptr.p, A->optr.p, A->dcol.p, A->dval.p, A->ocol.p, A->oval.p, A->diag.p, bitmap.p, wbase.p)
#define CFILL(WW) if (col32) CFILL_T(WW, int32_t, col32); else CFILL_T(WW, int64_t, col)
      switch (SW) { case 8: CFILL(8); break; case 16: CFILL(16); break; case 32: CFILL(32); break; default: CFILL(64); }
#undef CFILL
#undef CFILL_T
    } else {
#define SPLITF(WW) fill_split_seg_kernel<WW><<<sgrid, 256, 0, st>>>(m, rowptr, cnt_out.p, ccol.p, cval.p, A->cstart, A->cend, A->rstart, A->dptr.p, A->optr.p, A->dcol.p, A->dval.p, A->ocol.p, A->oval.p, A->diag.p, bitmap.p, wbase.p)
      switch (SW) { case 8: SPLITF(8); break; case 16: SPLITF(16); break; case 32: SPLITF(32); break; default: SPLITF(64); }
#undef SPLITF
    }
    HIPCHECK(hipGetLastError());
  }
  A->garray_h.resize((size_t)A->nghost);
  if (A->nghost) HIPCHECK(hipMemcpyAsync(A->garray_h.data(), A->garray.p, sizeof(int64_t) * A->nghost, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  const double t_split = wall_ms();

  // ---- SpMV layouts
  VDict vd;
  if (g_knobs.vcodes && m) vd.init(st);
  build_sell(A->sd, m, A->n, A->dptr.p, A->dcol.p, A->dval.p, st, g_knobs.dia != 0, vd.tab.p ? &vd : nullptr);
  build_sell(A->so, m, A->nghost, A->optr.p, A->ocol.p, A->oval.p, st, false);
  build_value_codes(A->sd, A->so.nslices ? A->so.width.p : nullptr, m, A->n, st, vd);
  build_pair_f64(A->sd, m, A->n, A->so.nslices ? A->so.width.p : nullptr, st);
  build_cb(A.get(), st);   // unstructured blocks: the column-block MatMult
  A->partials.alloc((size_t)std::max(spmv_blocks(A.get()) + 64, RED_BLOCKS) * 4 + 64);
  HIPCHECK(hipStreamSynchronize(st));
  const double t_layout = wall_ms();

  // ---- halo plan (collective) + the slices that need ghosts
  if (multi) {
    build_halo(A.get());
    std::vector<int32_t> wo((size_t)A->so.nslices), lst;
    if (A->so.nslices)
      HIPCHECK(hipMemcpy(wo.data(), A->so.width.p, sizeof(int32_t) * A->so.nslices, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < A->so.nslices; ++k)
      if (wo[k] > 0) lst.push_back((int32_t)k);
    A->halo.nbnd = (int)lst.size();
    A->halo.bnd_slices.alloc(std::max<size_t>(lst.size(), 1));
    if (!lst.empty())
      HIPCHECK(hipMemcpy(A->halo.bnd_slices.p, lst.data(), sizeof(int32_t) * lst.size(), hipMemcpyHostToDevice));
  }
  const double t_end = wall_ms();
  g_asm_times.canon_ms = t_canon - t_start;
  g_asm_times.split_ms = t_split - t_canon;
  g_asm_times.layout_ms = t_layout - t_split;
  g_asm_times.halo_ms = t_end - t_layout;
  return A.release();
}

// ---------------------------------------------------------------- stencil generator
// Rows [row0, row0+m) of the synthetic operators of SURVEY.md §8d, written as
// a fixed-stride CSR (S slots per row, missing neighbours = column -1, which
// assembly ignores).  Values are dyadic, identical to oracle/petsc_oracle.c.
__device__ __forceinline__ double kappa_d(int64_t a, int64_t b, int64_t c) {
  int64_t t = ((a + 2 * b + 3 * c) % 4 + 4) % 4;
  return 1.0 + (double)t * 0.25;
}

// One thread per (row, slot), so a wave's stores are contiguous runs of the
// fixed-stride arrays (a thread per row wrote 27 strided doubles: 13.9 ms for
// a 27-point share, round 5).  Grid coordinates in 32-bit arithmetic when the
// global row count allows (I32), 64-bit otherwise; the values and the order of
// the diagonal's sum are the row kernel's.
template <int KIND, bool I32>
__global__ void stencil_kernel(int64_t nx, int64_t ny, int64_t nz, int64_t row0, int64_t m,
                               typename std::conditional<I32, int32_t, int64_t>::type *__restrict__ cols,
                               double *__restrict__ vals) {
  constexpr int S = KIND == 0 ? 5 : (KIND == 2 ? 27 : 7);
  const int64_t total = m * S;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t li = t / S;
    const int q = (int)(t - li * S);
    const int64_t row = row0 + li;
    int64_t i, j, k;
    if (I32) {
      const uint32_t r = (uint32_t)row, nx32 = (uint32_t)nx, ny32 = (uint32_t)ny;
      const uint32_t rest = r / nx32;
      i = r - rest * nx32;
      j = KIND == 0 ? rest : rest % ny32;
      k = KIND == 0 ? 0 : rest / ny32;
    } else {
      i = row % nx;
      j = (row / nx) % ny;
      k = KIND == 0 ? 0 : row / (nx * ny);
    }
    int di, dj, dk;
    if (KIND == 0) {
      di = q == 1 ? -1 : q == 3 ? 1 : 0;
      dj = q == 0 ? -1 : q == 4 ? 1 : 0;
      dk = 0;
    } else if (KIND == 2) {
      dk = q / 9 - 1;
      dj = (q / 3) % 3 - 1;
      di = q % 3 - 1;
    } else {
      di = q == 2 ? -1 : q == 4 ? 1 : 0;
      dj = q == 1 ? -1 : q == 5 ? 1 : 0;
      dk = q == 0 ? -1 : q == 6 ? 1 : 0;
    }
    const int64_t ii = i + di, jj = j + dj, kk = k + dk;
    const bool in = ii >= 0 && ii < nx && jj >= 0 && jj < ny && kk >= 0 && kk < nz;
    cols[t] = in ? ii + nx * (jj + ny * kk) : -1;   // 32-bit columns when the row count allows
    double v;
    if (KIND == 0) v = q == 2 ? 4.0 : -1.0;
    else if (KIND == 1) v = q == 3 ? 6.0 : -1.0;
    else if (KIND == 2) v = q == 13 ? 26.0 : -1.0;
    else if (q == 3)
      v = kappa_d(i - 1, j, k) + kappa_d(i, j, k) + kappa_d(i, j - 1, k) + kappa_d(i, j, k) +
          kappa_d(i, j, k - 1) + kappa_d(i, j, k) + 0.5;
    else {
      v = -kappa_d(i < ii ? i : ii, j < jj ? j : jj, k < kk ? k : kk);
      if (q == 2) v = v - 0.5;
    }
    vals[t] = v;
  }
}

__global__ void stride_rowptr_kernel(int64_t m, int S, int64_t *__restrict__ rowptr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= m; i += stride) rowptr[i] = i * S;
}

// Columns go to `cols32` (4 B an entry, read as is by the fused assembly
// passes) when the global row count fits 31 bits, else to `cols`.
void stencil_coo(Comm *c, int kind, int64_t nx, int64_t ny, int64_t nz, int64_t row0, int64_t m,
                 DBuf<int64_t> &rowptr, DBuf<int64_t> &cols, DBuf<int32_t> &cols32, DBuf<double> &vals) {
  const int S = kind == 0 ? 5 : (kind == 2 ? 27 : 7);
  const bool i32 = (kind == 0 ? nx * ny : nx * ny * nz) < ((int64_t)1 << 31);
  rowptr.alloc((size_t)m + 1);
  if (i32) cols32.alloc((size_t)std::max<int64_t>(m * S, 1));
  else cols.alloc((size_t)std::max<int64_t>(m * S, 1));
  vals.alloc((size_t)std::max<int64_t>(m * S, 1));
  stride_rowptr_kernel<<<grid_for(m + 1, 256, 8192), 256, 0, c->stream>>>(m, S, rowptr.p);
  HIPCHECK(hipGetLastError());
  if (m) {
    const unsigned g = grid_for(m * S, 256, 65536);
#define STK(K) if (i32) stencil_kernel<K, true><<<g, 256, 0, c->stream>>>(nx, ny, nz, row0, m, cols32.p, vals.p); \
               else stencil_kernel<K, false><<<g, 256, 0, c->stream>>>(nx, ny, nz, row0, m, cols.p, vals.p)
    switch (kind) { case 0: STK(0); break; case 1: STK(1); break; case 2: STK(2); break; default: STK(3); }
#undef STK
    HIPCHECK(hipGetLastError());
  }
}

// this translation unit's code object, loaded now rather than at the first
// launch of one of its kernels (load_code_objects)
void load_code_assembly() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&row_len_max_kernel));
  (void)hipGetLastError();
}

}  // namespace mx
