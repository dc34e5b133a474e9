// mx_internal.hpp -- shared internals of libmxsolve.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mxsolve.h"

namespace mx {

// ---------------------------------------------------------------- errors
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void fail(int code, const std::string &msg);
void hip_check(hipError_t e, const char *what, const char *file, int line);
#define HIPCHECK(x) ::mx::hip_check((x), #x, __FILE__, __LINE__)

// ---------------------------------------------------------------- device buffers
// hipMalloc (library-owned arrays)
hipError_t dev_malloc(void **p, size_t bytes);
// Transient (scratch) buffers of one call.  Buffers of 1 MiB or more of either
// kind come from / go back to a small per-device cache instead of hipMalloc /
// hipFree (dev_free; scratch_trim empties the cache; mx_vec.hip).
hipError_t scratch_malloc(void **p, size_t bytes);
void dev_free(void *p);
void scratch_trim();
struct ScratchTag {};
constexpr ScratchTag kScratch{};

// Owning device allocation (hipMalloc).  The library allocates matrix storage
// and solver work vectors itself; user vectors arrive as raw device pointers.
// DBuf(kScratch): a transient buffer of one call (scratch_malloc / scratch_free).
template <class T> struct DBuf {
  T *p = nullptr;
  size_t n = 0;
  bool scratch = false;
  DBuf() = default;
  explicit DBuf(ScratchTag) : scratch(true) {}
  explicit DBuf(size_t count) { alloc(count); }
  DBuf(size_t count, ScratchTag) : scratch(true) { alloc(count); }
  DBuf(const DBuf &) = delete;
  DBuf &operator=(const DBuf &) = delete;
  DBuf(DBuf &&o) noexcept : p(o.p), n(o.n), scratch(o.scratch) { o.p = nullptr; o.n = 0; }
  DBuf &operator=(DBuf &&o) noexcept {
    reset(); p = o.p; n = o.n; scratch = o.scratch; o.p = nullptr; o.n = 0; return *this;
  }
  ~DBuf() { reset(); }
  void alloc(size_t count) {
    reset();
    n = count;
    if (count) {
      void **q = reinterpret_cast<void **>(&p);
      hipError_t e = scratch ? scratch_malloc(q, count * sizeof(T)) : dev_malloc(q, count * sizeof(T));
      if (e != hipSuccess) { p = nullptr; n = 0; fail(MX_ERR_MEM, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed"); }
    }
  }
  void reset() {
    if (p) dev_free(p);
    p = nullptr; n = 0;
  }
  T *get() const { return p; }
};

// ---------------------------------------------------------------- communicator
struct Msg { int peer; void *buf; size_t bytes; };

// One rank's view of a communicator.  Device payloads move on `stream`.
struct Comm {
  int rank = 0, size = 1, device = 0;
  bool capturable = true;    // host-synchronous transports (LocalComm) cannot be graph-captured
  hipStream_t stream = nullptr;
  DBuf<double> red_scratch;  // scratch for reductions
  virtual ~Comm();
  // In-place SUM all-reduce of n doubles living in device memory, on stream.
  virtual void allreduce_sum(double *dev, int n) = 0;
  hipStream_t comm_stream = nullptr;  // halo exchange stream (overlaps the interior SpMV)
  // Grouped point-to-point exchange of device buffers, on stream `s` (default: stream).
  virtual void exchange(const std::vector<Msg> &sends, const std::vector<Msg> &recvs,
                        hipStream_t s = nullptr) = 0;
  // Host all-to-all of one int64 per peer (setup only; synchronous).
  virtual void alltoall_i64(const int64_t *send, int64_t *recv) = 0;
  // Host all-gather of one int64 per rank (setup only; synchronous).
  virtual void allgather_i64(int64_t v, int64_t *all) = 0;
  virtual void barrier() = 0;
  // Host waits for device work that may include this communicator's
  // collectives.  RCCL communicators poll the stream/event together with
  // ncclCommGetAsyncError under a deadline and abort the communicator
  // (MX_ERR_COMM) instead of hanging on a peer that never arrives.
  virtual void wait_stream(hipStream_t s) { HIPCHECK(hipStreamSynchronize(s ? s : stream)); }
  virtual void wait_event(hipEvent_t e) { HIPCHECK(hipEventSynchronize(e)); }
  // Host spins until ready() (a word the device writes into pinned host
  // memory) or until stream s has drained (then the caller re-reads the word);
  // a device error on s raises.  progress (optional): a count the device
  // advances -- RCCL communicators re-arm their no-progress deadline on it,
  // once it has moved off `baseline` (the count before the waited-for work
  // was enqueued): until then a peer may simply not have arrived yet, and the
  // plain wait deadline (knob 47) applies.
  virtual void wait_until(const std::function<bool()> &ready, hipStream_t s,
                          const std::function<long long()> &progress = {}, long long baseline = 0);
};

Comm *make_self_comm(int device);
Comm *make_rccl_comm(int rank, int size, int device, const void *uid, size_t len);
Comm *make_shm_comm(int rank, int size, int device, const char *name, int64_t slot_kib);
void abort_comm_async(Comm *c);   // mx_comm_abort: shared-memory world or RCCL communicator
void *make_local_world(int size);
Comm *make_local_comm(void *world, int rank, int device);
void destroy_local_world(void *world);
void abort_local_world(void *world);
void get_unique_id(void *out, size_t len);

// ---------------------------------------------------------------- matrix
constexpr int SLICE = 64;  // SELL-C with C = one wavefront

// SELL-64: slice s = rows [64 s, 64 s + 64), `width[s]` slots per row.
// Paired layout: entries (2p, 2p+1) of a row are adjacent, so a lane loads
// 16 B of values and 8 B of column ids per pair; an odd last entry sits in a
// trailing single region:  pair p at sptr + 128 p + 2 lane (+0/+1), tail at
// sptr + 128 (w/2) + lane.  Same slot count as plain SELL (entry j at
// sptr + 64 j + lane), which measured 9.5% slower.
//
// Aligned-offset slices ("DIA-in-SELL"): when the 64 rows of a slice use few
// distinct column offsets d = col - row (stencils: the stencil's offsets), the
// slice stores k slots per row at those offsets (sorted ascending = PETSc's
// column order), no column ids, and a per-row bitmask of the slots present.
// width[s] < 0 marks such a slice (k = -width[s]); the offsets live in
// doff[s * DIA_MAX + j].  Per row: 8 k + 4 bytes instead of 12 w.
constexpr int DIA_MAX = 32;
constexpr int32_t DPAT_INB = 1 << 30;
constexpr int32_t DPAT_PAIR = 1 << 29;   // on slice 2u: unit u is stored as row pairs
constexpr int32_t DPAT_ID = DPAT_PAIR - 1;
// one uniform-slot dictionary block (Sell::puni): slot-row q = slot q of
// row 0 (q < K) or slot q - K of row 1
struct PairUni {
  double v[16];                 // the slot-row's value
  unsigned long long pm[16];    // lanes whose row stores it
  // the masks transposed for the lean kernel's select body: lane l's bit q =
  // pm[q] bit l (one vector load per unit instead of 2K wave-uniform masks)
  uint32_t lane[64];
};
// the same for 27-point row pairs (54 slot-rows), with the block's select-free
// flags: bit r = run r empty for both rows, U27_ELO / U27_EHI = lane 0 row 0
// lacks every non-empty run's -1 entry / lane 63 row 1 its +1 entry
struct PairUni27 {
  double v[54];                 // v[j] == v[27 + j]: one value per slot (the build requires it)
  unsigned long long pm[54];
  uint32_t flags, clean;        // clean: the block needs no presence select
  uint32_t pad[2];
  // the masks transposed, for the select body: lane l's bit j = pm[j] bit l
  // (row 0), bit 27 + j = pm[27 + j] bit l (row 1) -- one vector load per unit
  // instead of 54 wave-uniform masks (which do not fit the SGPR file)
  unsigned long long lane[64];
};
constexpr uint32_t U27_ELO = 1u << 9;
constexpr uint32_t U27_EHI = 1u << 10;
constexpr uint32_t U27C_YLO = 1u << 0;   // Sell::pcol27: the column's dy = -1 runs are empty
constexpr uint32_t U27C_YHI = 1u << 1;   // ... dy = +1

struct Sell {
  int64_t nslices = 0, slots = 0, dia_slices = 0;
  int dia_k = 0;         // most common aligned-offset width (kernel specialisation)
  DBuf<int64_t> sptr;    // [nslices] slot offset of each slice
  DBuf<int32_t> width;   // [nslices]  (< 0: aligned-offset slice with k = -width)
  DBuf<int32_t> col;     // [slots], -1 = padding (unused for aligned-offset slices)
  DBuf<double> val;      // [slots]
  DBuf<int32_t> doff;    // [npat * DIA_MAX] the distinct offset patterns of aligned-offset slices
  DBuf<int32_t> dpat;    // [nslices] pattern of each aligned-offset slice (a stencil has a handful),
                         // | DPAT_INB when all of the slice's gathers are in range
  int64_t npat = 0;
  DBuf<uint32_t> mask;   // [nslices * 64] slot-present bits of aligned-offset rows
  DBuf<uint8_t> mask8;   // the same in one byte per row when every slice has <= 8 offsets
  // value codes (diagonal block): when the block holds at most VCODE_MAX
  // distinct values, code[cptr[s] + b * CODE_BATCH + 8 lane + q] is the index
  // into vtab of slot 8 b + q of the lane's row (one byte per slot instead of 8)
  int ntab = 0;          // 0: no codes
  int64_t code_bytes = 0;
  DBuf<uint8_t> code;
  DBuf<int64_t> cptr;    // [nslices] byte offset of each slice's code block
  DBuf<double> vtab;     // [ntab] the distinct values, ascending bit pattern
  // row-pair copy of the codes (mx_assembly.hip, pair_fill_kernel)
  int32_t pat_star = -1;              // the dominant pattern of width dia_k
  std::vector<int32_t> pat_star_off;
  std::vector<int32_t> pat_len;       // [npat] offsets per shared pattern (host copy; empty: per-slice lists)
  std::vector<int32_t> pat_host;      // [npat * DIA_MAX] the shared patterns (host copy)
  int pair_shape = 0;                 // 0, 5, 7, 27
  int64_t nunits = 0;
  DBuf<uint8_t> pcode;    // unit code blocks (64 * pair_bytes per unit), or the distinct ones
  // unit u's codes are block pblk[u] of pcode: u itself, or (pair_blocks > 0)
  // an index into the dictionary of the distinct blocks (a stencil has a few
  // dozen: boundary classes x value classes), which then stays in L2
  DBuf<int32_t> pblk;     // [nunits] | PBLK_GHOST_LO/HI: the unit's first/second slice has A_o entries
  int64_t pair_blocks = 0;
  int64_t pair_used = 0;   // units stored as row pairs
  bool pair_ghosts = false;  // some pair unit has A_o entries (SpMV then always splits)
  bool pair_all = false;     // every full unit is a pair unit
  // uniform-slot dictionary (5/7-point row pairs): every present code of a
  // block's slot-row is one value, so block b is puni[b] -- the 2K values and
  // the 2K lane masks of present slots -- read by scalar loads (no code bytes,
  // no LDS table lookups); empty when some block is not uniform
  DBuf<PairUni> puni;
  bool pair_clean = false;  // every puni block is select-free (PBLK_RUN0/ELO/EHI flags in pblk)
  DBuf<PairUni27> puni27;   // 27-point uniform-slot dictionary (mx_spmv_pair.hip z-march)
  // fp64 row pairs (uncoded 5/7-point layouts, any rank count): per unit u,
  // slot j, lane l the values of rows 128u + 2l and + 1 (0.0 where absent) as
  // one 16-byte pair at pval[(u * K + j) * 64 + l]; pflag[u] = the unit's
  // select-free flags (PBLK_RUN0 << r, PBLK_ELO / EHI) and, on P > 1 ranks,
  // PBLK_GHOST_LO / HI (the unit's first / second slice has A_o entries: the
  // product splits and the boundary kernel finishes those rows).  Built only
  // when every unit is select-free (mx_spmv_pair.hip spmv_pair_zmf64_kernel)
  DBuf<double> pval;
  DBuf<int32_t> pflag;
  int pair_f64 = 0;         // 5 / 7: the fp64 row-pair layout's shape, 0 none
  bool pair_clean27 = false;  // every puni27 block is select-free
  // every puni27 block's slot values but the diagonal's are -1, 0 or +1: the
  // 27-point z-march forms those slots' terms by fma (exact products, the same bits)
  bool pair_unit27 = false;
  // the column-word 27-point layout is symmetric: every block's off-diagonal
  // slot values are one value per slot across blocks and v[j] == v[26 - j]
  // (with the box-boundary presence of the column words, a_ij == a_ji): CG
  // mode 5's p.Ap pass sums each row's forward half (mx_spmv_pair.hip pair_fwd27)
  bool pair_sym27 = false;
  // the column words pair up by lines (knob 70, mx_spmv_pair.hip
  // spmv_pair_zm27p2l_kernel): whole 128-row columns per line, an even number
  // of lines per plane, and each even line's column and the next line's column
  // at the same x have equal edge words, no dy = +1 boundary on the first and
  // no dy = -1 boundary on the second
  bool pair_2l27 = false;
  bool pair_4l27 = false;   // the same by groups of four lines (knob 70 = 2)
  // 27-point column words (one per 128-row column of a plane): when every
  // unit's empty runs are exactly its plane's z-boundary runs (plane 0: dz =
  // -1, the last plane: dz = +1 -- read out of range anyway) plus its column's
  // y-boundary runs (U27C_YLO: dy = -1, U27C_YHI: dy = +1) and its x-line
  // edges are its column's (U27_ELO / U27_EHI), the z-march zeroes those
  // operands where it loads them (out-of-range reads) and needs neither
  // per-run branches nor selects (mx_spmv_pair.hip, form 2)
  DBuf<int32_t> pcol27;
  // 1 / value per code (1 for a zero value and for absent slots): PCJacobi's
  // dinv of a row is dtab[its diagonal slot's code] -- the division the
  // Jacobi setup does, so the Jacobi-fused row-pair MatMult reads no dinv
  // vector (the same bits)
  DBuf<double> dtab;
  // a non-uniform code dictionary (pair_blocks > 0, no puni) whose every block
  // is select-free: the flags are in pblk, and the coded z-march runs on it
  bool pair_code_clean = false;
  // column-block two-pass MatMult (mx_spmv_cb.hip) for unstructured blocks:
  // the entries in (column block of 2^cb_bs columns, row, column) order --
  // cb_col / cb_val, block b at [cb_bstart[b], cb_bstart[b+1]) -- the
  // products' buffer cb_prod in that order, and cb_perm: each SELL slot's
  // position in it (-1 padding); cb_nblk = 0: not built
  int cb_bs = 0, cb_nblk = 0;
  DBuf<int64_t> cb_bstart;
  DBuf<int32_t> cb_col, cb_perm;
  DBuf<double> cb_val, cb_prod;
};
constexpr uint32_t PBLK_GHOST_LO = 1u << 30;
constexpr uint32_t PBLK_GHOST_HI = 1u << 31;
// select-free ("clean") uniform-slot units: run r's slot-rows are empty for
// both rows (PBLK_RUN0 << r), lane 0 row 0 lacks the tri run's -1 entry
// (PBLK_ELO), lane 63 row 1 lacks its +1 entry (PBLK_EHI); mx_spmv_pair.hip
constexpr uint32_t PBLK_RUN0 = 1u << 22;
constexpr uint32_t PBLK_ELO = 1u << 27;
constexpr uint32_t PBLK_EHI = 1u << 28;
constexpr uint32_t PBLK_ID = PBLK_RUN0 - 1;   // block ids < 2^22 (units < 2^21, dictionaries <= 2048 blocks)
// the flag fields must not reach the ghost bits: runs 0..4 (RUN0 << 4), the edges
static_assert((PBLK_RUN0 << 4) < PBLK_ELO && PBLK_ELO < PBLK_EHI && PBLK_EHI < PBLK_GHOST_LO,
              "PBLK select-free flags overlap the ghost bits");
static_assert(((PBLK_RUN0 << 5) - PBLK_RUN0 | PBLK_ELO | PBLK_EHI | PBLK_ID) < PBLK_GHOST_LO, "PBLK field overlap");
constexpr int64_t PAIR_MAX_ROWS = int64_t(1) << 28;   // operand byte offsets (unsigned 32-bit voffset, bound n * 8 < 2^31)
constexpr int VCODE_MAX = 256;      // table entries; code 255 marks an absent slot
constexpr int VCODE_ABSENT = VCODE_MAX - 1;
constexpr int CODE_BATCH = 8 * SLICE;   // bytes per 8-slot batch of a slice
struct VCodes { const uint8_t *code; const int64_t *cptr; const double *tab; int ntab; };

// Runtime switches (mx_debug_set, include/mxsolve.h): the product path's
// defaults, and the alternatives the tests compare it with bit for bit.
// The settings measured and fixed in rounds 1-5 are compile-time constants
// (round 6: 37 keys retired; static members, so every `g_knobs.x` reads on).
struct Knobs {
  int overlap = 1; int graph = 1; int force_coll = 0; int cg_fuse = 3; int cg_vec = 0; int cg_unroll = 2;
  int vcodes = 1; int spmv_pairs = 1; int cg_xbatch = 0; int comm_timeout_ms = 120000;
  int pair_lean = 1; int pair_zm = 1; int pair_zm_bpc = 4; int pair_zm_len = 32; int spmv_fp64_grid = 8192;
  int comm_wait_ms = 600000; int pair_col27 = 1; int pair_zmc = 1; int pair_unitv = 1; int pw_sym27 = 1;
  int pair_zm27p = 1; int gm_stall_us = 0; int ru_2line = 3; int cg_pbw = 5; int zm27_2line = 1;
  int asm_fused = 1; int cg_pbws = 1; int scratch_cache = 1; int cb = 1;
  // fixed (the value each former key's A/B chose; DESIGN.md sections 4-11)
  static constexpr int spmv_nt = 1, spmv_grid = 0, dia = 1, jac_const = 1, cg_fold = 1, ws_skew = 0;
  static constexpr int cg_vec_grid = 0, cg_nts = 0, bnd_grid = 0, mask8 = 1, cg_upd_grid = 0, spmv_ynt = 0;
  static constexpr int spmv_bpc = 6, spmv_pair_bpc = 4, pdict = 1, cg_ntl = 3, norm_grid = 0, pair_uni = 1;
  static constexpr int mdot_grid = 0, pair_dtab = 1, pair_zm_units = 2, pair_f64 = 1, pair_zm27_bpc = 6;
  static constexpr int cg5_fold = 1, pair_zm27_units = 1, gm_pad = 256, cg5_27 = 1, pair_zm27_ru_bpc = 5;
  static constexpr int pw_bpc = 0, ru_bpc = 3, zm_balance = 1, zm27_xcol = 1, zm27_xcol_ru = 2, zm27_xcol_pw = 3;
  static constexpr int maxpy_grid = 0, zmc_units = 1, zmc_bpc = 0;
};
extern Knobs g_knobs;

struct Halo {
  // receive side: ghosts arrive grouped by owner, contiguous in lvec
  std::vector<int> recv_peer;
  std::vector<int64_t> recv_off, recv_cnt;
  // send side
  std::vector<int> send_peer;
  std::vector<int64_t> send_off, send_cnt;
  std::vector<int64_t> send_contig_start;  // >= 0: x + start is the payload (no pack)
  DBuf<int32_t> send_idx;                   // [nsend] local rows to pack
  DBuf<double> send_buf;                    // [nsend]
  DBuf<double> lvec;                        // [nghost]
  int64_t nsend = 0, nrecv = 0;
  bool need_pack = false;
  // slices with ghost entries: finished after the exchange (overlap)
  DBuf<int32_t> bnd_slices;
  int nbnd = 0;
  hipEvent_t ev_x = nullptr, ev_done = nullptr;
  ~Halo() {
    if (ev_x) (void)hipEventDestroy(ev_x);
    if (ev_done) (void)hipEventDestroy(ev_done);
  }
};

struct Mat {
  Comm *comm = nullptr;
  int64_t M = 0, N = 0, m = 0, n = 0, rstart = 0, cstart = 0, cend = 0;
  std::vector<int64_t> rranges, cranges;  // P+1 each
  // canonical PETSc MPIAIJ split (CSR)
  DBuf<int64_t> dptr, optr;
  DBuf<int32_t> dcol, ocol;
  DBuf<double> dval, oval, diag;
  DBuf<int64_t> garray;
  int64_t nnz_d = 0, nnz_o = 0, nghost = 0;
  std::vector<int64_t> garray_h;
  Sell sd, so;  // SELL-64 copies used by SpMV
  Halo halo;
  DBuf<double> partials;   // per-block reduction partials
  DBuf<double> scratch_x;  // helper vectors
  // KSPSetUp work vectors / device state, kept across solves with this operator
  DBuf<double> ksp_ws;
  DBuf<char> ksp_state;
  // PCSetUp_Jacobi result, computed once per assembled operator (KSPSetUp)
  DBuf<double> jac_dinv;
  int jac_mode = -1;       // -1: not set up; 1: vector; 2: uniform scalar
  double jac_c = 1.0;
  // A_d symmetric, entries and values (one rank, checked once by
  // pair_sym_prepare for CG mode 5's forward-half p.Ap pass): -1 not checked
  int sym = -1;
  // captured CG iteration batch (hipGraph), reused while its key matches
  hipGraphExec_t cg_graph = nullptr;
  std::vector<uintptr_t> cg_key;
  bool cg_graph_failed = false;     // capture failed once: this operator stays eager
  // per-solve host resources, created at the first solve and kept: the
  // pinned convergence-flag slots the host polls and the solve's timing
  // events (a pinned allocation per solve costs more than a short solve)
  int *poll_pinned = nullptr;
  void *state_pinned = nullptr;     // KspState staging for the host <-> device state copies
  hipEvent_t poll_ev[2] = {nullptr, nullptr};
  hipEvent_t solve_ev[2] = {nullptr, nullptr};
  void release_ksp();               // KSPReset: work space, state, graph, Jacobi setup
  ~Mat() { release_ksp(); }
};

// Phase times of this thread's last assembly (mx_debug_assembly_times): host
// wall clock between stream synchronisations, milliseconds.
struct AsmTimes {
  double h2d_ms = 0, canon_ms = 0, split_ms = 0, layout_ms = 0, halo_ms = 0, total_ms = 0;
  double alloc_ms = 0;     // device buffers of the copied input (within total, not within h2d)
  double host_bytes = 0;   // bytes read from host memory (createAIJ from host arrays)
};
extern thread_local AsmTimes g_asm_times;
double wall_ms();          // steady clock, milliseconds

// assembly entry (mx_assembly.hip)
struct AssemblyInput {
  // grouped input: rows [0, m), entries of row i at [rowptr[i], rowptr[i+1])
  // for CSR; for COO, `coo_rows` is set and rowptr is built internally.
  const int64_t *rowptr = nullptr;   // device, m+1 (CSR)
  const int64_t *coo_rows = nullptr; // device, nnz (COO, global rows)
  const int64_t *cols = nullptr;     // device, nnz (global cols)
  const int32_t *cols32 = nullptr;   // device, nnz: 32-bit global cols instead (CSR only, cols unset)
  const double *vals = nullptr;      // device, nnz
  int64_t nnz = 0;
  int insert_mode = MX_INSERT_VALUES;
};
Mat *assemble(Comm *c, int64_t M, int64_t N, int64_t m_local, int64_t n_local,
              const AssemblyInput &in);
void stencil_coo(Comm *c, int kind, int64_t nx, int64_t ny, int64_t nz, int64_t row0,
                 int64_t m, DBuf<int64_t> &rows, DBuf<int64_t> &cols, DBuf<int32_t> &cols32,
                 DBuf<double> &vals);
void convert_index(const void *src, int bytes, int64_t n, int64_t *dst, hipStream_t s);

// PCJacobi application z_i = r_i * d_i.  mode 0: no PC; 1: per-row d (HBM
// vector); 2: every diagonal entry equal, d is one scalar (bitwise the same
// products, 8 B/row less traffic per application).
struct Jac {
  const double *d = nullptr;
  double c = 1.0;
  int mode = 0;
};
__device__ __forceinline__ double papply(const Jac &J, double r, int64_t i) {
  return J.mode == 1 ? r * J.d[i] : (J.mode == 2 ? r * J.c : r);
}

// SpMV (mx_spmv.hip)
enum SpmvMode { SPMV_PLAIN = 0, SPMV_JACOBI = 1, SPMV_DOT = 2, SPMV_CG = 3,
                // the operand is s * x with s = *xscale: a GMRES basis vector kept
                // unnormalised (VecScale applied at every read, the same bits)
                SPMV_PLAIN_S = 4, SPMV_JACOBI_S = 5,
                // CG mode 5 (z-march only, one rank): the p.Ap partials without
                // storing the product, and the residual update that recomputes
                // it (mx_spmv_pair.hip spmv_pair_zm_kernel)
                SPMV_PW = 6, SPMV_RUPD = 7 };
constexpr bool spmv_jac(int mode) { return mode == SPMV_JACOBI || mode == SPMV_JACOBI_S; }
constexpr bool spmv_scaled(int mode) { return mode == SPMV_PLAIN_S || mode == SPMV_JACOBI_S; }
// SPMV_CG: the CG direction update and the deferred solution update ride in
// the MatMult.  The operand is p_i = z + b p_{i-1} (z = jac(r), i == 0: p = z),
// formed on the fly wherever the product reads it and stored once for the
// owned rows; x += xa p_{i-1} is applied to the owned rows when xpend != 0.
// The kernel evaluates the iteration's scalar top (cg_top, mx_cg.hpp) from
// the solver state `st` itself; the main MatMult launch commits it.
struct KspState;
struct Fold;
struct CgFuse {
  const double *r = nullptr;
  const double *pold = nullptr;
  double *pnew = nullptr;
  double *x = nullptr;
  KspState *st = nullptr;
  double *hist = nullptr;   // residual history (device) or null
  Jac jac;
};
void halo_begin(Mat *A, const double *x);  // pack + exchange into A->halo.lvec (compute stream)
void spmv_launch(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                 int *done_flag);
// MatMult with the halo on the comm stream overlapping the interior slices;
// returns the number of partials written (DOT / CG mode).  fold != null: the
// p.w partials are folded into fold->out inside the launch(es).
int matmult_overlap(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                    int *done_flag, const CgFuse *cg = nullptr, const Fold *fold = nullptr,
                    const double *xscale = nullptr);
int spmv_blocks(const Mat *A, int mode = SPMV_PLAIN);
// MatMult kernel timing from the dispatch's own timestamps (hipExtLaunchKernel
// start/stop events: no event packets between the kernels, so the measured
// span is the kernel's, as a profiler's trace sees it).  The KSP's SpMV timer
// arms it on one-rank solves; the next main SpMV launch of this host thread
// consumes it (mx_spmv.hip launch_timed).
struct ExtTiming { hipEvent_t a = nullptr, b = nullptr; bool armed = false, used = false; };
extern thread_local ExtTiming g_ext_timing;
// Host-side counts of the MatMult-family launches enqueued (or captured) by
// kind, for tests that must show which kernel a configuration ran
// (mx_debug_dispatch_counts); a relaxed atomic add per launch.
enum Dispatch {
  DSP_SELL = 0,          // spmv_sell_kernel (general SELL), any mode but SPMV_CG
  DSP_SELL_CG = 1,       // spmv_sell_kernel<SPMV_CG> (CG mode 1)
  DSP_PAIR_LEAN = 2,     // spmv_pair_lean_kernel (sweep form)
  DSP_PAIR_ZM = 3,       // spmv_pair_zm_kernel, one rank / no ghost units
  DSP_PAIR_ZM_SPLIT = 4, // spmv_pair_zm_kernel<SPLIT> (ghost units, boundary kernel after)
  DSP_PAIR_ZM27 = 5,
  DSP_PAIR_ZM27_SPLIT = 6,
  DSP_PAIR_ZMF64 = 7,
  DSP_PAIR_ZMF64_SPLIT = 8,
  DSP_PAIR_ZMCG = 9,     // retired (round 2's CG mode 4, removed in round 4); slot kept for the ABI's order
  DSP_BOUNDARY = 10,     // spmv_boundary_kernel
  DSP_ZM_PW = 11,        // CG mode 5: the z-march p.Ap pass (no product stored)
  DSP_ZM_RUPD = 12,      // CG mode 5: the z-march residual update (product recomputed)
  DSP_PAIR_ZMC = 13,     // spmv_pair_zmc_kernel (coded z-march), one rank / no ghost units
  DSP_PAIR_ZMC_SPLIT = 14,
  DSP_ZM_PBW = 15,       // CG mode 5: the direction update fused into the p.Ap pass (knob 69)
  DSP_ZM_PBWS = 16,      // CG mode 5 on P > 1 ranks: the same fused into the split p.Ap pass (knob 80)
  DSP_CB = 17,           // the column-block two-pass MatMult (mx_spmv_cb.hip, knob 84)
  DSP_COUNT = 18
};
void note_dispatch(int kind);
extern std::atomic<long long> g_dispatch[DSP_COUNT];
int device_cu_count();
int main_grid(const Mat *A, int mode, const void *kf, bool pairs);   // the SpMV's resident grid
// lean row-pair MatMult (mx_spmv_pair.hip): launched when it applies (returns its grid, else 0)
int pair_lean_launch(Mat *A, int mode, bool split, const double *x, double *y, double *partials, const int *done,
                     const Fold &fold, hipStream_t st, const Jac &jac = Jac{}, const double *xscale = nullptr);
bool pair_code_applies(const Mat *A);   // the coded z-march (mx_mat_info.pair_code)
void pair_sym_prepare(Mat *A);          // Mat::sym, once per operator, before a CG solve's capture
int pair_lean_kind(const Mat *A);   // 0 general kernel, 1 lean, 2 lean select-free (mx_mat_info.pair_lean)
bool pair_zm_applies(const Mat *A);  // the lean kernel's z-march form (mx_mat_info.pair_zmarch)
int pair_f64_kind(const Mat *A);     // 5 / 7: the fp64 row-pair z-march applies (mx_mat_info.pair_f64)
// CG mode 5: w = A p is not stored -- the p.Ap pass (matmult_overlap with
// SPMV_PW; on P > 1 ranks only the ghost units' rows are stored and finished
// by the boundary kernel) gives p.w, the update pass recomputes A p where it
// forms r - alpha A p (SPMV_RUPD; the ghost units' rows read w)
bool pair_cg5_applies(const Mat *A, int jac_mode);
int pair_cg5_rupd_launch(Mat *A, KspState *s, const double *p, const double *w, double *r, const double *r0,
                         int jac_mode, double jac_c, double *partials, const Fold &fold, const double *dot_part,
                         int ndot, int xb, int *hw, hipStream_t st);
// knob 69: CG mode 5's direction update fused into the p.Ap pass (one rank,
// clean symmetric 5/7-point; iterations i % xb != 0): forms and stores p_i
// (buffer i % xb) from r_i and p_{i-1}, leaves the p.Ap partials
bool pair_cg5_pbw_applies(const Mat *A, int jac_mode, int xb);
int pair_cg5_pbw_launch(Mat *A, KspState *s, const double *r, const double *r0, double *const pb[8], int xb,
                        double *hist, int jac_mode, double jac_c, double *partials, const Fold &fold,
                        hipStream_t st);
// knob 80: the same on P > 1 ranks with the split p.Ap pass (full rows; the
// ghost units' diagonal-block sums stored into y for the boundary kernel).
// cg5_pbws_matmult: the halo pack forms and sends the ghost planes' p_i, the
// fused pass runs meanwhile, the boundary kernel finishes the ghost rows
bool pair_cg5_pbws_applies(const Mat *A, int jac_mode, int xb);
int pair_cg5_pbws_launch(Mat *A, KspState *s, const double *r, double *const pb[8], int xb, double *hist, int jac_mode,
                         double jac_c, double *y, double *partials, hipStream_t st);
int cg5_pbws_matmult(Mat *A, KspState *s, const double *r, double *const pb[8], int xb, int it, double *hist,
                     const Jac &jac, double *y, double *partials, int *done, const Fold *fold);
// true when matmult_overlap splits the product: interior launch || halo, then
// a boundary launch (P > 1 with ghost entries and overlap on)
bool matmult_splits(const Mat *A);
void mat_mult(Mat *A, const double *x, double *y);
// column-block two-pass MatMult (mx_spmv_cb.hip): built at assembly for
// unstructured one-rank blocks; cb_launch returns the pass-2 grid (partials)
void build_cb(Mat *A, hipStream_t st);
bool cb_applies(const Mat *A, int mode, bool split);
int cb_launch(Mat *A, int mode, bool split, const double *x, double *y, const Jac &jac, double *partials,
              const int *done, const Fold &fold, const double *xscale, hipStream_t st);

// vector kernels (mx_vec.hip)
constexpr int RED_BLOCKS = 1024;   // fixed grid of the reduction kernels
void finish_reduce(const double *partials, int nblocks, int nvals, double *out, hipStream_t s,
                   int *done_flag = nullptr);
double host_dot(Comm *c, int64_t n, const double *x, const double *y);
// VecMDot: out_host[k] = x . y[k] (collective); VecMAXPY: y += sum_k alpha[k] x[k]
// with PETSc's grouping (VecMAXPY_Seq)
void host_mdot(Comm *c, int64_t n, const double *x, int nv, const double *const *y, double *out_host);
void vec_maxpy(hipStream_t s, int64_t n, double *y, int nv, const double *alpha, const double *const *x);
void vec_axpy(hipStream_t s, int64_t n, double a, const double *x, double *y);
void vec_aypx(hipStream_t s, int64_t n, double a, const double *x, double *y);
void vec_pmult(hipStream_t s, int64_t n, const double *x, const double *y, double *w);
void vec_scale(hipStream_t s, int64_t n, double a, double *x);
void vec_set(hipStream_t s, int64_t n, double a, double *x);
void vec_rhs_hash(hipStream_t s, int64_t i0, int64_t n, double *b);
void debug_stall(hipStream_t s, int stall_us);
void flush_read(hipStream_t s, const double *x, int64_t n, double *partials);   // RED_BLOCKS partials
void debug_stream_read(hipStream_t s, const double *x, int64_t n, int width, double *out);
void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, hipStream_t s,
                        int64_t *total_host);

// direct solve (mx_direct.hip)
void dense_lu_solve(Comm *c, int64_t n, const int64_t *ip, const int64_t *cj, const double *vv,
                    const double *b, double *x);

// KSP (mx_ksp.hip)
void ksp_solve(Mat *A, const mx_ksp_params &p, const double *b, double *x, mx_ksp_result &r,
               double *hist);

// grid helpers
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 16) {
  int64_t g = cdiv(n, block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// HIP loads a translation unit's code object at the first launch of one of
// its kernels (1-25 ms each for this library, 11 ms for the row-pair SpMV's
// alone): load_code_objects (mx_abi.hip) loads every unit's when a
// communicator is created, so that cost is paid at initialisation, not inside
// the first assembly or solve that needs a new kernel family.
void load_code_comm();
void load_code_vec();
void load_code_assembly();
void load_code_spmv();
void load_code_spmv_pair();
void load_code_spmv_cb();
void load_code_ksp();
void load_code_direct();
void load_code_objects();
// the first pinned, pipelined host-to-device copy's one-time costs (mx_abi.hip)
void h2d_warm();

}  // namespace mx
