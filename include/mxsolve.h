/*
 * mxsolve.h -- C ABI of libmxsolve.so, the MI355X-native (gfx950) hot path of
 * the Dxslab/mpi-petsc4py-example workflow:
 *
 *     createAIJ(csr=...)  ->  MatMult (VecScatter halo + SpMV)  ->  KSPSolve CG/GMRES + Jacobi
 *
 * Every entry point replaces one petsc4py/PETSc call the reference makes; the
 * "replaces" line cites the reference call site (file:line in the read-only
 * reference tree) and the PETSc routine it reaches.  Plain C types only: opaque
 * handles, raw pointers, sizes.  Device pointers ("_dev") are HIP device
 * addresses on the handle's GPU (the Python shim passes torch tensor
 * data_ptr()s); everything else is host memory.
 *
 * Return value of every function: 0 (MX_OK) or an MX_ERR_* class;
 * mx_last_error() returns the calling thread's last message.  The Python shim
 * maps MX_ERR_ARG to ValueError and the other classes to PETSc.Error.
 *
 * Collective calls (marked [collective]) must be made by every rank of the
 * communicator in the same order, as PETSc requires.
 */
#ifndef MXSOLVE_H
#define MXSOLVE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: mx_ksp_result grew the pbw / mdot / maxpy timing fields (its size changed) */
#define MX_ABI_VERSION 3

enum {
  MX_OK = 0,
  MX_ERR_ARG = 1,         /* bad argument (petsc4py ValueError)               */
  MX_ERR_OUTOFRANGE = 2,  /* index out of range (PETSC_ERR_ARG_OUTOFRANGE)    */
  MX_ERR_HIP = 3,         /* HIP runtime failure                              */
  MX_ERR_COMM = 4,        /* RCCL / communicator failure                      */
  MX_ERR_MEM = 5,         /* device allocation failure                        */
  MX_ERR_UNSUPPORTED = 6, /* valid request outside what this build implements */
  MX_ERR_INTERNAL = 7
};

typedef struct mx_comm_s *mx_comm;
typedef struct mx_mat_s *mx_mat;

/* ---- KSP parameters / results (KSPSetType, KSPSetTolerances, PCSetType) ---- */
enum { MX_KSP_CG = 0, MX_KSP_GMRES = 1, MX_KSP_PREONLY = 2 };
enum { MX_PC_NONE = 0, MX_PC_JACOBI = 1 };
enum { MX_NORM_DEFAULT = -1, MX_NORM_NONE = 0, MX_NORM_PRECONDITIONED = 1,
       MX_NORM_UNPRECONDITIONED = 2, MX_NORM_NATURAL = 3 };
enum { MX_INSERT_VALUES = 0, MX_ADD_VALUES = 1 };

typedef struct {
  int ksp_type;        /* MX_KSP_*                              (KSPSetType)          */
  int pc_type;         /* MX_PC_*                               (PCSetType)           */
  int norm_type;       /* MX_NORM_*                             (KSPSetNormType)      */
  int max_it;          /* default 10000                         (KSPSetTolerances)    */
  int restart;         /* GMRES restart, default 30             (KSPGMRESSetRestart)  */
  int guess_nonzero;   /* 0: x <- 0 first   (KSPSetInitialGuessNonzero)               */
  double rtol, atol, dtol; /* 1e-5, 1e-50, 1e5                                         */
  double haptol;       /* GMRES happy breakdown, 1e-30                                */
  double breakdowntol; /* GMRES restart consistency check, 0.1                        */
  int poll_every;      /* host polls the device convergence flag every k its (0: 16) */
  int profile;         /* bit 0: time every SpMV launch with HIP events (CG mode 5:
                          the plain p.Ap passes; GMRES: the MatMult); bit 1: every CG
                          mode-5 residual-update launch / GMRES MDot; bit 2: every CG
                          direction-update launch with batched x steps (cg_pb_kernel)
                          / GMRES MAXPY + norm; bit 3: every CG fused direction +
                          p.Ap pass (one rank: events attached to the kernel's
                          dispatch)                                                  */
} mx_ksp_params;

typedef struct {
  int its;             /* KSPGetIterationNumber                                     */
  int reason;          /* KSPConvergedReason value                                  */
  double rnorm;        /* KSPGetResidualNorm                                        */
  double solve_ms;     /* device time of the solve (HIP events, first to last kernel) */
  double spmv_ms;      /* sum of profiled SpMV launch times (profile = 1)           */
  int spmv_count;      /* SpMV launches profiled                                    */
  int launched_its;    /* iterations enqueued (>= its; the tail are device no-ops)  */
  int cg_mode;         /* CG: the fusion mode that ran (key 9's modes 0/1/2/4/5)     */
  double upd_ms;       /* sum of profiled residual-update launch times (profile bit 1) */
  int upd_count;       /* residual-update launches profiled                         */
  int cg_xbatch;       /* CG: deferred x steps applied every this many iterations    */
  double pb_ms;        /* sum of profiled direction-update launch times (profile bit 2) */
  int pb_count;        /* direction-update launches profiled                        */
  double pbw_ms;       /* sum of profiled fused direction + p.Ap pass times (bit 3)  */
  int pbw_count;       /* fused direction + p.Ap launches profiled                  */
  double mdot_ms;      /* GMRES: sum of profiled MDot launch times (profile bit 1)   */
  int mdot_count;
  double maxpy_ms;     /* GMRES: sum of profiled MAXPY + norm launch times (bit 2)   */
  int maxpy_count;
} mx_ksp_result;

typedef struct {
  int64_t M, N;          /* global sizes                       (MatGetSize)          */
  int64_t m, n;          /* local rows / cols                  (MatGetLocalSize)     */
  int64_t rstart, cstart;/* ownership starts                   (MatGetOwnershipRange) */
  int64_t nnz_d, nnz_o;  /* diagonal / off-diagonal block nonzeros                    */
  int64_t nghost;        /* |garray|                                                  */
  int64_t sell_slots_d, sell_slots_o; /* padded SELL-64 slots (bytes model)           */
  int nsend_peers, nrecv_peers;       /* halo neighbours                              */
  int64_t nsend, nrecv;               /* halo values per MatMult                      */
  int64_t dia_slices;                 /* A_d slices stored with aligned offsets       */
  int64_t value_codes;                /* A_d values as 1-byte codes into a table of this
                                         many distinct values (0: stored as fp64)       */
  int64_t code_bytes;                 /* bytes of those codes                         */
  int64_t pair_shape;                 /* row-pair SpMV layout: 5 / 7 / 27-point, 0 none */
  int64_t pair_units;                 /* 128-row units stored as row pairs (all units
                                         when pair_blocks is 0)                        */
  int64_t pair_blocks;                /* distinct unit code blocks streamed from the
                                         dictionary (0: one block per unit)           */
  int64_t pair_block_bytes;           /* bytes of one unit's code block               */
  int64_t pair_uniform;               /* 1: every dictionary block is uniform per slot
                                         (5/7/27-point): SpMV reads each block's slot
                                         values and lane masks, not code bytes (key 35) */
  int64_t pair_lean;                  /* MatMult kernel of the uniform-slot layout:
                                         0 general SELL kernel, 1 lean row-pair kernel
                                         with presence selects, 2 lean select-free
                                         ("clean": absent operands read as 0.0; key 38) */
  int64_t pair_zmarch;                /* 1: the lean kernel marches columns of units one
                                         plane (3D) / line (2D) apart, carrying two
                                         operand pairs in registers (key 39)          */
  int64_t pair_f64;                   /* 5 / 7: the fp64-valued (uncoded) layout also has
                                         row pairs -- each unit's values streamed as
                                         16-byte pairs -- and the z-march MatMult runs on
                                         them (one rank, select-free units; key 44)    */
  int64_t pair_form27;                /* 27-point z-march body: 2 column-zeroed (no branches,
                                         no selects; key 48), 1 per-run branches, 0 lane
                                         selects; -1 when the 27-point z-march does not run */
  int64_t pair_code;                  /* 1: the coded z-march MatMult runs -- 5/7-point code
                                         dictionary not uniform per slot, every block
                                         select-free (values from the LDS table; key 52) */
  int64_t cb_blocks;                  /* > 0: the column-block two-pass MatMult runs, with
                                         this many blocks of x (unstructured blocks whose
                                         entries mostly lie far from the diagonal; key 84) */
} mx_mat_info;

/* ---- library ---------------------------------------------------------------- */
int mx_version(void);
/* PetscFinalize: waits for all device work the library queued and returns
 * the device buffer cache (key 81: freed buffers kept for reuse, at most 1/8
 * of HBM) to the driver -- the library's counterpart of torch's empty_cache.
 * Handles must be destroyed before (or not used after) this call; calling it
 * again later (more work, then a trim) is allowed.                           */
int mx_finalize(void);
int mx_last_error(char *buf, size_t len);

/* ---- communicators (the comm= argument of createAIJ / KSP().create:
 *      test.py:24,33 ; petsc_funcs.py:6) ----------------------------------------- */
/* RCCL unique id for mx_comm_create_rccl (rank 0 creates, shim broadcasts it). */
int mx_get_unique_id(void *out, size_t len);
/* One process per GPU over RCCL/xGMI (replaces MPI_COMM_WORLD, test.py:55).   */
int mx_comm_create_rccl(int rank, int size, int device, const void *uid, size_t uid_len,
                        mx_comm *out);
/* Processes of one node that share GPUs (more ranks than devices, e.g.
 * `mpiexec -n 2 python test.py` on a one-GPU machine; RCCL refuses two ranks
 * on one device): device payloads staged through the POSIX shared-memory
 * segment `name` (rank 0 creates it, the others open it; unlinked once all
 * have mapped it), slot_kib KiB of staging per rank (<= 0: 64 MiB; larger
 * exchanges run in rounds).  Host-ordered correctness
 * transport; collectives fail with MX_ERR_COMM after mx_comm_abort on any rank.
 * [collective]                                                                  */
int mx_comm_create_shm(int rank, int size, int device, const char *name, int64_t slot_kib,
                       mx_comm *out);
/* Release peers blocked in a shared-memory collective (a failing rank calls
 * it), or abort an RCCL communicator (ncclCommAbort: its in-flight kernels
 * stop; waits on this rank fail with MX_ERR_COMM).  May be called from another
 * host thread than the one blocked in the collective (a wall-time watchdog);
 * every later collective on the communicator fails with MX_ERR_COMM.          */
int mx_comm_abort(mx_comm c);
/* Single-rank communicator (PETSC_COMM_SELF / MPI.COMM_WORLD of size 1).       */
int mx_comm_create_self(int device, mx_comm *out);
/* In-process virtual ranks that share one GPU (testing N>1 on a 1-GPU box):
 * one world, then one comm per rank, each used from its own host thread.       */
int mx_world_create_local(int size, void **world);
int mx_comm_create_local(void *world, int rank, int device, mx_comm *out);
int mx_world_destroy(void *world);
/* Mark the local world failed: every rank blocked in (or entering) one of its
 * collectives returns MX_ERR_COMM instead of waiting for the failed rank.    */
int mx_world_abort(void *world);
int mx_comm_destroy(mx_comm c);
int mx_comm_info(mx_comm c, int *rank, int *size, int *device);
/* The HIP stream every kernel of this communicator runs on (hipStream_t).      */
int mx_comm_stream(mx_comm c, void **stream);
int mx_comm_barrier(mx_comm c);  /* [collective] */

/* ---- layout: PetscSplitOwnership (test.py:68-74, test2.py:33-37) ---------- */
int mx_layout_split(int64_t N, int P, int64_t *ranges /* P+1 */);

/* ---- Mat ------------------------------------------------------------------ */
/* replaces PETSc.Mat().createAIJ(comm, size=(M,N), csr=(indptr, indices, data))
 * + assemble()  (petsc_funcs.py:6-7, test.py:24-28) -> MatCreate/MatSetSizes/
 * MatSetType(AIJ)/MatMPIAIJSetPreallocationCSR/MatSetValues/MatAssemblyEnd/
 * MatSetUpMultiply_MPIAIJ.  [collective]
 * m_local/n_local < 0 mean PETSC_DECIDE (PetscSplitOwnership).  indptr has
 * m_local+1 entries of indptr_bytes (4|8), cols nnz entries of col_bytes (4|8)
 * holding GLOBAL column ids.  Negative column ids are ignored, duplicates
 * follow insert_mode (INSERT: last wins; ADD: summed in input order).
 * Checks (petsc4py Mat_AllocAIJ_CSR): indptr[0] == 0, indptr[m] == nnz,
 * nondecreasing -> MX_ERR_ARG; column >= N -> MX_ERR_OUTOFRANGE.
 * src_is_device: the three arrays are device pointers, read in place (they
 * must stay valid and unchanged until the call returns).  4-byte column ids
 * are read as they are (no widened copy) whenever every row has at most 64
 * entries.                                                                       */
int mx_mat_create_csr(mx_comm c, int64_t M, int64_t N, int64_t m_local, int64_t n_local,
                      const void *indptr, int indptr_bytes, const void *cols, int col_bytes,
                      const double *vals, int64_t nnz, int insert_mode, int src_is_device,
                      mx_mat *A);
/* MatSetPreallocationCOO/MatSetValuesCOO-style assembly of locally owned rows
 * (global row/col ids, any order; negative ids ignored).  [collective]        */
int mx_mat_create_coo(mx_comm c, int64_t M, int64_t N, int64_t m_local, int64_t n_local,
                      const int64_t *rows, const int64_t *cols, const double *vals, int64_t n,
                      int insert_mode, int src_is_device, mx_mat *A);
/* Device-side generator of the synthetic operators feeding the
 * same COO assembly; kind 0: 2D 5-pt nx*ny, 1: 3D 7-pt, 2: 3D 27-pt,
 * 3: 3D convection-diffusion 7-pt.  Each rank generates its own rows.  [collective] */
int mx_mat_create_stencil(mx_comm c, int kind, int64_t nx, int64_t ny, int64_t nz, mx_mat *A);
int mx_mat_get_info(mx_mat A, mx_mat_info *info);
/* replaces Mat.getValuesCSR (MatGetRow_MPIAIJ): local rows, GLOBAL sorted cols. */
int mx_mat_get_csr(mx_mat A, int64_t *indptr, int64_t *cols, double *vals);
/* The PETSc MPIAIJ split: A_d (local cols), A_o (ghost index), garray.      */
int mx_mat_get_split(mx_mat A, int64_t *dptr, int32_t *dcol, double *dval, int64_t *optr,
                     int32_t *ocol, double *oval, int64_t *garray);
/* replaces MatMult (KSP_MatMult inside ksp.solve, test.py:50): halo + SpMV.  [collective] */
int mx_mat_mult(mx_mat A, const double *x_dev, double *y_dev);
/* replaces MatGetDiagonal (PCSetUp_Jacobi).                                  */
int mx_mat_get_diagonal(mx_mat A, double *d_dev);
/* Timing helper for bench.py: `iters` back-to-back MatMults; average device ms
 * per SpMV kernel launch and per full MatMult (halo included).  [collective]     */
int mx_mat_bench_mult(mx_mat A, const double *x_dev, double *y_dev, int iters,
                      double *spmv_ms, double *mult_ms);
/* Cold-cache timing for bench.py: `iters` times, stream the
 * flush_n-double device buffer flush_dev in (plain loads: L2 and the
 * memory-side cache then hold clean flush lines only), then one MatMult.  Medians over iters, device ms: the SpMV kernel
 * alone (one rank: events attached to its dispatch; else < 0) and the whole
 * MatMult from an event queued right behind the flush.  Every launch is
 * enqueued while the flush still runs, so no host gap is inside the spans.
 * [collective]                                                                 */
int mx_mat_bench_mult_cold(mx_mat A, const double *x_dev, double *y_dev, double *flush_dev, int64_t flush_n,
                           int iters, double *spmv_ms, double *mult_ms);
int mx_mat_destroy(mx_mat A);

/* ---- Vec (local length n, device pointers; reductions are collective) ----- */
int mx_vec_dot(mx_comm c, int64_t n, const double *x_dev, const double *y_dev, double *out);
int mx_vec_norm2(mx_comm c, int64_t n, const double *x_dev, double *out);
int mx_vec_axpy(mx_comm c, int64_t n, double alpha, const double *x_dev, double *y_dev);
int mx_vec_aypx(mx_comm c, int64_t n, double alpha, const double *x_dev, double *y_dev);
int mx_vec_pointwise_mult(mx_comm c, int64_t n, const double *x_dev, const double *y_dev,
                          double *w_dev);
int mx_vec_scale(mx_comm c, int64_t n, double alpha, double *x_dev);
int mx_vec_set(mx_comm c, int64_t n, double alpha, double *x_dev);
/* VecMDot (GMRES orthogonalisation): out_host[k] = x . y_k for
 * the nv device vectors listed in the host array y; one all-reduce of nv
 * values.  [collective]                                                      */
int mx_vec_mdot(mx_comm c, int64_t n, const double *x_dev, int nv, const double *const *y_dev_list,
                double *out_host);
/* VecMAXPY: y += sum_k alpha[k] x_k (alpha on the host), PETSc's VecMAXPY_Seq
 * grouping: the first nv % 4 vectors together, then groups of four.          */
int mx_vec_maxpy(mx_comm c, int64_t n, double *y_dev, int nv, const double *alpha_host,
                 const double *const *x_dev_list);
/* b_i = (splitmix64(i + 42 phi) >> 11) 2^-53 for global i in [i0, i0+n) */
int mx_vec_rhs_hash(mx_comm c, int64_t i0, int64_t n, double *b_dev);

/* ---- KSP: replaces ksp.solve(b, x) (test.py:50) -> KSPSolve with the
 *      configuration of test.py:33-47 + options.  [collective]              */
int mx_ksp_solve(mx_mat A, const mx_ksp_params *p, const double *b_dev, double *x_dev,
                 mx_ksp_result *res, double *history_host /* NULL or max_it+2 */);
void mx_ksp_default_params(mx_ksp_params *p);
/* KSPDestroy / KSPReset (test.py's ksp object going away): releases the solver
 * state kept on operator A between solves -- KSPSetUp work space, the device
 * convergence state, the captured CG iteration graph and the PCSetUp_Jacobi
 * result.  A stays usable; the next solve sets them up again.              */
int mx_ksp_destroy(mx_mat A);

/* ---- direct solve: replaces KSPPREONLY + PCLU (+ MUMPS) of test.py:38-43,138
 *      (SURVEY.md §8f F1).  The caller gathers the whole square system (global
 *      CSR, host) to one rank; it is densified and LU-factored with partial
 *      pivoting on that rank's GPU.  n <= 16384.                              */
int mx_lu_solve_csr(mx_comm c, int64_t n, const int64_t *indptr, const int64_t *cols,
                    const double *vals, const double *b, double *x);

/* ---- measurement knobs (A/B runs only; defaults are the product path) -------
 * key 6: halo exchange overlapping the interior slices when P > 1 (0/1, default 1)
 * key 7: CG iterations replayed from a captured hipGraph batch after one eager
 *        batch: 0 never, 1 single-rank communicators (default; equal at 256^3,
 *        2% faster at 64^3 per rank), 2 also multi-rank RCCL communicators
 * key 8: run the collective path (unfused folds + RCCL all-reduce) on a one-rank
 *        RCCL communicator (testing, default 0)
 * key 9: CG fusion: 0 separate passes; 1 direction update + x step inside the
 *        MatMult; 2 x step deferred into the direction update; 3 auto (default:
 *        5 on one rank where it applies, 2 on P > 1 ranks with the z-march
 *        MatMult, else 1 for <= 3M local rows, else 2); 4 (retired in round 4:
 *        runs as 2); 5 mode 2 whose
 *        MatMult stores no product: a p.Ap pass, and the update pass
 *        recomputes A p where it forms r - alpha A p (one rank, lean 5/7-point
 *        z-march layout, no or uniform Jacobi; else 2)
 * key 13: CG vector passes walk row pairs with 16-B accesses when every
 *         vector is aligned (0/1, default 0: one row per thread per step)
 * key 21: CG vector passes issue four steps' loads together: 0 never, 1 always,
 *         2 auto (default: up to 6M local rows)
 * key 23: value codes -- one byte per slot into a table of <= 255 distinct
 *         values -- for the diagonal block (read at assembly and at launch;
 *         0/1, default 1)
 * key 27: row-pair SpMV layout for 5/7/27-point patterns (read at assembly and
 *         at launch; 0/1, default 1)
 * key 29: CG modes 2/5 apply the deferred x steps every B iterations from B
 *         rotating direction buffers (1, 2, 4 or 8; default 0 = auto: 4 in
 *         mode 5, else 2; 8 -- the same bits -- measured within +-1% of 4 per
 *         256^3 iteration: the batch launch's eleven streams give back what
 *         the rarer x pass saves)
 * key 33: no-progress deadline in ms of the KSP poller's wait on an RCCL
 *         communicator (re-armed whenever the device's count of iterations
 *         begun moves); past it the communicator is aborted and the call fails
 *         with MX_ERR_COMM (default 120000).  An RCCL asynchronous error aborts
 *         at once in every wait
 * key 38: the lean row-pair MatMult (mx_spmv_pair.hip) for uniform-slot 5/7-point
 *         layouts (0/1, default 1; the same bits)
 * key 39: its z-march form (a wave marches a column of units one plane apart,
 *         two operand pairs carried in registers; 0 = the sweep form; default 1)
 * key 40: z-march resident workgroups per CU (1..8, default 4)
 * key 41: z-march segment length in planes (default 32, shortened when a slab
 *         has too few columns for every wave)
 * key 43: grid of the SpMV for fp64-valued (uncoded) layouts (default 8192
 *         workgroups; 0 = one resident generation)
 * key 47: deadline in ms of the RCCL waits that observe no progress (stream /
 *         event waits, setup collectives, barrier); 0 = none (default 600000:
 *         a slow peer is not an error, a dead one fails the call after 10 min).
 *         The GMRES restart read-back observes the step count (key 33)
 * key 48: 27-point column words (read at assembly; 0/1, default 1): the
 *         27-point z-march zeroes empty runs and x-line edges where it loads
 *         them (no per-run branches, no selects; the same bits)
 * key 59: CG mode 5's p.Ap pass on a symmetric operator sums each row's
 *         forward half, p^T A p = sum_i p_i (a_ii p_i + 2 fwd_i) -- 27-point:
 *         symmetry from the column-word layout; 5/7-point: A_d checked once
 *         per operator (1, default; 0: the full rows -- mode 2's p.w bits)
 * key 60: 27-point column-word z-march plane-pipelined -- each loaded plane
 *         advances three units' running sums, nothing but two sums and the
 *         centre pair carried (1, default; 0: six operand pairs carried)
 * key 52: coded z-march MatMult for 5/7-point code dictionaries that are not
 *         uniform per slot (1, default; 0: the general SELL kernel)
 * key 53: z-march terms of slots whose value is -1, 0 or +1 formed by fma (an
 *         exact product: the same bits; 1, default; 0: multiply and add)
 * key 61: testing: a device stall of this many us before each GMRES restart
 *         read-back (default 0), so the no-progress deadline can be driven
 * (keys 16, 24, 31, 50, 51, 62-64, 66, 67 -- variants measured and not kept --
 *  were retired in round 5; setting them has no effect)
 * key 68: CG mode 5's 7-point residual update with two lines per wave (line
 *         y's +n operand is line y + 1's centre pair: 8 vector loads per two
 *         units instead of 10; the same row sums, the norm partials grouped
 *         by other rows): 0 off, 1 on, 2 on with a 5-waves-per-SIMD register
 *         budget, 3 (default) 2 from 2^23 rows, else off
 * key 69: CG mode 5's direction update p = z + b p fused into its p.Ap pass
 *         (one rank, a clean symmetric 5/7-point layout, x batches of 2 or 4):
 *         the pass forms p_i from r_i and p_{i-1} for every operand it needs,
 *         stores the centre rows' (the iterations between x-step batches;
 *         the batch iterations keep the separate passes) -- the same bits as
 *         the separate direction update + PW pass: 0 off, 1 on, 5 (default)
 *         by size: 7-point up to 2^23 rows (128^3 -20% per iteration, 2^23
 *         -8%; 256^3 +2%: the residual update after it slows by more than it
 *         saves), 5-point up to 2^24 (2048^2 -14%, C2's 4096^2 -1.7%)
 * key 70: the 27-point plane-pipelined z-march with two lines per wave (the
 *         column words pair up by lines: line y's dy = +1 run is line y + 1's
 *         centre run, 8 loads per plane for two units instead of 12; the same
 *         row sums) for the MatMult, CG mode 5's residual update and its
 *         forward-half p.Ap pass (1, default: C5's share 199.7 -> 185.9 us per
 *         CG iteration, residual update 86 -> 78 us, p.Ap pass 37 -> 30 us,
 *         MatMult -5%; 0 off; 2: the p.Ap pass by groups of four lines,
 *         27.5 us, the iteration unchanged)
 * key 72: assembly canonicalises and splits rows in two register passes
 *         (count, then fill after the row-pointer scans) when every row has
 *         at most 64 entries (1, default; 0: the canonical copy in HBM, then
 *         the split passes -- the path rows longer than 64 always take; the
 *         same arrays bit for bit)
 * key 80: CG mode 5 on P > 1 ranks fuses the direction update into the split
 *         p.Ap pass on the iterations between x-step batches (the halo pack
 *         forms the ghost planes' p_i from r and p_{i-1}; the same bits as
 *         the separate passes): 1 on (default), 0 off
 * key 81: freed device buffers >= 1 MiB (assembly's transients, a
 *         destroyed operator's arrays, KSP work space) go to a per-device
 *         cache (at most 1/8 of HBM, 48 GiB) instead of hipFree, for the next
 *         allocation of a similar size to take (1, default; 0 off and the
 *         cache emptied; emptied too by mx_comm_destroy and mx_finalize; 2: as
 *         1, and every block handed out is filled with 0xA5 bytes first --
 *         tests: a buffer read before it is written shows up)
 * key 84: the column-block two-pass MatMult for unstructured blocks (read at
 *         assembly; mx_spmv_cb.hip): 1 (default) on one rank when A_d is a
 *         general SELL block of >= 2^20 rows with half its entries or more
 *         2^17 columns or further from the diagonal, 2 for every general
 *         block (tests), 0 never; the same bits as the one-pass kernel
 * (key 18, physically contiguous allocations, was retired in round 6: freed
 *  contiguous blocks whose address range was reused were still reached through
 *  stale translations -- DESIGN.md section 12.1)
 * (keys 1, 3, 4, 5, 10, 11, 12, 14, 15, 19, 22, 25, 26, 28, 30, 32, 34-37,
 *  42, 44-46, 49, 54-58, 65, 74-79 -- settings measured in rounds 1-5 and
 *  fixed at their chosen values -- are compile-time constants since round 6
 *  (mx_internal.hpp Knobs); setting them has no effect and returns -1)
 * Returns the previous value.                                                   */
int mx_debug_set(int key, int value);
/* Test hook: host-side counts of the MatMult-family kernel launches
 * enqueued (or captured into a graph) since the last reset, by kind --
 * 0 general SELL, 1 SELL CG-fused (mode 1), 2 row-pair sweep, 3 / 4 7/5-point
 * z-march (split: ghost units), 5 / 6 27-point z-march, 7 / 8 fp64 row-pair
 * z-march, 9 retired (round 2's CG mode 4), 10 halo-boundary kernel, 11 / 12
 * CG mode 5's p.Ap and residual-update z-march passes, 13 / 14 coded z-march
 * (split: ghost units), 15 CG mode 5's direction update fused into the p.Ap
 * pass (key 69), 16 the same fused into the split p.Ap pass on P > 1 ranks
 * (key 80), 17 the column-block two-pass MatMult (key 84).  Writes min(n, 18)
 * counts; reset != 0
 * zeroes them.  Not a PETSc call: it lets the parity tests show which
 * kernel ran (replayed graph launches are not counted).                     */
int mx_debug_dispatch_counts(int64_t *out, int n, int reset);
/* Phase times (ms, host wall clock between stream synchronisations) of the
 * calling thread's last mx_mat_create_csr: 0 host-to-device copy of the CSR
 * arrays (+ index widening), 1 row canonicalisation (longest row, sort,
 * duplicate fold), 2 MPIAIJ split (A_d / A_o / garray), 3 SpMV layouts (SELL,
 * value codes, row pairs, dictionary), 4 halo plan, 5 total, 6 bytes read
 * from host memory, 7 allocation of the copied input's device buffers (before
 * phase 0, within 5).  Writes min(n, 8) values.                             */
int mx_debug_assembly_times(double *out, int n);
/* Calibration stream for PMC byte counters: reads n doubles once with
 * width_bytes (8 or 16) per lane, non-temporal like the SpMV matrix stream,
 * and writes one partial sum per workgroup to out_dev.                      */
int mx_debug_stream_read(mx_comm c, const double *x_dev, int64_t n, int width_bytes, double *out_dev);
/* Device memory for vectors (what PETSc's VecCreate allocates): hipMalloc;
 * the shim wraps it as a torch tensor.  Blocks >= 1 MiB come from / return to
 * the library's device buffer cache (key 81).                                */
int mx_dev_alloc(int device, size_t bytes, void **ptr);
int mx_dev_free(void *ptr);
/* Communication latency on the communicator's stream, iters back to back
 * (device time per operation, microseconds): what 0 = all-reduce of 1 double,
 * 1 = of 3 doubles (the CG reductions), 2 = the halo exchange of A (pack +
 * send/recv, VecScatter).  [collective]                                       */
int mx_debug_comm_bench(mx_comm c, mx_mat A, int what, int iters, double *us_per);
/* Failure-detection test hook: enqueues ~stall_us of device time on the
 * communicator's stream (a bounded spin) and waits for it through the
 * communicator's watched wait (key 47 deadline, RCCL async-error polling).  */
int mx_debug_comm_stall(mx_comm c, int stall_us);

#ifdef __cplusplus
}
#endif
#endif
