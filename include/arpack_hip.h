/*
 * arpack_hip.h — drop-in C-ABI of the MI355X-native IRL/IRA engine.
 *
 * The first block re-exports, unchanged, the ISO_C_BINDING entry points of
 * arpack-ng (reference: ICB/arpack.h:10-21, implemented by SRC/icbads.F90:3-92,
 * SRC/icbadn.F90, SRC/icbazn.F90), plus the statistics/debug hooks
 * (ICB/stat_c.h, ICB/debug_c.h).  Existing callers re-link against
 * libarpack_hip.so and keep their reverse-communication loop as is:
 *
 *   - host pointers (malloc'ed resid/v/workd): the engine mirrors V, resid and
 *     workd in HBM and copies only the workd slice named by ipntr across PCIe
 *     at each ido = -1/1/2 return;
 *   - device pointers (hipMalloc'ed resid/v/workd): zero-copy; the caller's OP
 *     kernel reads workd[ipntr[0]-1] and writes workd[ipntr[1]-1] on device.
 *     Before calling *aupd_c again the caller must have finished its OP (or
 *     share the engine's stream via arpack_hip_set_stream).
 *   workl, iparam, ipntr, select, d, workev are host memory.
 *
 * The second block (arpack_hip_*) is the native extension: a device CSR
 * operator and an entry that serves every OP*x request on the GPU without
 * returning to the caller (used by bench.py and the multi-GPU layer).
 */
#ifndef ARPACK_HIP_H
#define ARPACK_HIP_H

#include <stddef.h>
#include <stdint.h>

/* a_int: int (LP64, libarpack_hip.so) or int64_t (ILP64, libarpack_hip64.so: define
 * a_int as int64_t before including, as arpackdef.h.in:6-14 does with INTERFACE64=1) */
#ifndef a_int
#define a_int int
#endif

/* complex128 as the ICB passes it (arpackdef.h.in:40-41): C99 double _Complex */
#ifndef a_dcomplex
#define a_dcomplex _Complex double
#endif
/* complex64 (arpackdef.h.in:39): C99 float _Complex */
#ifndef a_fcomplex
#define a_fcomplex _Complex float
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference ICB (ICB/arpack.h:16-17; SRC/icbads.F90:3-92) ------------------ */
void dsaupd_c(a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
              double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
              a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int* info);
void dseupd_c(a_int rvec, char const* howmny, a_int const* select, double* d, double* z,
              a_int ldz, double sigma, char const* bmat, a_int n, char const* which,
              a_int nev, double tol, double* resid, a_int ncv, double* v, a_int ldv,
              a_int* iparam, a_int* ipntr, double* workd, double* workl, a_int lworkl,
              a_int* info);

/* dnaupd_c (ICB/arpack.h:18; SRC/icbadn.F90): same arguments as dsaupd_c, but
 * ipntr has 14 entries and lworkl >= 3*ncv^2 + 6*ncv. */
void dnaupd_c(a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
              double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
              a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int* info);

/* dneupd_c (ICB/arpack.h:19; SRC/icbadn.F90): dr/di (nev+1), z(ldz, nev+1),
 * workev(3*ncv); sigmar/sigmai by value. */
void dneupd_c(a_int rvec, char const* howmny, a_int const* select, double* dr, double* di,
              double* z, a_int ldz, double sigmar, double sigmai, double* workev,
              char const* bmat, a_int n, char const* which, a_int nev, double tol, double* resid,
              a_int ncv, double* v, a_int ldv, a_int* iparam, a_int* ipntr, double* workd,
              double* workl, a_int lworkl, a_int* info);

/* znaupd_c / zneupd_c (ICB/arpack.h:20-21; SRC/icbazn.F90): complex128 arrays,
 * lworkl >= 3*ncv^2 + 5*ncv, rwork(ncv), workev(2*ncv). */
void znaupd_c(a_int* ido, char const* bmat, a_int n, char const* which, a_int nev, double tol,
              a_dcomplex* resid, a_int ncv, a_dcomplex* v, a_int ldv, a_int* iparam,
              a_int* ipntr, a_dcomplex* workd, a_dcomplex* workl, a_int lworkl, double* rwork,
              a_int* info);
void zneupd_c(a_int rvec, char const* howmny, a_int const* select, a_dcomplex* d,
              a_dcomplex* z, a_int ldz, a_dcomplex sigma, a_dcomplex* workev, char const* bmat,
              a_int n, char const* which, a_int nev, double tol, a_dcomplex* resid, a_int ncv,
              a_dcomplex* v, a_int ldv, a_int* iparam, a_int* ipntr, a_dcomplex* workd,
              a_dcomplex* workl, a_int lworkl, double* rwork, a_int* info);

/* ---- single precision (ICB/arpack.h:16-19; SRC/ssaupd.f, snaupd.f, sseupd.f,
 *      sneupd.f).  V, resid, workd and the kernels are fp32 in HBM (half the
 *      bytes of the d* family); the ncv-sized host work runs in double on a
 *      shadow of workl, rounded into the caller's float workl at every return.
 *      tol <= 0 selects slamch('EpsMach') = 2^-24.  One GPU, reverse
 *      communication (no device-CSR or distributed entries). */
void ssaupd_c(a_int* ido, char const* bmat, a_int n, char const* which, a_int nev, float tol,
              float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam, a_int* ipntr,
              float* workd, float* workl, a_int lworkl, a_int* info);
void sseupd_c(a_int rvec, char const* howmny, a_int const* select, float* d, float* z,
              a_int ldz, float sigma, char const* bmat, a_int n, char const* which, a_int nev,
              float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
              a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int* info);
void snaupd_c(a_int* ido, char const* bmat, a_int n, char const* which, a_int nev, float tol,
              float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam, a_int* ipntr,
              float* workd, float* workl, a_int lworkl, a_int* info);
void sneupd_c(a_int rvec, char const* howmny, a_int const* select, float* dr, float* di,
              float* z, a_int ldz, float sigmar, float sigmai, float* workev, char const* bmat,
              a_int n, char const* which, a_int nev, float tol, float* resid, a_int ncv,
              float* v, a_int ldv, a_int* iparam, a_int* ipntr, float* workd, float* workl,
              a_int lworkl, a_int* info);
void ssaupd_(a_int* ido, char const* bmat, a_int* n, char const* which, a_int* nev, float* tol,
             float* resid, a_int* ncv, float* v, a_int* ldv, a_int* iparam, a_int* ipntr,
             float* workd, float* workl, a_int* lworkl, a_int* info, size_t bmat_len,
             size_t which_len);
void snaupd_(a_int* ido, char const* bmat, a_int* n, char const* which, a_int* nev, float* tol,
             float* resid, a_int* ncv, float* v, a_int* ldv, a_int* iparam, a_int* ipntr,
             float* workd, float* workl, a_int* lworkl, a_int* info, size_t bmat_len,
             size_t which_len);
void sseupd_(a_int* rvec, char const* howmny, a_int* select, float* d, float* z, a_int* ldz,
             float* sigma, char const* bmat, a_int* n, char const* which, a_int* nev, float* tol,
             float* resid, a_int* ncv, float* v, a_int* ldv, a_int* iparam, a_int* ipntr,
             float* workd, float* workl, a_int* lworkl, a_int* info, size_t howmny_len,
             size_t bmat_len, size_t which_len);
void sneupd_(a_int* rvec, char const* howmny, a_int* select, float* dr, float* di, float* z,
             a_int* ldz, float* sigmar, float* sigmai, float* workev, char const* bmat, a_int* n,
             char const* which, a_int* nev, float* tol, float* resid, a_int* ncv, float* v,
             a_int* ldv, a_int* iparam, a_int* ipntr, float* workd, float* workl, a_int* lworkl,
             a_int* info, size_t howmny_len, size_t bmat_len, size_t which_len);

/* ---- complex64 (ICB/arpack.h:10-11; SRC/cnaupd.f, SRC/cneupd.f): complex64
 *      n-length data and kernels, complex128 reductions and host work (workl
 *      shadow), tol <= 0 -> slamch('EpsMach'); reverse communication on one GPU. */
void cnaupd_c(a_int* ido, char const* bmat, a_int n, char const* which, a_int nev, float tol,
              a_fcomplex* resid, a_int ncv, a_fcomplex* v, a_int ldv, a_int* iparam,
              a_int* ipntr, a_fcomplex* workd, a_fcomplex* workl, a_int lworkl, float* rwork,
              a_int* info);
void cneupd_c(a_int rvec, char const* howmny, a_int const* select, a_fcomplex* d,
              a_fcomplex* z, a_int ldz, a_fcomplex sigma, a_fcomplex* workev, char const* bmat,
              a_int n, char const* which, a_int nev, float tol, a_fcomplex* resid, a_int ncv,
              a_fcomplex* v, a_int ldv, a_int* iparam, a_int* ipntr, a_fcomplex* workd,
              a_fcomplex* workl, a_int lworkl, float* rwork, a_int* info);
void cnaupd_(a_int* ido, char const* bmat, a_int* n, char const* which, a_int* nev, float* tol,
             a_fcomplex* resid, a_int* ncv, a_fcomplex* v, a_int* ldv, a_int* iparam,
             a_int* ipntr, a_fcomplex* workd, a_fcomplex* workl, a_int* lworkl, float* rwork,
             a_int* info, size_t bmat_len, size_t which_len);
void cneupd_(a_int* rvec, char const* howmny, a_int* select, a_fcomplex* d, a_fcomplex* z,
             a_int* ldz, a_fcomplex* sigma, a_fcomplex* workev, char const* bmat, a_int* n,
             char const* which, a_int* nev, float* tol, a_fcomplex* resid, a_int* ncv,
             a_fcomplex* v, a_int* ldv, a_int* iparam, a_int* ipntr, a_fcomplex* workd,
             a_fcomplex* workl, a_int* lworkl, float* rwork, a_int* info, size_t howmny_len,
             size_t bmat_len, size_t which_len);

/* ---- Fortran symbols (SRC/dsaupd.f:182-186, SRC/dseupd.f:218-223): every
 *      argument by reference + hidden trailing CHARACTER lengths ---------------- */
void dsaupd_(a_int* ido, char const* bmat, a_int* n, char const* which, a_int* nev,
             double* tol, double* resid, a_int* ncv, double* v, a_int* ldv, a_int* iparam,
             a_int* ipntr, double* workd, double* workl, a_int* lworkl, a_int* info,
             size_t bmat_len, size_t which_len);
void dnaupd_(a_int* ido, char const* bmat, a_int* n, char const* which, a_int* nev,
             double* tol, double* resid, a_int* ncv, double* v, a_int* ldv, a_int* iparam,
             a_int* ipntr, double* workd, double* workl, a_int* lworkl, a_int* info,
             size_t bmat_len, size_t which_len);
void dneupd_(a_int* rvec, char const* howmny, a_int* select, double* dr, double* di, double* z,
             a_int* ldz, double* sigmar, double* sigmai, double* workev, char const* bmat,
             a_int* n, char const* which, a_int* nev, double* tol, double* resid, a_int* ncv,
             double* v, a_int* ldv, a_int* iparam, a_int* ipntr, double* workd, double* workl,
             a_int* lworkl, a_int* info, size_t howmny_len, size_t bmat_len, size_t which_len);
void znaupd_(a_int* ido, char const* bmat, a_int* n, char const* which, a_int* nev,
             double* tol, a_dcomplex* resid, a_int* ncv, a_dcomplex* v, a_int* ldv,
             a_int* iparam, a_int* ipntr, a_dcomplex* workd, a_dcomplex* workl, a_int* lworkl,
             double* rwork, a_int* info, size_t bmat_len, size_t which_len);
void zneupd_(a_int* rvec, char const* howmny, a_int* select, a_dcomplex* d, a_dcomplex* z,
             a_int* ldz, a_dcomplex* sigma, a_dcomplex* workev, char const* bmat, a_int* n,
             char const* which, a_int* nev, double* tol, a_dcomplex* resid, a_int* ncv,
             a_dcomplex* v, a_int* ldv, a_int* iparam, a_int* ipntr, a_dcomplex* workd,
             a_dcomplex* workl, a_int* lworkl, double* rwork, a_int* info, size_t howmny_len,
             size_t bmat_len, size_t which_len);
void dseupd_(a_int* rvec, char const* howmny, a_int* select, double* d, double* z,
             a_int* ldz, double* sigma, char const* bmat, a_int* n, char const* which,
             a_int* nev, double* tol, double* resid, a_int* ncv, double* v, a_int* ldv,
             a_int* iparam, a_int* ipntr, double* workd, double* workl, a_int* lworkl,
             a_int* info, size_t howmny_len, size_t bmat_len, size_t which_len);

/* ---- statistics / debug (ICB/stat_c.h, ICB/debug_c.h; stat.h:8-21) ---------- */
void sstats_c(void);
void sstatn_c(void);
void cstatn_c(void);
void stat_c(a_int* nopx, a_int* nbx, a_int* nrorth, a_int* nitref, a_int* nrstrt,
            float* tsaupd, float* tsaup2, float* tsaitr, float* tseigt, float* tsgets,
            float* tsapps, float* tsconv, float* tnaupd, float* tnaup2, float* tnaitr,
            float* tneigh, float* tngets, float* tnapps, float* tnconv, float* tcaupd,
            float* tcaup2, float* tcaitr, float* tceigh, float* tcgets, float* tcapps,
            float* tcconv, float* tmvopx, float* tmvbx, float* tgetv0, float* titref,
            float* trvec);
void debug_c(a_int logfil, a_int ndigit, a_int mgetv0, a_int msaupd, a_int msaup2,
             a_int msaitr, a_int mseigt, a_int msapps, a_int msgets, a_int mseupd,
             a_int mnaupd, a_int mnaup2, a_int mnaitr, a_int mneigh, a_int mnapps,
             a_int mngets, a_int mneupd, a_int mcaupd, a_int mcaup2, a_int mcaitr,
             a_int mceigh, a_int mcapps, a_int mcgets, a_int mceupd);

/* ---- native extension ---------------------------------------------------------- *
 * LP64 (plain int) in both builds: only the reference ABI above follows a_int. */
typedef struct arpack_hip_csr arpack_hip_csr;

/* Version / capability probe: returns a static string. */
const char* arpack_hip_version(void);
/* Number of visible GPUs (0 on a CPU-only host; never initialises a context). */
int arpack_hip_device_count(void);
/* PCI bus id "dddd:bb:dd.f" of `device` into buf (len >= 13); 0 or -1. */
int arpack_hip_device_pci_bus_id(int device, char* buf, int len);
/* Share a HIP stream (hipStream_t) with the engine; NULL = engine-owned stream. */
void arpack_hip_set_stream(void* stream);

/* Device memory helpers (so callers need no other GPU runtime binding). */
void* arpack_hip_malloc(size_t bytes);
void arpack_hip_free(void* p);
int arpack_hip_memcpy(void* dst, const void* src, size_t bytes); /* any direction; complete on return */
int arpack_hip_memset(void* dst, int value, size_t bytes); /* complete on return */
int arpack_hip_synchronize(void);

/* Register a CSR matrix (rowptr int64[n+1], col int32[nnz], val f64[nnz]).
 * Pointers may be host or device; host data is copied to HBM.  0; -1 if the
 * arrays could not be placed in HBM; -2 if a HIP call of the SpMV plan
 * analysis failed (nothing is kept). */
int arpack_hip_csr_create(arpack_hip_csr** A, int64_t n, int64_t nnz, const int64_t* rowptr,
                          const int32_t* col, const double* val);
void arpack_hip_csr_destroy(arpack_hip_csr* A);
/* SpMV kernel choice: 0 vector (G lanes/row), 1 CSR-stream, 2 CSR-stream with
 * non-temporal val/col loads; tile = nonzeros per workgroup (2048 or 4096). */
int arpack_hip_csr_set_kernel(arpack_hip_csr* A, int kernel, int tile);
/* Declare A symmetric (on != 0): the SpMV then streams only the upper
 * triangle (col >= row, diagonal included); stored entries below the diagonal
 * are ignored, as with MKL's symmetric/upper matrix descriptor.  Square,
 * unsharded matrices whose upper rows reach at most ~4096 columns past the
 * superblock fit the LDS windows; otherwise returns -1 and A keeps its
 * full-storage kernel.  y is then not bitwise reproducible run to run
 * (transposed terms are summed in LDS in schedule order).  on == 0 restores
 * the full-storage kernel.  For a row-distributed operator (after
 * arpack_hip_dist_create, until arpack_hip_dist_destroy) the call is
 * COLLECTIVE, with on = 1 and with on = 0: the halo and spill exchanges differ
 * between the modes, so every rank must call it; the ranks agree (one
 * allreduce) and if any rank's plan fails every rank keeps the full-storage
 * kernel and returns nonzero (its own plan error, or -2 when only another
 * rank's plan failed); -3 if the distribution's communicator has been
 * destroyed.  The transposed terms are summed in the kernel's fixed-point
 * form (exact 64-bit integers: y bitwise reproducible, each term rounded to
 * 2^-51 of the window's largest |a_ij| max|x|) wherever the operator fits it
 * on every rank and its upper off-diagonal magnitudes span at most 2^20 -- the
 * default since round 6 -- else (a graded operator, unless deterministic mode
 * asks for the fixed-point form) as LDS fp64 atomics in
 * schedule order (y reproducible to ~1 ulp, not bitwise; also selected by
 * arpack_hip_csr_set_sym_accumulator(A, 1)).  The form does not fit with no
 * free LDS word past a window, columns receiving more than 2^22 transposed
 * terms, or a largest off-diagonal magnitude outside [2^-900, 2^900].  In
 * deterministic mode (arpack_hip_set_deterministic) on = 1 returns 0 with the
 * fixed-point form, or keeps the full-storage kernel and returns 1 for an
 * operator outside it. */
int arpack_hip_csr_set_symmetric(arpack_hip_csr* A, int on);
/* The symmetric kernel's accumulator for A: 0 the fixed-point form where it
 * fits (default), 1 the LDS fp64 atomics.  -1 on a bad argument.  Takes
 * effect at the next product; deterministic mode overrides 1. */
int arpack_hip_csr_set_sym_accumulator(arpack_hip_csr* A, int acc);
/* The SpMV form A runs now: 0 full storage, 1 symmetric with the fp64
 * accumulator (not bitwise reproducible), 2 symmetric fixed-point (bitwise). */
int arpack_hip_csr_sym_form(const arpack_hip_csr* A);
/* Average device time (ms, hipEvents) of `reps` back-to-back SpMVs. */
double arpack_hip_csr_time(const arpack_hip_csr* A, const double* x, double* y, int reps);
/* y = A x on device (x, y device pointers). */
int arpack_hip_csr_spmv(const arpack_hip_csr* A, const double* x, double* y);

/* dsaupd_c with OP = A served on the GPU: same arguments and results as
 * dsaupd_c (mode 1, bmat 'I'), but returns only with ido = 99 (or ido = 3 when
 * iparam[0] = 0 asks for user shifts). */
void arpack_hip_dsaupd_csr(const arpack_hip_csr* A, int* ido, char const* bmat, int n,
                           char const* which, int nev, double tol, double* resid, int ncv,
                           double* v, int ldv, int* iparam, int* ipntr, double* workd,
                           double* workl, int lworkl, int* info);

/* Same, but parks after at most `max_cycles` further restart cycles with
 * ido = 98 (tol by reference, as dsaupd_).  Call again with ido = 98 to
 * continue; ido = 99 when the solve is complete.  Used to time exactly K
 * restart cycles (bench.py); max_cycles < 0 never parks. */
void arpack_hip_dsaupd_csr_cycles(const arpack_hip_csr* A, int max_cycles, int* ido,
                                  char const* bmat, int n, char const* which, int nev,
                                  double* tol, double* resid, int ncv, double* v, int ldv,
                                  int* iparam, int* ipntr, double* workd, double* workl,
                                  int lworkl, int* info);

/* dnaupd with OP = A served on the GPU (mode 1), cycle-parked like
 * arpack_hip_dsaupd_csr_cycles (SRC/dnaupd.f semantics, ipntr[14]). */
void arpack_hip_dnaupd_csr_cycles(const arpack_hip_csr* A, int max_cycles, int* ido,
                                  char const* bmat, int n, char const* which, int nev,
                                  double* tol, double* resid, int ncv, double* v, int ldv,
                                  int* iparam, int* ipntr, double* workd, double* workl,
                                  int lworkl, int* info);

/* Complex CSR operator (rowptr int64[n+1], col int32[nnz], val complex128[nnz]
 * interleaved) and the complex random operator of BASELINE config 5 (SURVEY.md
 * §8d S5: per_row hashed columns, U(-1,1)+iU(-1,1) on a 2^-10 grid, duplicate
 * columns summed, diagonal += dshift).  The product's scratch (the column
 * slices' partial sums and, in deterministic mode, the block maxima of |x| that
 * set the fixed-point scale) belongs to the operator: products of one
 * arpack_hip_zcsr must be ordered on one stream (two solves sharing it run one
 * after the other, or each holds its own operator). */
typedef struct arpack_hip_zcsr arpack_hip_zcsr;
int arpack_hip_zcsr_create(arpack_hip_zcsr** A, int64_t n, int64_t nnz, const int64_t* rowptr,
                           const int32_t* col, const double* val);
int arpack_hip_gen_zrandom(arpack_hip_zcsr** A, int64_t n, int per_row, uint32_t seed,
                           double dshift);
void arpack_hip_zcsr_destroy(arpack_hip_zcsr* A);
int arpack_hip_zcsr_info(const arpack_hip_zcsr* A, int64_t* n, int64_t* nnz);
/* The product's layout: *form 0 wave-per-row CSR, 1 XCD column split (slice
 * CSRs), 2 column-sorted tiles (20 B an entry), 3 packed tiles (16-B value +
 * 16-bit row/column-step code + a base column per 64 entries); *stored: the
 * entries the product streams (packed: incl. zero-valued fillers and padding). */
int arpack_hip_zcsr_tile_info(const arpack_hip_zcsr* A, int* form, int64_t* stored);
int arpack_hip_zcsr_download(const arpack_hip_zcsr* A, int64_t* rowptr, int32_t* col,
                             double* val);
int arpack_hip_zcsr_spmv(const arpack_hip_zcsr* A, const double* x, double* y);
/* znaupd (mode 1) with OP = A served on the GPU; returns with ido = 99. */
void arpack_hip_znaupd_zcsr(const arpack_hip_zcsr* A, int* ido, char const* bmat, int n,
                            char const* which, int nev, double* tol, a_dcomplex* resid,
                            int ncv, a_dcomplex* v, int ldv, int* iparam, int* ipntr,
                            a_dcomplex* workd, a_dcomplex* workl, int lworkl, double* rwork,
                            int* info);

/* Shift-invert operator on the device: y = (A - sigma I)^{-1} x by BiCGStab on
 * the complex CSR operator (complex128; products on the XCD-split SpMV, scalar
 * recurrences on the device).  The caller-side solve of znaupd's mode 3
 * (SRC/znaupd.f:27: OP = inv[A - sigma M] M, here M = I), which the reference's
 * drivers do with a banded LU (EXAMPLES/COMPLEX/zndrv2.f:179,250 zgttrf/zgttrs).
 * Stops when ||r|| <= rtol ||x|| (r the recursively updated residual) or after
 * maxit iterations.  A solve object serves one stream at a time. */
/* S keeps a reference to A: A must outlive S. */
typedef struct arpack_hip_zshift arpack_hip_zshift;
int arpack_hip_zshift_create(arpack_hip_zshift** S, const arpack_hip_zcsr* A, double sigma_re,
                             double sigma_im, double rtol, int maxit);
void arpack_hip_zshift_destroy(arpack_hip_zshift* S);
/* x, y device pointers (interleaved complex, y != x); synchronous.  Returns the
 * iterations (>= 0; *relres = ||r||/||x||), -1 if BiCGStab broke down or missed
 * rtol within maxit, -2 on a HIP error. */
int arpack_hip_zshift_solve(arpack_hip_zshift* S, const double* x, double* y, double* relres);
/* The solve's method: 0 BiCGStab (the default), 1 a DIRECT solve of a
 * tridiagonal A - sigma I -- LAPACK's zgttrf restated (pivoting by |re| + |im|),
 * once on the host, the two triangular solves as device scans of complex affine
 * maps (csrc/ztri.hip): what EXAMPLES/COMPLEX/zndrv2.f does with zgttrf /
 * zgttrs.  Returns 0, or -1 (unknown method; method 1 with A not tridiagonal or
 * A - sigma I singular: the solve stays BiCGStab). */
int arpack_hip_zshift_set_method(arpack_hip_zshift* S, int method);
/* Totals over the solves so far: solves, iterations, failures, worst final
 * relative residual, device time (ms, hipEvents around each solve) and the
 * algorithmic HBM bytes of one iteration (two CSR products at 20 B a stored
 * entry + rowptr + x/y, plus the fused vector passes). */
int arpack_hip_zshift_stats(const arpack_hip_zshift* S, long long* solves, long long* iters,
                            long long* failures, double* max_relres, double* ms,
                            double* bytes_per_iter);
/* znaupd in mode 3 (iparam[6] = 3, bmat = 'I') with OP = (A - sigma I)^{-1}
 * served on the GPU by S; returns with ido = 99.  A failed solve ends the run
 * with info = -9999. */
void arpack_hip_znaupd_zshift(arpack_hip_zshift* S, int* ido, char const* bmat, int n,
                              char const* which, int nev, double* tol, a_dcomplex* resid, int ncv,
                              a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd,
                              a_dcomplex* workl, int lworkl, double* rwork, int* info);

/* Folded complex Arnoldi steps enqueued so far by this process (free-running
 * znaupd mode 1, ncv <= 40: step j-1's DGKS sweep carried by step j's two
 * passes; AHIP_ZFOLD=0 turns the fold off).  A diagnostic for tests. */
long long arpack_hip_zfold_steps(void);

/* ---- znaupd's generalized modes on the device (bmat = 'G') -------------------
 * The caller's half of znaupd's modes 2-3 (SRC/znaupd.f:23-31; the reference's
 * drivers EXAMPLES/COMPLEX/zndrv3.f and zndrv4.f factor M, or A - sigma M, with
 * zgttrf on the host) served on the GPU: mode 2 OP = inv[M] A, mode 3 OP =
 * inv[A - sigma M] M (complex sigma), B = M.  The inverse is the device
 * BiCGStab (as arpack_hip_zshift) to relative residual rtol on C = A - sigma M,
 * formed once entry by entry over the union pattern (mode 2: on M).  A and M
 * must outlive the pair.  Returns 0, -1 (bad arguments: sizes differ, mode not
 * 2 or 3), -2 (HIP / allocation failure). */
typedef struct arpack_hip_zgen arpack_hip_zgen;
int arpack_hip_zgen_create(arpack_hip_zgen** G, const arpack_hip_zcsr* A, const arpack_hip_zcsr* M,
                           int mode, double sigma_re, double sigma_im, double rtol, int maxit);
void arpack_hip_zgen_destroy(arpack_hip_zgen* G);
/* The inverse's method: 0 BiCGStab (the default), 1 the direct tridiagonal
 * solve of C (zgttrf + device scans, as arpack_hip_zshift_set_method) when A and
 * M are tridiagonal -- zndrv3/zndrv4.f's pairs, which the drivers factor with
 * zgttrf.  0, or -1 (unknown method, C not tridiagonal or singular: the solve
 * stays BiCGStab). */
int arpack_hip_zgen_set_method(arpack_hip_zgen* G, int method);
/* solves, BiCGStab iterations, failed solves, worst final relative residual */
int arpack_hip_zgen_stats(const arpack_hip_zgen* G, long long* solves, long long* iters,
                          long long* failures, double* max_relres);
/* znaupd with bmat = 'G' and iparam[6] = the pair's mode, every OP*x and B*x on
 * the device; returns with ido = 99 (info = -11 when bmat, mode or n do not
 * match the pair; -9999 when a solve misses rtol).  zneupd_c follows as usual
 * (bmat 'G', the pair's sigma). */
void arpack_hip_znaupd_gen(arpack_hip_zgen* G, int* ido, char const* bmat, int n, char const* which,
                           int nev, double* tol, a_dcomplex* resid, int ncv, a_dcomplex* v, int ldv,
                           int* iparam, int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int lworkl,
                           double* rwork, int* info);

/* ---- shift-invert on the device, symmetric (dsaupd mode 3) ------------------
 * y = (A - sigma I)^{-1} x by conjugate gradients (or MINRES, below) on the device CSR operator A
 * (full or symmetric storage), to ||r|| <= rtol ||x|| within maxit iterations:
 * the caller-side solve of dsaupd's mode 3 (SRC/dsaupd.f:30-48), which the
 * reference's EXAMPLES/SYM/dsdrv2.f does with dgttrf/dgttrs.  A - sigma I must be
 * positive definite (sigma below the spectrum of A, the usual smallest-
 * eigenvalue use); an indefinite shift makes CG break down, which is reported
 * as a failed solve.  Returns as arpack_hip_zshift_*. */
/* S keeps a reference to A: A must outlive S (and must not be changed --
 * e.g. arpack_hip_csr_set_symmetric -- while S serves a solve). */
typedef struct arpack_hip_dshift arpack_hip_dshift;
int arpack_hip_dshift_create(arpack_hip_dshift** S, const arpack_hip_csr* A, double sigma,
                             double rtol, int maxit);
void arpack_hip_dshift_destroy(arpack_hip_dshift* S);
/* 0: conjugate gradients (the default; A - sigma I positive definite), 1: MINRES
 * (any symmetric A - sigma I, e.g. sigma inside the spectrum for interior
 * eigenvalues; 16 instead of 11 vector passes an iteration), 2: BiCGStab (a
 * nonsymmetric A: dnaupd's real shift-invert; two products an iteration),
 * 3: a DIRECT solve for a tridiagonal A - sigma I (LAPACK's dgttrf restated,
 * once on the host; the two triangular solves as device scans of affine maps,
 * csrc/dtri.hip) -- what the reference's drivers do (EXAMPLES/NONSYM/dndrv2.f,
 * dsdrv2.f), for operators a Krylov solve cannot serve (dndrv2's).  0, or -1
 * (unknown method; method 3 with A not tridiagonal or A - sigma I singular). */
int arpack_hip_dshift_set_method(arpack_hip_dshift* S, int method);
/* x, y device pointers (y != x); synchronous.  The iterations (>= 0; *relres =
 * ||r||/||x||), -1 on breakdown / missed rtol, -2 on a HIP error. */
int arpack_hip_dshift_solve(arpack_hip_dshift* S, const double* x, double* y, double* relres);
/* Totals: solves, iterations, failures, worst final relative residual, device
 * time (ms) and the algorithmic HBM bytes of one CG iteration (the CSR product
 * in its storage + 11 n-vector passes). */
int arpack_hip_dshift_stats(const arpack_hip_dshift* S, long long* solves, long long* iters,
                            long long* failures, double* max_relres, double* ms,
                            double* bytes_per_iter);
/* dsaupd in mode 3 (iparam[6] = 3, bmat = 'I') with OP = (A - sigma I)^{-1}
 * served on the GPU by S; returns with ido = 99 (dseupd_c with the same sigma
 * then gives the eigenvalues of A).  A failed solve ends the run with
 * info = -9999. */
void arpack_hip_dsaupd_shift(arpack_hip_dshift* S, int* ido, char const* bmat, int n,
                             char const* which, int nev, double* tol, double* resid, int ncv,
                             double* v, int ldv, int* iparam, int* ipntr, double* workd,
                             double* workl, int lworkl, int* info);
/* dnaupd in mode 3 with a real shift (iparam[6] = 3, bmat = 'I'; S set to
 * BiCGStab, method 2); dneupd_c with sigmar = sigma, sigmai = 0 afterwards. */
void arpack_hip_dnaupd_shift(arpack_hip_dshift* S, int* ido, char const* bmat, int n,
                             char const* which, int nev, double* tol, double* resid, int ncv,
                             double* v, int ldv, int* iparam, int* ipntr, double* workd,
                             double* workl, int lworkl, int* info);

/* Generalized modes on the device (bmat = 'G', dsaupd modes 2-5; SRC/dsaupd.f:30-77):
 * the caller's OP and B of the reverse-communication loop, served on the GPU so
 * the solve runs without returning for every OP*x / B*x:
 *   mode 2  OP = inv[M] A,  B = M (and x <- A x)     A = A, B = M
 *   mode 3  OP = inv[A - sigma M] M,  B = M           A = A, B = M
 *   mode 4  OP = inv[K - sigma KG] K, B = K           A = K, B = KG
 *   mode 5  OP = inv[A - sigma M](A + sigma M), B = M
 * The inverse is a device Krylov solve to relative residual rtol (method 0 CG:
 * positive-definite C; 1 MINRES: indefinite; 2 BiCGStab: nonsymmetric; 3 a
 * direct tridiagonal solve, dgttrf + device scans, for a tridiagonal C -- the
 * reference drivers' own dgttrf/dgttrs) on C = A - sigma B formed once
 * entry by entry over the union pattern (mode 2: on M).  Returns 0, -1 for bad
 * arguments, -2 on a HIP failure.  arpack_hip_dsaupd_gen takes dsaupd_c's
 * arguments (bmat 'G', iparam(7) = the operator pair's mode); a solve that
 * misses rtol ends the run with info = -9999. */
typedef struct arpack_hip_dgen arpack_hip_dgen;
int arpack_hip_dgen_create(arpack_hip_dgen** G, const arpack_hip_csr* A, const arpack_hip_csr* B,
                           int mode, double sigma, double rtol, int maxit, int method);
/* dnaupd's complex shifts (SRC/dnaupd.f:28-33; EXAMPLES/NONSYM/dndrv5.f, dndrv6.f):
 * mode 3 OP = Real_Part{inv[A - sigma M] M}, mode 4 OP = Imag_Part{...}, B = M,
 * sigma = (sigmar, sigmai) with sigmai != 0.  C = A - sigma M is formed once in
 * complex arithmetic over the union pattern and solved on the device by the
 * complex BiCGStab (method 0) or, for tridiagonal A and M as dndrv5/6's, the
 * direct tridiagonal solve (method 1: zgttrf + device scans, the drivers' own
 * factorization).  arpack_hip_dnaupd_gen then runs the loop (iparam[6] = mode);
 * dneupd_c takes sigmar, sigmai.  Returns 0, -1 (bad arguments), -2. */
int arpack_hip_dgen_create_cshift(arpack_hip_dgen** G, const arpack_hip_csr* A,
                                  const arpack_hip_csr* M, int mode, double sigmar, double sigmai,
                                  double rtol, int maxit, int method);
void arpack_hip_dgen_destroy(arpack_hip_dgen* G);
int arpack_hip_dgen_stats(const arpack_hip_dgen* G, long long* solves, long long* iters,
                          long long* fails, double* max_relres);
void arpack_hip_dsaupd_gen(arpack_hip_dgen* G, int* ido, char const* bmat, int n, char const* which,
                           int nev, double* tol, double* resid, int ncv, double* v, int ldv,
                           int* iparam, int* ipntr, double* workd, double* workl, int lworkl,
                           int* info);
/* dnaupd_c's generalized modes on the device (replaces the caller's ido = -1 /
 * 1 / 2 loop of EXAMPLES/NONSYM/dndrv3.f:215-255 and dndrv4.f:243-310; SRC/
 * dnaupd.f:18-33): A nonsymmetric, M symmetric positive semi-definite, and
 *   mode 2  OP = inv[M] A, B = M (no write-back of A x, unlike dsaupd's)
 *   mode 3  OP = inv[A - sigma M] M, B = M, sigma real (method 2 BiCGStab on
 *           the nonsymmetric C); dneupd_c with sigmar = sigma, sigmai = 0.
 * Modes 4 (Im part, complex sigma) and the operator pair's modes 4-5 return
 * info = -11. */
void arpack_hip_dnaupd_gen(arpack_hip_dgen* G, int* ido, char const* bmat, int n, char const* which,
                           int nev, double* tol, double* resid, int ncv, double* v, int ldv,
                           int* iparam, int* ipntr, double* workd, double* workl, int lworkl,
                           int* info);

/* ---- multi-GPU (row-block sharding, PARPACK's decomposition) ----------------
 * Reference: ICB/parpack.h:17-33 (pdsaupd_c(MPI_Fint comm, ...), n = LOCAL
 * rows) and PARPACK/SRC/MPI/pdsaitr.f.  One process per GPU; the communicator
 * is RCCL (NCCL_UNIQUE_ID_BYTES = 128-byte id created by rank 0 and broadcast
 * by the launcher). */
int arpack_hip_comm_unique_id(char* id128);
int arpack_hip_comm_init(int nranks, int rank, const char* id128, int device);
void arpack_hip_comm_destroy(void);
int arpack_hip_comm_rank(void);
int arpack_hip_comm_size(void);
int arpack_hip_comm_allreduce(double* dev, int count); /* in-place SUM (test hook) */
/* Nonzero once a collective of the engine's communicator failed (an RCCL call
 * returned an error, RCCL reported an asynchronous error, or a HIP copy of the
 * host-staged transport failed).  The solve entry points then return with
 * info = -9999 at their next return to the caller on every rank whose
 * communicator saw the failure. */
int arpack_hip_comm_failed(void);
/* Host-staged transport in place of RCCL: the engine stages every allreduce
 * (in-place SUM of `count` host doubles) and every point-to-point group of the
 * distributed SpMV through the launcher's own collectives.  A group is `nops`
 * transfers: op k sends count[k] doubles from buf[k] to rank peer[k]
 * (is_send[k] = 1) or receives count[k] doubles from peer[k] into buf[k]
 * (is_send[k] = 0); the callback posts them all non-blocking and returns when
 * every one has completed (between one pair of ranks, transfers in one
 * direction match in posting order, as MPI / gloo guarantee).  The groups are
 * exactly the ones RCCL runs (the same device slices, counts and offsets:
 * neighbour halos, the symmetric form's spill, ghost lists, the all-gather), so
 * rehearsing P ranks where RCCL cannot run them (several ranks on one GPU; CI)
 * exercises the whole data path apart from the wire. */
typedef void (*arpack_hip_host_allreduce_fn)(double* buf, int count, void* ctx);
typedef void (*arpack_hip_host_p2p_fn)(int nops, const int* peer, const int* is_send,
                                       double* const* buf, const int64_t* count, void* ctx);
int arpack_hip_comm_init_host(int nranks, int rank, arpack_hip_host_allreduce_fn allreduce,
                              arpack_hip_host_p2p_fn p2p, void* ctx, int device);

typedef struct arpack_hip_dist arpack_hip_dist;
/* Distributed operator from this rank's CSR rows [row0, row0 + A.n) with GLOBAL
 * column indices: computes the halo plan with the other ranks (collective) and
 * remaps A's columns to the local extended-x layout.  A banded operator (every
 * rank's columns within its neighbours' rows) exchanges slab halos with the
 * neighbours; any other operator gets per-peer ghost lists (each rank receives
 * exactly the off-block x entries its rows read: grouped send / recv), or,
 * where the ghosts exceed half of the off-block rows, an all-gather of x.
 * Returns 0; -3 if the row blocks are not contiguous; -1 on every rank if any
 * rank fails to set up.  A CSR declared symmetric before this call keeps
 * symmetric storage only for a banded operator, if every rank declared it and
 * every rank's symmetric plan succeeds; otherwise all ranks run full storage. */
int arpack_hip_dist_create(arpack_hip_dist** D, arpack_hip_csr* A, int64_t n_global, int64_t row0);
void arpack_hip_dist_destroy(arpack_hip_dist* D);
/* y = A x on this rank's rows (device pointers), collective over the ranks:
 * halo exchange + local SpMV (+ the forward spill exchange when the local CSR
 * was declared symmetric with arpack_hip_csr_set_symmetric). */
int arpack_hip_dist_spmv(const arpack_hip_dist* D, const double* x, double* y);
int arpack_hip_dist_info(const arpack_hip_dist* D, int64_t* halo_lo, int64_t* halo_hi,
                         int64_t* send_lo, int64_t* send_hi);
/* Exchange form: 0 neighbour halos, 1 ghost lists (halo_hi = ghosts), 2
 * all-gather (halo_lo / halo_hi = the rows before / after this rank's). */
int arpack_hip_dist_mode(const arpack_hip_dist* D);
// 1: the block's symmetric-storage SpMV sends its transposed terms for the next
// rank's leading rows forward as a spill exchange after the SpMV, under
// AHIP_DIST_SPILL=1 or a structurally unsymmetric coupling; 0: no spill -- full
// storage, or the spill-free symmetric form: one two-sided halo, the leading
// rows' lower ghost terms from the rank's own rows; -1: no operator.
int arpack_hip_dist_spill(const arpack_hip_dist* D);
/* Row-block decomposition without an operator: rank owns rows [row0, row0+nloc)
 * of the global n_global (collective-free; needs arpack_hip_comm_init). */
int arpack_hip_dist_rows(arpack_hip_dist** D, int64_t nloc, int64_t row0, int64_t n_global);
/* PARPACK-style reverse communication (ICB/parpack.h:20 pdsaupd_c, :26 pdnaupd_c
 * with n = LOCAL rows): every rank calls collectively; at ido = -1/1 the caller
 * applies OP to its local slice (its own halo exchange), as in
 * PARPACK/EXAMPLES/MPI/pdsdrv1.f.  Post-processing: arpack_hip_pdseupd_c
 * (ICB/parpack.h:21; collective B-norm for bmat = 'G', PARPACK/SRC/MPI/pdseupd.f:456)
 * and arpack_hip_pdneupd_c (ICB/parpack.h:27; no collective). */
void arpack_hip_pdsaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, double tol, double* resid, int ncv,
                          double* v, int ldv, int* iparam, int* ipntr, double* workd,
                          double* workl, int lworkl, int* info);
void arpack_hip_pdnaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, double tol, double* resid, int ncv,
                          double* v, int ldv, int* iparam, int* ipntr, double* workd,
                          double* workl, int lworkl, int* info);
void arpack_hip_pdseupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, double* d, double* z, int ldz, double sigma,
                          char const* bmat, int n, char const* which, int nev, double tol,
                          double* resid, int ncv, double* v, int ldv, int* iparam,
                          int* ipntr, double* workd, double* workl, int lworkl, int* info);
void arpack_hip_pdneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, double* dr, double* di, double* z, int ldz,
                          double sigmar, double sigmai, double* workev, char const* bmat, int n,
                          char const* which, int nev, double tol, double* resid, int ncv,
                          double* v, int ldv, int* iparam, int* ipntr, double* workd,
                          double* workl, int lworkl, int* info);
/* The same for the other families of ICB/parpack.h: fp32 symmetric / nonsymmetric
 * (pssaupd_c :17, psseupd_c :18, psnaupd_c :23, psneupd_c :24) and complex
 * (pcnaupd_c :29, pcneupd_c :30, pznaupd_c :32, pzneupd_c :33).  The complex
 * engine on a row block takes its host-driven Arnoldi step with allreduced
 * inner products (PARPACK/SRC/MPI/pznaitr.f); p*neupd need no collective. */
void arpack_hip_pssaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, float tol, float* resid, int ncv, float* v,
                          int ldv, int* iparam, int* ipntr, float* workd, float* workl,
                          int lworkl, int* info);
void arpack_hip_psseupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, float* d, float* z, int ldz, float sigma,
                          char const* bmat, int n, char const* which, int nev, float tol,
                          float* resid, int ncv, float* v, int ldv, int* iparam, int* ipntr,
                          float* workd, float* workl, int lworkl, int* info);
void arpack_hip_psnaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, float tol, float* resid, int ncv, float* v,
                          int ldv, int* iparam, int* ipntr, float* workd, float* workl,
                          int lworkl, int* info);
void arpack_hip_psneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, float* dr, float* di, float* z, int ldz,
                          float sigmar, float sigmai, float* workev, char const* bmat, int n,
                          char const* which, int nev, float tol, float* resid, int ncv, float* v,
                          int ldv, int* iparam, int* ipntr, float* workd, float* workl,
                          int lworkl, int* info);
void arpack_hip_pznaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, double tol, a_dcomplex* resid, int ncv,
                          a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd,
                          a_dcomplex* workl, int lworkl, double* rwork, int* info);
void arpack_hip_pzneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, a_dcomplex* d, a_dcomplex* z, int ldz,
                          a_dcomplex sigma, a_dcomplex* workev, char const* bmat, int n,
                          char const* which, int nev, double tol, a_dcomplex* resid, int ncv,
                          a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd,
                          a_dcomplex* workl, int lworkl, double* rwork, int* info);
void arpack_hip_pcnaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, float tol, a_fcomplex* resid, int ncv,
                          a_fcomplex* v, int ldv, int* iparam, int* ipntr, a_fcomplex* workd,
                          a_fcomplex* workl, int lworkl, float* rwork, int* info);
void arpack_hip_pcneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, a_fcomplex* d, a_fcomplex* z, int ldz,
                          a_fcomplex sigma, a_fcomplex* workev, char const* bmat, int n,
                          char const* which, int nev, float tol, a_fcomplex* resid, int ncv,
                          a_fcomplex* v, int ldv, int* iparam, int* ipntr, a_fcomplex* workd,
                          a_fcomplex* workl, int lworkl, float* rwork, int* info);
/* Start vector of info = 0 on a distribution: mode 0 (default) draws one dlarnv
 * stream and gives each rank its rows' slice, so every rank count sees the
 * single-GPU iterates; mode 1 is PARPACK's: each rank draws its local rows from
 * its own process-persistent stream seeded with the digits of 1000 + 2 rank + 1
 * (PARPACK/SRC/MPI/pdgetv0.f:234-245), as libparpack_hip.so sets it. */
int arpack_hip_dist_set_seed_mode(arpack_hip_dist* D, int mode);
/* Halo plan (host only, CPU-testable): tab = [row0, nloc, min col, max col] per
 * rank (4*P doubles, global indices); out = {halo_lo, halo_hi, send_lo, send_hi}
 * of rank r.  Returns 0, -3 (blocks not contiguous) or -4 (halo too wide). */
int arpack_hip_kit_halo_plan(int P, int r, const double* tab, int64_t* out);
/* Host half of arpack_hip_csr_set_symmetric's analysis (no GPU): the symmetric
 * superblock plan from each row's largest upper column cmax[i] for an LDS
 * window of `win` columns; spill_in / spill_out: rows reached from / into the
 * neighbouring ranks (0 on one GPU).  Writes *nsb, r0s[0..nsb] (row bounds), spans[0..nsb)
 * (window lengths) and pre[0..nsb) (leading rows combined with the previous
 * superblock's spill); the caller sizes the arrays n + 1.  -1 if the matrix
 * does not fit (a row wider than the window, or a spill past the next
 * superblock). */
int arpack_hip_kit_symsell_plan(int64_t n, const int32_t* cmax, int win, int64_t spill_in,
                                int64_t spill_out, int64_t* nsb, int64_t* r0s, int32_t* spans,
                                int32_t* pre);
/* Distributed free-running dsaupd (n = LOCAL rows, device arrays), cycle-parked
 * like arpack_hip_dsaupd_csr_cycles.  All ranks call it collectively. */
void arpack_hip_pdsaupd_csr_cycles(const arpack_hip_dist* D, int max_cycles, int* ido,
                                   char const* bmat, int n, char const* which, int nev,
                                   double* tol, double* resid, int ncv, double* v, int ldv,
                                   int* iparam, int* ipntr, double* workd, double* workl,
                                   int lworkl, int* info);
void arpack_hip_pdnaupd_csr_cycles(const arpack_hip_dist* D, int max_cycles, int* ido,
                                   char const* bmat, int n, char const* which, int nev,
                                   double* tol, double* resid, int ncv, double* v, int ldv,
                                   int* iparam, int* ipntr, double* workd, double* workl,
                                   int lworkl, int* info);

/* Per-kernel-class device timing with hipEvents on the launch stream.
 * Classes: 0 SpMV, 1 CGS dots, 2 update(+fused DGKS dots), 3 V*Q, 4 place,
 * 5 finalize, 6 other.  read() synchronises and resets; returns #classes. */
/* Test hook: the k-th checked HIP call of the engine from now on (copies,
 * syncs and plan-table uploads of the solve, post-processing and CSR plan
 * paths) reports hipErrorInvalidValue; the solve then returns info = -9999 and
 * a CSR create -2.  k <= 0 disarms.  AHIP_FAULT_AT=k arms it at load. */
void arpack_hip_fault_inject(long k);
/* Test hook standing in for a caller's own in-flight GPU work: on a private
 * non-blocking stream, a kernel waits `delay_us` microseconds (device wall
 * clock) and then writes count doubles dst[k] = src[k] (src == NULL: value).
 * Returns at once (0), without waiting for the kernel. */
int arpack_hip_test_delayed_fill(double* dst, const double* src, double value, int64_t count,
                                 int delay_us);
/* Test hook (the fused symmetric SpMV's cross-workgroup hand-off): y = A x on a
 * CSR declared symmetric, with the in-kernel chain-head combine (fuse = 1, the
 * one-GPU default) or the separate combine launch (fuse = 0), issued while a
 * read / write stream over `load` (load_n doubles; may be NULL) runs on a
 * second stream.  Writes the chain-head row ranges as (first row, count)
 * pairs into heads (at most cap) and, when lo_out (host, n doubles) is given,
 * the slot halves those rows read from the previous chain into lo_out at
 * their rows.  Returns the number of ranges, or < 0. */
int arpack_hip_test_symspmv_handoff(const arpack_hip_csr* A, const double* x, double* y, int fuse,
                                    double* load, int64_t load_n, int64_t* heads, int64_t cap,
                                    double* lo_out);
/* Deterministic mode: every SpMV sum independent of the wave schedule, so a
 * solve is bitwise reproducible run to run.  A later
 * arpack_hip_csr_set_symmetric(A, 1) selects the symmetric kernel's
 * fixed-point form (transposed terms summed as exact 64-bit integers; the
 * default kernel's rate) and returns 0, or keeps the full-storage kernel
 * (bitwise SciPy's csr_matvec) and returns 1 for an operator outside that
 * form; the complex operator's column-sorted tiles take their fixed-point
 * form (else the column-split kernel).  Products of operators already
 * declared symmetric follow the switch when they run: the fixed-point form
 * where it serves the operator (on every rank of a distributed one), else the
 * full-storage kernel over the still-resident full CSR.  Off by default
 * (ARPACK_HIP_DETERMINISTIC=1 in the environment: on, read at first use). */
void arpack_hip_set_deterministic(int on);
int arpack_hip_deterministic(void);
void arpack_hip_profile(int enable);
int arpack_hip_profile_read(double* ms, double* bytes, long long* count, int nclass);

/* Synthetic operators generated directly in HBM (bench/test workloads, see
 * DESIGN.md §5).  Each allocates device CSR arrays owned by *A. */
int arpack_hip_gen_laplace2d(arpack_hip_csr** A, int64_t m, double scale);
/* 2-D convection-diffusion -Lap u + rho du/dx, m x m interior grid
 * (EXAMPLES/NONSYM/dndrv1.f:397-475; complex spectrum once rho*h/2 > 1). */
int arpack_hip_gen_convdiff2d(arpack_hip_csr** A, int64_t m, double rho);
int arpack_hip_gen_laplace3d(arpack_hip_csr** A, int64_t m, double scale);
/* Rows [row_begin, row_end) of the m^3 7-pt Laplacian with global columns: one
 * rank's z-slab block of BASELINE config 4 (the row-block decomposition of
 * PARPACK/EXAMPLES/MPI/pdsdrv1.f:429-480), bit-identical to those rows of
 * arpack_hip_gen_laplace3d; -1 on an empty or out-of-range block. */
int arpack_hip_gen_laplace3d_rows(arpack_hip_csr** A, int64_t m, int64_t row_begin, int64_t row_end,
                                  double scale);
int arpack_hip_gen_anderson(arpack_hip_csr** A, int64_t m, int dim, double disorder, uint32_t seed);
int arpack_hip_gen_banded_sym(arpack_hip_csr** A, int64_t n, int64_t row_begin,
                              int64_t row_end, uint32_t seed, int bandwidth, int per_row);
/* Copy a registered CSR back to host buffers (sizes from arpack_hip_csr_info). */
/* SELL-64 layout statistics (slices, stored entries incl. padding); -1 if not built */
int arpack_hip_csr_sell_info(const arpack_hip_csr* A, int64_t* nslices, int64_t* padded);
int arpack_hip_csr_info(const arpack_hip_csr* A, int64_t* n, int64_t* nnz);
int arpack_hip_csr_download(const arpack_hip_csr* A, int64_t* rowptr, int32_t* col, double* val);

/* Host-side small-dense kit exports (CPU-testable, no GPU needed). */
int arpack_hip_kit_dstqrb(int n, double* d, double* e, double* z, double* work);
int arpack_hip_kit_dsteqr(int n, double* d, double* e, double* z, int ldz, double* work);
void arpack_hip_kit_dlartg(double f, double g, double* c, double* s, double* r);
void arpack_hip_kit_dsortr(char const* which, int apply, int n, double* x1, double* x2);
void arpack_hip_kit_dsapps_host(int kev, int np, const double* shift, double* h, int ldh,
                                double* q, int ldq);
void arpack_hip_kit_dlarnv(int* iseed, int n, double* x);
void arpack_hip_kit_slarnv(int* iseed, int n, float* x); /* slarnv(idist=2), LAPACK slaruv rules */
/* LAPACK dgttrf / dgttrs (trans 'N', one right-hand side) restated: the host
 * factor behind arpack_hip_dshift_set_method(S, 3) and its sequential solve
 * (tests/test_kit_tri.py against the image's LAPACK).  dgttrf returns LAPACK's
 * info (0, or k > 0 for a zero pivot u(k,k)); ipiv is 0-based (LAPACK's
 * ipiv minus one). */
int arpack_hip_kit_dgttrf(int64_t n, double* dl, double* d, double* du, double* du2, int* ipiv);
void arpack_hip_kit_dgttrs(int64_t n, const double* dl, const double* d, const double* du,
                           const double* du2, const int* ipiv, double* b);
/* zgttrf / zgttrs likewise (complex arrays interleaved re, im; pivoting by CABS1) */
int arpack_hip_kit_zgttrf(int64_t n, double* dl, double* d, double* du, double* du2, int* ipiv);
void arpack_hip_kit_zgttrs(int64_t n, const double* dl, const double* d, const double* du,
                           const double* du2, const int* ipiv, double* b);
/* The device generators behind dgetv0/sgetv0's start vector on a device buffer
 * x (prec 'd': double, 's': float); iseed is advanced like dlarnv/slarnv's. */
int arpack_hip_larnv_device(char prec, int* iseed, int64_t n, void* x);
/* nonsymmetric kit (restated LAPACK dlahqr/dtrevc/dlanv2/dnrm2 and ARPACK
 * dsortc/dngets/dneigh/dnapps; compared against SRC/dsortc.f, dngets.f,
 * dneigh.f, dnapps.f and the image's LAPACK in tests/test_kit_ns.py) */
double arpack_hip_kit_dnrm2(int n, const double* x);
void arpack_hip_kit_dlanv2(double* a, double* b, double* c, double* d, double* rt1r,
                           double* rt1i, double* rt2r, double* rt2i, double* cs, double* sn);
int arpack_hip_kit_dlahqr(int wantt, int wantz, int n, int ilo, int ihi, double* h, int ldh,
                          double* wr, double* wi, int iloz, int ihiz, double* z, int ldz);
int arpack_hip_kit_dtrevc(char howmny, int* select, int n, const double* t, int ldt, double* vr,
                          int ldvr, double* work);
void arpack_hip_kit_dsortc(char const* which, int apply, int n, double* xr, double* xi, double* y);
void arpack_hip_kit_dngets(int ishift, char const* which, int* kev, int* np, double* ritzr,
                           double* ritzi, double* bounds);
int arpack_hip_kit_dneigh(double rnorm, int n, const double* h, int ldh, double* ritzr,
                          double* ritzi, double* bounds, double* q, int ldq, double* workl);
int arpack_hip_kit_dtrsen(const int* select, int n, double* t, int ldt, double* q, int ldq,
                          double* wr, double* wi, int* m); /* job='N', compq='V' */
/* complex kit (zdense.cpp; tests/test_kit_z.py) */
int arpack_hip_kit_zlahqr(int n, a_dcomplex* h, int ldh, a_dcomplex* w, a_dcomplex* z, int ldz);
int arpack_hip_kit_ztrevc(char howmny, int* select, int n, a_dcomplex* t, int ldt, a_dcomplex* vr,
                          int ldvr);
int arpack_hip_kit_ztrsen(const int* select, int n, a_dcomplex* t, int ldt, a_dcomplex* q, int ldq,
                          a_dcomplex* w, int* m);
void arpack_hip_kit_zsortc(char const* which, int apply, int n, a_dcomplex* x, a_dcomplex* y);
void arpack_hip_kit_zngets(int ishift, char const* which, int kev, int np, a_dcomplex* ritz,
                           a_dcomplex* bounds);
int arpack_hip_kit_zneigh(double rnorm, int n, const a_dcomplex* h, int ldh, a_dcomplex* ritz,
                          a_dcomplex* bounds, a_dcomplex* q, int ldq);
void arpack_hip_kit_znapps_host(int kev, int np, const a_dcomplex* shift, a_dcomplex* h, int ldh,
                                a_dcomplex* q, int ldq, int64_t nglob);
int arpack_hip_kit_dnapps_host(int kev, int np, const double* shiftr, const double* shifti,
                               double* h, int ldh, double* q, int ldq, double* workl,
                               int64_t nglob);

#ifdef __cplusplus
}
#endif
#endif /* ARPACK_HIP_H */
