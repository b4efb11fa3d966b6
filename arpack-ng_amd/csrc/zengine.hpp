// Complex (znaupd family) engine: device workspace, complex CSR operator and
// the ZSolver coroutine (zsolver.cpp).  The complex path keeps the shared
// Arrays mirror (n complex = 2n doubles) and drives its step decisions from
// the host: config 5 is shift-invert, where the caller's solve dominates.
#pragma once
#include <hip/hip_runtime.h>

#include <complex>
#include <cstdint>
#include <optional>
#include <vector>

#include "engine.hpp"
#include "zdense.hpp"

namespace ahip {

struct Comm;
namespace zdev {
struct ZGen;
struct Ws {
    hipStream_t stream = nullptr;
    // row-distributed solve: every reduction of `dots` is allreduced over the
    // ranks before it reaches the host (PARPACK/SRC/MPI/pznaitr.f's MPI_ALLREDUCEs)
    const Comm* comm = nullptr;
    // the owning solve's sticky error record (nullptr: unchecked)
    DevErr* err = nullptr;
    void ck(hipError_t e) const {
        if (err) err->ck(e);
    }
    int nblk = 0;
    double* part = nullptr;  // 2*(ncv+2) slots x nblk
    double* sums = nullptr;
    double* coef = nullptr;  // complex coefficients (h) staged for the update
    double* q = nullptr;     // complex ncv x ncv (V*Q, eupd)
    double* host = nullptr;  // pinned
    double* scratch = nullptr;  // ncv > 64: nblk * kB * ncv complex (k_zgemm_generic)
    // device-resident Arnoldi step (zstep.hip, bmat = 'I'): the decisions'
    // state, the coefficient vectors (4 x cstride complex: CGS, DGKS-1, DGKS-2
    // and the fold's t = H s -- slot 0 also stages the host-driven update's h),
    // the recorded columns h(1:j,j) (hld = ncv) and the subdiagonals h(j,j-1)
    // per step
    dev::LzState* st = nullptr;
    dev::LzState* st_host = nullptr;  // pinned mirror
    int cstride = 0;
    double* hcol = nullptr;  // ncv x ncv complex
    int hld = 0;
    double* rec = nullptr;   // ncv + 1
};
// widest basis of the device-resident complex step: its finalize keeps 2 doubles
// per complex slot (j + 1 <= ncv + 1 slots) in dynamic LDS next to ~100 B of
// static state, within the 64 KB a workgroup may allocate
constexpr int kMaxDevStepNcv = 4000;
// The split operator's partial products s_y belong to the operator: one SpMV
// at a time per ZCsr (the engine's stream); concurrent SpMVs on the same ZCsr
// from different streams need separate operators.
struct ZCsr {
    int64_t n = 0, nnz = 0;
    const int64_t* rowptr = nullptr;
    const int32_t* col = nullptr;
    const double* val = nullptr;  // interleaved complex
    bool owned = false;
    // XCD column split (zsplit.hip, zcsr_build_split): the columns cut into s_n
    // slices of sw; slice s's entries as a CSR of their own (int32 row offsets
    // s_rp[s*(n+1) + r] relative to s_base[s]), slice-relative columns (16 bit
    // when sw <= 65536), partial products y_s in s_y (s_n x n complex)
    bool split = false;
    int s_n = 8;  // column slices: 4 or 8 (zcsr_build_split)
    int64_t s_w = 0;
    bool s_col16 = true;
    int32_t* s_rp = nullptr;
    int64_t* s_base = nullptr;  // 9 (device)
    void* s_col = nullptr;
    double* s_val = nullptr;
    double* s_y = nullptr;
    // column-sorted tiles (zsplit.hip, default when the slice width < 2^20): the
    // entries of each (row block of kTileRows rows, slice) sorted by column,
    // segment q = slice * t_nrb + row block at [t_seg[q], t_seg[q + 1]); t_idx:
    // uint32 row_local << 20 | slice column (20 B an entry with the value), or
    // packed (t_pk): uint16 row_local << 4 | column step in the 64-entry chunk,
    // t_cbase[chunk] its first column (18.06 B an entry; t_stored entries incl.
    // zero-valued fillers and chunk padding)
    bool tile = false;
    bool t_pk = false;
    int64_t t_nrb = 0;
    int64_t t_stored = 0;
    int64_t* t_seg = nullptr;
    void* t_idx = nullptr;
    int32_t* t_cbase = nullptr;
    double* t_val = nullptr;
    // deterministic mode's tile form (k_ztile_det: the row sums as 64-bit
    // fixed-point integers): per-(slice, row block) largest |re|, |im| of the
    // entries (s_n x t_nrb), 256 block maxima of the bits of |x| of the
    // product in flight, B bits a term; t_det = 1 when the operator fits
    double* t_amax = nullptr;
    unsigned long long* t_xmax = nullptr;
    int t_bits = 0;
    int t_det = 0;
};
// Build the XCD column split of A when it pays (n >= 2^18: x larger than one
// XCD's L2; >= 32 entries a row: the partials' 256 B a row stay small against
// the row's stream); AHIP_ZSPLIT=0 disables.  0: built, 1: not applicable, < 0: error.
int zcsr_build_split(ZCsr& A);
void zcsr_free_split(ZCsr& A);
// algorithmic HBM bytes of the split product's matrix stream (values + the
// entry encoding: 20 B an entry, or the packed tiles' 18 B + a base column per
// 64-entry chunk over the stored entries)
double zcsr_split_matrix_bytes(const ZCsr& A);
// y = A x through the split (8 slice launches in one grid + the fixed-order combine);
// gate (device int, may be null): the kernels return at once while *gate != 0
void zcsr_split_spmv(hipStream_t s, const ZCsr& A, const double* x, double* y,
                     const int* gate = nullptr);
// The slice products alone (no combine): y_s = A(:, slice s) x into A.s_y (s_n x
// n complex, slice-major), for a caller that sums them in zc::slice_sum's order
// inside its own pass (zsolve.hip).  Returns A.s_y; nullptr (nothing launched)
// when A is not split.
const double* zcsr_split_partials(hipStream_t s, const ZCsr& A, const double* x,
                                  const int* gate = nullptr);
hipError_t ws_create(Ws& ws, int64_t n, int ncv, hipStream_t s);
void ws_destroy(Ws& ws);
// Launchers over the component type R of the interleaved complex vectors
// (double: complex128, z*; float: complex64, c*); arithmetic in complex128.
// out[c] = V(:,c)^H u for c < j; out[j] = w^H u if w
template <class R>
void dots(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, const R* u, const R* w,
          std::complex<double>* out);
// rout = rin - V(:,0:j) h
template <class R>
void update(const Ws& ws, int64_t n, int j, const R* V, int64_t ld,
            const std::complex<double>* h, const R* rin, R* rout);
// Z(:,0:nz) = V(:,0:k) M (k x nz); Z may alias V
template <class R>
void gemm(const Ws& ws, int64_t n, const R* V, int64_t ld, int k, int nz,
          const std::complex<double>* M, R* Z, int64_t ldz);
// y = a*y + b*x (x may be null)
template <class R>
void axpby(const Ws& ws, int64_t n, std::complex<double> a, R* y, std::complex<double> b,
           const R* x);
// Z(:,c) += x * w[c]
template <class R>
void ger(const Ws& ws, int64_t n, int k, const R* x, const std::complex<double>* w, R* Z,
         int64_t ldz);
// device-resident step (zstep.hip): v_j = r/rnorm (+ copy), partials of
// [V(:,0:j)^H u ; u^H u], r = rin - V coef[which] (+ partials of [V^H r ; r^H r]),
// the single-block finalize of m complex slots, r = 0 if st.zero
template <class R>
void step_place(const Ws& ws, int64_t n, const R* r, R* vcol, R* copy1, R* copy2, double safmin,
                int j);
template <class R>
void step_dots(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, const R* u, int gate);
template <class R>
void step_update(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, int which, const R* rin,
                 R* rout, bool spec, int gate);
void step_finalize(const Ws& ws, int m, dev::FinPhase ph, int j, int rstart, int gate);
// folded step j (zstep.hip; free-running znaupd mode 1, complex128): r' and
// A r' from the raw residual r and y = A r, the CGS sums (k_zfold_dots), then
// v_j, r_j and the next sweep's sums (k_zfold_update); j - 1 <= kZFoldMax
constexpr int kZFoldMax = 39;
void step_fold_dots(const Ws& ws, int64_t n, int j, const double* V, int64_t ld, const double* r,
                    const double* y);
void step_fold_update(const Ws& ws, int64_t n, int j, double* V, int64_t ld, const double* y,
                      double* r);
template <class R>
void step_zero_if(const Ws& ws, int64_t n, R* r);
void zcsr_spmv(hipStream_t s, const ZCsr& A, const double* x, double* y, const int* gate = nullptr);
int gen_zrandom(ZCsr& A, int64_t n, int per_row, uint32_t seed, double dshift);
}  // namespace zdev

// R: component type of the n-length complex data (double: znaupd, float:
// cnaupd); the ncv-sized host work is complex128 in both (workl shadow for c*).
template <class R>
class ZSolverT {
public:
    using cd = std::complex<double>;
    char bmat = 'I';
    la::Which which = la::Which::LM;
    int n = 0, ncv = 0, mode = 1, ishift = 1, mxiter = 0, nev0 = 0, np = 0, lworkl = 0;
    double tol = 0.0;
    int* iparam = nullptr;
    int* ipntr = nullptr;
    cd* workl = nullptr;
    double* rwork = nullptr;
    int info = 0;
    int ih = 0, iritz = 0, ibounds = 0, iq = 0, iw = 0;
    double rnorm = 0.0;

    ArraysT<R> a;  // n complex = 2n reals; offsets below are in complex units
    std::vector<cd> wshadow;  // c*: complex128 shadow of the caller's workl
    zdev::Ws ws;
    RciCtx ctx;
    std::optional<Task> root;
    const zdev::ZCsr* csr = nullptr;  // free-running OP (mode 1)
    zdev::ZGen* gen = nullptr;        // generalized modes: OP and B on the device (zgen.cpp)
    const DistOp* dist = nullptr;      // row block of a distributed solve (or null)
    uint64_t dist_gen = 0;             // generation of dist->comm when the solve started
    int64_t row0 = 0, n_global = 0;
    const R* op_x = nullptr;
    R* op_y = nullptr;

    ~ZSolverT();
    Task run();  // znaup2
    // failed HIP call of this solve -> info = -9999, agreed across the ranks of
    // a distribution once per restart cycle (see SolverT::check_halt)
    bool halted = false;
    bool check_halt();

private:
    Task getv0(bool initv, int j, int itry, int& ierr);
    Task naitr(int k, int npk, int& iinfo);
    RciAwait rci(int ido, int64_t x, int64_t y, int64_t bx = -1);
    RciAwait op(int ido, int64_t x, int64_t y, int64_t bx);
    // free-running OP on a device vector that is not a workd slice (the folded
    // step's raw residual)
    RciAwait op_raw(R* x, int64_t y);
    R* col(int j) { return a.d_v + (int64_t)(j - 1) * a.d_ld; }  // 1-based, reals
    R* wd(int64_t off) { return a.d_workd + 2 * off; }           // complex offset
    int64_t ldc() const { return a.d_ld / 2; }                    // ld in complex units
    double cnorm(const R* x);                                     // dznrm2 on device
    // device-resident step path (bmat = 'I', zstep.hip)
    Task naitr_dev(int k, int npk, int& iinfo);
    void dgks2_tail(int j, int rstart);
    void read_state();
    void write_state();
};
using ZSolver = ZSolverT<double>;

}  // namespace ahip
