// Device (HBM-resident) half of the engine: launchers for the n-length kernels.
//
// Data layout in HBM:
//   V      n x ncv, column-major, leading dimension ld (the caller's ldv in
//          device-pointer mode, n rounded up to a multiple of 2 in host mode)
//   resid  n, workd 3n (ARPACK slices ipj=0, irj=n, ivj=2n)
//   part   nblk x stride doubles: per-block partial sums of the two-stage,
//          fixed-order (hence bitwise reproducible) reductions
//   LzState  the device-resident scalar state of the current Lanczos step:
//          the DGKS decision (rnorm vs 0.717*wnorm, SRC/dsaitr.f:656,753) is
//          taken ON THE DEVICE by the finalize kernel, so a whole restart
//          cycle can be enqueued without a host round trip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ahip {

// Test hook (arpack_hip_fault_inject): the k-th checked HIP call from now on
// reports hipErrorInvalidValue (the call itself was issued); 0 disarms.
hipError_t fault_filter(hipError_t e);
void fault_inject(long k);

// Deterministic mode (arpack_hip_set_deterministic, ARPACK_HIP_DETERMINISTIC=1):
// only SpMV forms whose every sum has a fixed order -- a symmetric declaration
// takes the upper-triangle kernel's fixed-point form (k_csr_ssell_det: the
// transposed terms as exact 64-bit integer sums, whose order cannot matter),
// or, for an operator outside that form, keeps the full-storage SELL kernel
// (bitwise SciPy's csr_matvec); the complex operator takes the column-split
// kernel instead of the LDS-atomic row tiles.  The rest of the engine
// (fixed-order partial sums) is deterministic in either mode.
bool deterministic();
void set_deterministic(bool on);

// Sticky device-error record of one solve: the first failed HIP call (an
// enqueue, a copy, or a kernel fault surfacing at a stream sync) is kept, and
// the driver turns it into info = -9999 at its next return to the caller
// instead of running the restart loop on stale state.
struct DevErr {
    hipError_t e = hipSuccess;
    void ck(hipError_t r) {
        r = fault_filter(r);
        if (r != hipSuccess && e == hipSuccess) e = r;
    }
    bool bad() const { return e != hipSuccess; }
};

}  // namespace ahip

namespace ahip::dev {

constexpr int kBlock = 256;
// largest ncv the engine accepts (the finalize stages ncv + 2 sums in 64 KB of
// dynamic LDS); a larger ncv is rejected with info = -3 like ncv > n
constexpr int kMaxNcv = 8000;
constexpr int kMaxRedBlocks = 1024;  // partial-sum grid (A/B: 1024 vs 2048 +1.5% cycle rate with the fused finalize)

// XCD-contiguous block order: the hardware deals workgroups round-robin over
// the 8 XCDs, so logical block xcd_block(b) makes each XCD walk one contiguous
// range of superblocks (its 4 MB L2 then serves overlapping window loads).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    constexpr int64_t X = 8;
    const int64_t q = nb / X, r = nb % X, x = b % X, i = b / X;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// Scalar state of the current step j (device memory).
struct LzState {
    double rnorm;   // B-norm of the current residual (beta of the next step)
    double wnorm;   // B-norm of OP*v_j
    double alpha;   // h(j,2) being assembled (CGS coefficient + DGKS corrections)
    double beta;    // h(j,1)
    int dgks;       // 0: none pending, 1: first refinement pending, 2: second
    int zero;       // residual must be zeroed (refinement failed twice)
    int abort;      // 1: rnorm == 0 at the start of step abort_j (host restart);
                    // 2: step abort_j needs its second DGKS refinement (kFinDgks1Lazy)
    int abort_j;
    int nrorth;     // counters accumulated on device, drained by the host
    int nitref;
    int force_dgks2;  // test hook (AHIP_FORCE_DGKS2=1): always take the second refinement
    int fold;       // folded steps: step j's DGKS sweep (coef slot 1) was taken and is
                    // applied by step j+1's passes (kFinPostCgsFold sets it)
    double vscale;  // chained steps: 1/rnorm, applied by the update pass to the raw
                    // column V(:,j) and to A*r (1.0 after a plain kFinCgs)
};

// Finalize phases (which logic the single-block finalize kernel applies).
enum FinPhase : int {
    kFinNorm = 0,     // st.rnorm = sqrt|w'u|                      (getv0, after V*Q)
    kFinCgs = 1,      // coef0 = V'u, st.wnorm, st.alpha, st.beta  (SRC/dsaitr.f:551-594)
    kFinPostCgs = 2,  // st.rnorm, DGKS decision, coef1 = V'r      (SRC/dsaitr.f:634-695)
    kFinDgks1 = 3,    // first refinement check, coef2             (SRC/dsaitr.f:730-771)
    kFinDgks2 = 4,    // second refinement check / give up         (SRC/dsaitr.f:753-781)
    kFinRaw = 5,      // just store the sums (host reads them)
    kFinCoef = 6,     // coef0 = first m-1 sums, state untouched   (getv0 CGS)
    kFinDgks1Lazy = 7,  // kFinDgks1; a needed second refinement parks the cycle
                        // (st.abort = 2 at step j) for the host to finish it
    kFinCgsChained = 8, // step j of a chained (free-running) cycle: the deferred
                        // kFinDgks1Lazy of step j-1 (region 2 sums), then kFinCgs
                        // on the sums of the RAW residual (v_j not yet formed):
                        // coefficients rescaled by 1/rnorm (st.vscale).  abort = 3:
                        // rnorm outside the raw-vector range, redo step j unchained
    kFinCgsFolded = 9,  // step j of a folded cycle: as kFinCgsChained, but region 2 holds
                        // ONE slot (r'r' of step j-1's DGKS-corrected residual, formed by
                        // the fold pass); a needed second refinement parks with
                        // abort = 2 and leaves the coefficients to the host
    kFinPostCgsFold = 10,  // kFinPostCgs + t = T_j s (coef slot 3) and st.fold for the
                           // next step's fold pass
    kFinFoldCoef2 = 11,    // host fallback of a folded park: coef2 = V'r' sums,
                           // h(j,2) += the last one (refine_decision's take path)
};

// Arguments of one single-block finalize (finalize.hpp finalize_block).
struct FinArgs {
    const double* part;
    int nblk, from_sums, m, phase, j, rstart, gate;
    double* sums;
    double* coef;
    int cstride;
    double* rec;
    LzState* st;
    double* hcol;
    int hld;
    const double* part2;
    int m2, rstart_prev;
    int hs;      // the Arnoldi fold's H-staging variant
    int active;  // 0: nothing to run
};

// A finalize deferred into the next SpMV on the owning workspace's stream (one
// at a time: the solver defers only a step's last finalize, which the SpMV
// immediately follows).  Owned by the Workspace of one solve, so solves on
// other workspaces or streams never see it.
struct FinQueue {
    FinArgs a{};
    size_t lds = 0;
    bool set = false;
};

struct Workspace {
    hipStream_t stream = nullptr;
    FinQueue* defq = nullptr;  // the solve's deferred finalize (ws_create allocates it)
    int nblk = 0;        // partial-sum blocks for this n
    int stride = 0;      // >= ncv + 2
    double* part = nullptr;   // 2 regions of nblk * stride (region 2: chained steps)
    double* sums = nullptr;   // 2 * stride (raw sums of the last finalize)
    double* coef = nullptr;   // 4 * stride : CGS, DGKS-1, DGKS-2 coefficient vectors,
                              // t = T_j * DGKS-1 (folded steps)
    double* rec = nullptr;    // 2 * (ncv+1): alpha_j, beta_j per step
    double* q = nullptr;      // ncv * ncv  (V*Q matrix for dsapps / eupd)
    // Arnoldi (dnaitr): column j of H, h(1:j, j) = V_j' w + DGKS corrections,
    // recorded by the finalize kernel; hld = ncv (0 for the Lanczos path).
    double* hcol = nullptr;   // hld * ncv
    int hld = 0;
    // ncv > 64 only: nblk * kBlock * (ncv + 1) doubles of per-thread output
    // columns for the generic (alias-safe) V*Q and gemm kernels
    double* scratch = nullptr;
    // V-load policy of the Gram-Schmidt / V*Q passes (kernels.hip VPol): plain
    // loads when the n x ncv basis fits the Infinity Cache, else non-temporal
    bool v_plain = false;
    LzState* st = nullptr;
    LzState* st_host = nullptr;  // pinned mirror
    double* host_scratch = nullptr;  // pinned, >= 4*stride doubles
    double* host_hcol = nullptr;     // pinned ncv * ncv (ncv <= 64 only): H upload of a folded Arnoldi cycle
    double* host_q = nullptr;        // pinned ncv * ncv (ncv <= 64 only): Q staging of V*Q
};

int choose_nblk(int64_t n);
bool choose_v_plain(int64_t n, int ncv, int elem);
hipError_t ws_create(Workspace& ws, int64_t n, int ncv, hipStream_t s);
void ws_destroy(Workspace& ws);

// The n-length launchers are templates over the storage type R of V, resid and
// workd (double: the d* family; float: the s* family, ICB/arpack.h:10-13).  All
// reductions and the coefficient vectors (part, sums, coef, q) stay double.
//
// v_j = r / rnorm -> V(:,j) (+ optional copies); aborts the cycle if rnorm==0.
template <class R>
void place(const Workspace& ws, int64_t n, const R* r, R* vcol, R* copy1, R* scale_inplace, int j);
// partial sums of [V(:,0:j)' u ; w' u]  (w == u allowed); gate=-1: always,
// else only if st.dgks == gate.
template <class R>
void dots(const Workspace& ws, int64_t n, int j, const R* V, int64_t ld, const R* u, const R* w,
          int gate);
// Extras of a chained (free-running) Lanczos step's update passes
// (kernels.hip k_update_fused): normalise the raw column V(:,j) in place and
// scale w by st.vscale; store rout also to raw1/raw2; write the partials to
// `part` (default ws.part).
template <class R>
struct UpdateChain {
    bool chained = false;
    R* raw1 = nullptr;
    R* raw2 = nullptr;
    double* part = nullptr;
};
// Folded Lanczos step j (free-running, dsaupd): the DGKS sweep of step j-1 is
// applied here instead of in a pass of its own.  The SpMV ran on r (step j-1's
// residual BEFORE its DGKS correction); with s = coef[1] (step j-1's DGKS
// coefficients, applied only if st.fold) and t = T_{j-1} s (coef slot 3):
//   r' = r - V(:,1:j-1) s        (in registers; fold_update stores v_j)
//   w  = A r - V(:,1:j-1) t - s_{j-1} r'   (= A r' by the Lanczos relation
//        A V_{j-1} = V_{j-1} T_{j-1} + r' e', exact up to O(eps*|s|) terms)
// and the partials of [V(:,1:j)' w ; w'w] (region 1, j+1 slots) and r''r'
// (region 2, one slot) for kFinCgsFolded.
template <class R>
void fold_dots(const Workspace& ws, int64_t n, int j, R* V, int64_t ld, const R* r, const R* y);
// The folded step's second pass: r' and w again (bit-identically), v_j =
// r' / rnorm -> V(:,j), r_j = w / rnorm - V(:,1:j) h -> r (in place) and x2
// (nullable), partials of [V(:,1:j)' r_j ; r_j' r_j].
template <class R>
void fold_update(const Workspace& ws, int64_t n, int j, R* V, int64_t ld, const R* y, R* r, R* x2);
// rout = rin - V(:,0:j) * coef[which]; if spec: partials of [V' rout ; rout' rout]
template <class R>
void update(const Workspace& ws, int64_t n, int j, const R* V, int64_t ld, int which, const R* rin,
            R* rout, bool spec, int gate, const UpdateChain<R>& x = UpdateChain<R>{});
// single-block fixed-order finalize of m = j+1 sums and the phase logic
// from_sums: the m sums are already in ws.sums (reduced across ranks).
// m2 > 0 (kFinCgsChained): a second region of m2 partial slots at
// ws.part + nblk * stride (the deferred DGKS sums of step j-1).
// defer: do not launch it -- it waits in ws.defq and the next SpMV handed that
// queue runs it in a workgroup of its own launch (one launch fewer a step); an
// SpMV that cannot carry it, the next finalize, and every stream sync of the
// solve launch it first.
void finalize(const Workspace& ws, int m, FinPhase ph, int j, int rstart, int gate,
              bool from_sums = false, int m2 = 0, int rstart_prev = 0, bool defer = false);
// (false, and the finalize stays deferred, when it needs more than max_lds bytes
// of LDS or the H-column staging and allow_hs is false)
bool take_deferred_finalize(FinQueue* q, FinArgs* a, size_t* lds, size_t max_lds = (size_t)-1,
                            bool allow_hs = true);
// launch q's finalize (if any) on s
void flush_deferred_finalize(FinQueue* q, hipStream_t s);
// resid = 0 if st.zero
template <class R>
void zero_if(const Workspace& ws, int64_t n, R* r);
// V(:,0:kev) = V(:,0:kplusp) * Q(:,0:kev) in place (row-local) and
// r = sigmak*r + betak*Vnew(:,kev); partial r'r for the new rnorm.
template <class R>
void vq_update(const Workspace& ws, int64_t n, R* V, int64_t ld, int kplusp, int kev,
               double sigmak, double betak, R* r);
// Z(:,0:nz) = V(:,0:k) * M(k x nz) (M in ws.q, ld k); Z may alias V.
template <class R>
void vq_gemm(const Workspace& ws, int64_t n, const R* V, int64_t ld, int k, int nz, R* Z,
             int64_t ldz);
// dlarnv / slarnv(idist=2) continuation: x[m] = 2*u(seed*a^(m+1) mod 2^48) - 1;
// offset: global index of x[0] in the stream (row-block sharding).  Returns the
// advanced 48-bit seed (seed*a^n unless slaruv's float redraw rule fired).
// batch: slaruv draws per call (64 for s/dlarnv, 128 for c/zlarnv: 64 complex)
uint64_t larnv_uniform(const Workspace& ws, int64_t n, uint64_t seed48, double* x,
                       int64_t offset = 0, int batch = 64);
uint64_t larnv_uniform(const Workspace& ws, int64_t n, uint64_t seed48, float* x,
                       int64_t offset = 0, int batch = 64);
uint64_t slarnv_host(int64_t n, uint64_t seed48, float* x, int batch = 64);
template <class R>
void copy(hipStream_t s, int64_t n, const R* src, R* dst);
template <class R>
void scal(hipStream_t s, int64_t n, double a, R* x);
template <class R>
void fill(hipStream_t s, int64_t n, double a, R* x);
// y = alpha*y + beta*x
template <class R>
void axpby(hipStream_t s, int64_t n, double alpha, R* y, double beta, const R* x);
// Z(:,l) += x * w[l], l < k (dseupd purification)
template <class R>
void ger_cols(hipStream_t s, int64_t n, int k, const R* x, const double* w, R* Z, int64_t ldz);

// ------------------------------- CSR operator --------------------------------
struct Csr {
    int64_t n = 0, nnz = 0;
    const int64_t* rowptr = nullptr;  // n+1
    const int32_t* col = nullptr;     // nnz
    const double* val = nullptr;      // nnz
    int group = 16;                   // lanes per row for the vector kernel
    // CSR-stream row blocks: block b owns rows [rblk[b], rblk[b+1]) whose
    // nonzeros (<= tile) are streamed by one workgroup
    const int64_t* rblk = nullptr;
    int64_t nrblk = 0;
    int tile = 0;
    int kernel = 0;                   // CsrKernel
    // LDS x-window superblocks (csr_analyse_window)
    const int64_t* w_tiles = nullptr;     // tile row bounds (all superblocks)
    const int64_t* w_sb_tile0 = nullptr;  // first tile of each superblock (+ end)
    const int64_t* w_sb_c0 = nullptr;     // first column of each superblock window
    const int32_t* w_sb_span = nullptr;   // window length
    int64_t w_nsb = 0;
    const uint16_t* w_colw = nullptr;     // col - c0(superblock), 16 bit (owned separately)
    // multi-range windows (csr_analyse_ranges, operators whose rows span several
    // distant column bands, e.g. a 3-D stencil in natural order): per superblock
    // kMaxRanges x ranges staged back to back in LDS -- rng[8 sb + r] = first
    // column of range r, rng[8 sb + 4 + r] = LDS offset << 32 | length (0: unused);
    // w_colw is then the LDS slot.  nullptr: one range [c0, c0 + span).
    const int64_t* w_rng = nullptr;
    // SELL-64 slices inside each window superblock (kCsrSell, csr_build_sell):
    // the superblock's rows sorted by length, 64 per slice (one per lane),
    // entries stored column-step-major so a wave reads 64 consecutive values
    const int64_t* s_sb_slice0 = nullptr;  // first slice of each superblock (+ end)
    const int64_t* s_ptr = nullptr;        // slice start in s_val / s_colw (+ end)
    const int32_t* s_row = nullptr;        // 64 per slice: global row, -1 = padding lane
    const double* s_val = nullptr;
    const uint16_t* s_colw = nullptr;
    int64_t s_nslices = 0, s_padded = 0;
    int s_unroll = 8;                      // column steps per chunk (4, 8 or 16)
    // symmetric storage (kCsrSymSell, csr_build_symsell, spmv_sym.hip): upper
    // triangle only, symmetric superblocks [r0, r1) with x/y windows of span
    // columns, `pre` leading rows combined with the previous superblock's spill
    const int64_t* ss_sb_r0 = nullptr;     // nsb + 1 row bounds
    const int32_t* ss_sb_span = nullptr;
    const int32_t* ss_sb_pre = nullptr;
    const int64_t* ss_sb_off = nullptr;    // nsb + 1 offsets into the combine slots
    const int64_t* ss_slice0 = nullptr;    // first slice of each superblock (+ end)
    const int64_t* ss_ptr = nullptr;       // slice start (+ end)
    const int32_t* ss_row = nullptr;       // 64 per slice, -1 = padding lane
    const double* ss_val = nullptr;
    const uint16_t* ss_colw = nullptr;     // col - r0 (16 bit)
    // balanced walk: superblock b's slices flattened into column steps and cut
    // into one contiguous step range per wave: range (b, q) starts at step
    // ss_wg0[b * 16 + q] (nsb * 16 + 1 entries) inside slice ss_wsl[b * 16 + q]
    const int64_t* ss_wg0 = nullptr;
    const int32_t* ss_wsl = nullptr;
    int* ss_pair = nullptr;  // per-chain pair counters of the fused combine (zero between launches)
    double* ss_lo = nullptr;              // spill partials (written by superblock b-1)
    double* ss_hi = nullptr;               // prefix partials (written by superblock b)
    int64_t ss_nsb = 0, ss_nnz = 0, ss_padded = 0, ss_ncomb = 0;
    int ss_variant = 0;                    // kernel variant (tools/spmv_sym_time.py)
    int ss_chain = 1;                      // consecutive superblocks per workgroup
    int64_t ss_coff = 0;                   // x index of local row 0's diagonal (halo_lo)
    int64_t ss_spill_out = 0;              // rows of the next rank reached by the last window
    int64_t ss_pre0 = 0;                   // head rows of superblock 0 (the incoming spill's)
    int64_t ss_lg_rows = 0;                // 1 + last row with a column in the low halo
    int ss_lg = 0;                         // spill-free distributed form (k_ssell_combine_lg)
    // deterministic mode's form (k_csr_ssell_det): the transposed terms summed
    // as 64-bit fixed point scaled by ss_amax (largest |a_ij| off the diagonal
    // of the upper triangle) times the window's largest |x|, ss_bits bits a
    // term (headroom for the most transposed terms a row receives); usable when
    // every window leaves one LDS word free (ss_det = 1)
    double ss_amax = 0.0;
    int ss_bits = 0;
    int ss_det = 0;
    // ss_det on every rank of a distributed operator (agreed when the storage
    // was chosen; = ss_det on one GPU): deterministic mode switched on AFTER
    // the operator was declared symmetric runs the full-storage (fixed-order)
    // SpMV on every rank when this is 0 (csr_sym_det_fallback)
    int ss_det_all = 0;
    // the transposed terms' accumulator where ss_det_all holds: 0 (default
    // since round 6) the fixed-point form -- y bitwise reproducible; 1 the LDS
    // fp64 atomics (schedule order; arpack_hip_csr_set_sym_accumulator).
    // Deterministic mode always takes the fixed-point form.
    int ss_acc = 0;
    // the fixed-point form as the DEFAULT accumulator also needs the upper
    // off-diagonal magnitudes within 2^20 of each other (ss_fx_ok; on every
    // rank: ss_fx_all) -- a graded operator keeps the fp64 form unless
    // deterministic mode asks for the fixed-point one
    int ss_fx_ok = 0;
    int ss_fx_all = 0;
    int ss_detq = 0;  // most slices one wave walks in a superblock
};
enum CsrKernel : int {
    kCsrVector = 0,
    kCsrStream = 1,
    kCsrStreamNT = 2,
    kCsrWindow = 3,
    kCsrWindowNT = 4,
    kCsrWVec = 5,
    kCsrWVecNT = 6,
    kCsrWVec8 = 7,
    kCsrWVecX = 8,  // wvec with the XCD-contiguous superblock order
    kCsrWVecP3 = 9,  // XCD order, 3 row passes in flight
    kCsrWVecP4 = 10, // XCD order, 4 row passes in flight
    kCsrSell = 11,   // SELL-64 slices (length-sorted rows) over the x windows
    kCsrSymSell = 12,  // symmetric storage: upper-triangle SELL-64, LDS x and y windows
};
// Build the symmetric-storage layout (upper triangle of a square matrix the
// caller declares symmetric); -1 if the matrix does not fit the superblock
// scheme, -2 on allocation failure.  *owned receives the device allocation.
// ncols = coff + n + spill_out: x is [coff | n local | spill_out] (a rank's
// extended x; coff = spill_out = 0 on one GPU); spill_in = leading local rows
// that the previous rank's transposed terms reach (its spill_out).
int csr_build_symsell(Csr& A, int64_t ncols, int64_t coff, int64_t spill_in, int64_t spill_out,
                      void** owned);
void csr_spmv_sym(hipStream_t s, const Csr& A, const double* x, double* y, FinQueue* q = nullptr);
// the same with the in-kernel chain-head combine forced on (where the operator
// allows it, csr_spmv_sym_fusable) or off (test hook, whatever AHIP_SPMV_FUSE says)
void csr_spmv_sym_as(hipStream_t s, const Csr& A, const double* x, double* y, bool fuse,
                     FinQueue* q = nullptr);
bool csr_spmv_sym_fusable(const Csr& A);
// the two halves (the row-distributed SpMV exchanges the spills in between):
// main kernel, then y(prefix rows) = lo + hi.  The outgoing spill is
// ss_lo + ss_ncomb (ss_spill_out doubles); the incoming one lands in ss_lo[0, spill_in).
void csr_spmv_sym_main(hipStream_t s, const Csr& A, const double* x, double* y);
// x_ext (a distributed block's extended x): the spill-free form when A.ss_lg
void csr_spmv_sym_combine(hipStream_t s, const Csr& A, double* y, const double* x_ext = nullptr,
                          FinQueue* q = nullptr);
// Build the SELL-64 layout from a matrix with window tables; *owned receives the
// single device allocation.  0 on success.
int csr_build_sell(Csr& A, void** owned);
// Superblock analysis for the LDS x-window kernel; -1 if some row's column
// span exceeds the window (then the stream kernel is used).  *owned receives
// the single device allocation holding the tables.
int csr_analyse_window(Csr& A, int64_t ncols, void** owned);
// The same tables for rows that span more than one window but whose columns fall
// in at most kMaxRanges bands (w_rng); -1 if the operator does not fit, -2 on a
// HIP error.  Only the SELL kernel (kCsrSell) reads such windows.
constexpr int kMaxRanges = 4;
int csr_analyse_ranges(Csr& A, int64_t ncols, void** owned);
// Build the CSR-stream row blocks (host-side greedy pass over rowptr, once per
// matrix, like a sparse-library "analysis" step).  Returns 0, or -1 if a row
// is longer than the tile (the matrix then keeps the vector kernel).
int csr_analyse(Csr& A, int tile, int64_t** rblk_dev);
void csr_spmv(hipStream_t s, const Csr& A, const double* x, double* y, FinQueue* q = nullptr);
// the first superblock / chain lighter (its workgroup carries the deferred
// finalize); false under AHIP_LIGHT_SB=0
bool light_first_sb();
// AHIP_LIGHT_SB=2: the light superblock 0 shortened by 8% of a chain (A/B)
bool light_sb_chain();
// algorithmic HBM bytes of one SpMV: 12*nnz + 8*(n+1) (int64 rowptr) + 8n (x) + 8n (y)
double csr_bytes(const Csr& A);
// deterministic mode on a symmetric-storage operator whose fixed-point form is
// not available (on some rank): the SpMV runs the full-storage kernel instead
bool csr_sym_det_fallback(const Csr& A);

// ------------------------------------------------------- per-kernel profiler --
// hipEvent pairs around launches (enabled by arpack_hip_profile(1)); gives the
// live average duration and the algorithmic bytes of each kernel class over a
// timed region (bench.py's roofline numbers).
enum ProfClass : int {
    kProfSpmv = 0,
    kProfDots,
    kProfUpdate,    // CGS update + fused DGKS dots, and the first DGKS sweep
    kProfVq,        // dsapps V*Q
    kProfPlace,
    kProfFinalize,
    kProfOther,     // rarely-open gated kernels (2nd refinement, zeroing), copies
    kProfAllreduce, // row-distributed engine: each data-path RCCL allreduce (marker span)
    kProfHalo,      // row-distributed SpMV: each halo / spill / ghost exchange group
    kProfClasses
};
struct ProfStat {
    double ms = 0.0, bytes = 0.0;
    long long count = 0;
};
void prof_enable(bool on);
bool prof_on();
// Marker mode: an event pair recorded on the stream around the span (used
// where the span holds more than kernels, e.g. a row-distributed SpMV's halo
// exchange).
void prof_begin(ProfClass c, hipStream_t s);
void prof_end(ProfClass c, hipStream_t s, double bytes);
// Kernel mode: the span's launches go through AHIP_LAUNCH, which attaches the
// start event to the first kernel's dispatch and the stop event to the last
// one's (hipExtLaunchKernel), so the measured time is the kernels' own
// execution -- what rocprofv3's kernel trace reports -- without marker packets
// between the launches.  Nested spans are counted in the outermost one.
void prof_arm(ProfClass c, hipStream_t s);
void prof_disarm(ProfClass c, double bytes);
bool prof_kernel_events(hipStream_t s, hipEvent_t* start, hipEvent_t* stop);
void prof_collect(ProfStat out[kProfClasses]);  // synchronises, returns and resets

}  // namespace ahip::dev

#include <hip/hip_ext.h>
// hipLaunchKernelGGL, or hipExtLaunchKernelGGL with the profiler's events when
// a kernel-mode span is open (see prof_arm)
#define AHIP_LAUNCH(K, G, B, SH, S, ...)                                                        \
    do {                                                                                       \
        hipEvent_t ahip_ev0_, ahip_ev1_;                                                       \
        if (::ahip::dev::prof_kernel_events((S), &ahip_ev0_, &ahip_ev1_))                      \
            hipExtLaunchKernelGGL(K, G, B, SH, S, ahip_ev0_, ahip_ev1_, 0, __VA_ARGS__);       \
        else                                                                                   \
            hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                   \
    } while (0)
