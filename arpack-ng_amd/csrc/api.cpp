// C-ABI layer: the reference's ICB entry points (ICB/arpack.h), the Fortran
// symbols (dsaupd_ ...), stat_c/debug_c, and the arpack_hip_* extension.
//
// Argument checking, the workl layout and the iparam/info post-processing
// follow SRC/dsaupd.f:473-690 exactly; everything between ido = 0 and ido = 99
// is the Solver coroutine (sym.cpp).
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/arpack_hip.h"
#include "engine.hpp"
#include "zsolve.hpp"

const ahip::dev::Csr* ahip_csr_view(const arpack_hip_csr* A);
const ahip::DistOp* ahip_dist_view(const arpack_hip_dist* D);

namespace ahip {

Stats g_stats;
static hipStream_t g_stream = nullptr;
static std::mutex g_mu;
// live solves keyed by the caller's V (one registry per storage type)
template <class R>
static std::unordered_map<const void*, std::unique_ptr<SolverT<R>>>& registry() {
    static std::unordered_map<const void*, std::unique_ptr<SolverT<R>>> m;
    return m;
}

hipStream_t default_stream() { return g_stream; }

uint64_t seed48_from_iseed(const int is[4]) {
    return ((uint64_t)(is[0] & 4095) << 36) | ((uint64_t)(is[1] & 4095) << 24) |
           ((uint64_t)(is[2] & 4095) << 12) | (uint64_t)(is[3] & 4095);
}
void iseed_from_seed48(uint64_t s, int is[4]) {
    is[0] = (int)((s >> 36) & 4095);
    is[1] = (int)((s >> 24) & 4095);
    is[2] = (int)((s >> 12) & 4095);
    is[3] = (int)(s & 4095);
}
uint64_t lcg_advance(uint64_t seed, uint64_t steps) {
    const uint64_t mask = (1ull << 48) - 1;
    uint64_t base = 33952834046453ull, p = 1;
    while (steps) {
        if (steps & 1) p = (p * base) & mask;
        base = (base * base) & mask;
        steps >>= 1;
    }
    return (seed * p) & mask;
}

uint64_t& getv0_seed(char family) {
    static uint64_t seed[4];
    static bool init[4] = {false, false, false, false};
    const int f = family == 's' ? 1 : family == 'z' ? 2 : family == 'c' ? 3 : 0;
    if (!init[f]) {  // SRC/dgetv0.f:202-208: iseed = (1,3,5,7) once per process
        const int is[4] = {1, 3, 5, 7};
        seed[f] = seed48_from_iseed(is);
        init[f] = true;
    }
    return seed[f];
}

uint64_t& pgetv0_seed(char family, int rank) {
    static uint64_t seed[4];
    static bool init[4] = {false, false, false, false};
    const int f = family == 's' ? 1 : family == 'z' ? 2 : family == 'c' ? 3 : 0;
    if (!init[f]) {  // PARPACK/SRC/MPI/pdgetv0.f:234-245: igen = 1000 + 2 myid + 1
        int igen = 1000 + 2 * rank + 1;
        int is[4];
        is[0] = igen / 1000;
        igen %= 1000;
        is[1] = igen / 100;
        igen %= 100;
        is[2] = igen / 10;
        is[3] = igen % 10;
        seed[f] = seed48_from_iseed(is);
        init[f] = true;
    }
    return seed[f];
}

// dsaupd argument checks (SRC/dsaupd.f:501-543); returns ierr
static int sym_check(char bmat, int n, la::Which which, int nev, int ncv, int lworkl, int mode,
                     int ishift, int mxiter) {
    int ierr = 0;
    if (n <= 0) ierr = -1;
    else if (nev <= 0) ierr = -2;
    else if (ncv <= nev || ncv > n || ncv > dev::kMaxNcv) ierr = -3;
    if (mxiter <= 0) ierr = -4;
    if (which != la::Which::LM && which != la::Which::SM && which != la::Which::LA &&
        which != la::Which::SA && which != la::Which::BE)
        ierr = -5;
    if (bmat != 'I' && bmat != 'G') ierr = -6;
    if (lworkl < ncv * ncv + 8 * ncv) ierr = -7;
    if (mode < 1 || mode > 5) ierr = -10;
    else if (mode == 1 && bmat == 'G') ierr = -11;
    else if (ishift < 0 || ishift > 1) ierr = -12;
    else if (nev == 1 && which == la::Which::BE) ierr = -13;
    return ierr;
}

// dnaupd argument checks (SRC/dnaupd.f:436-466); returns ierr
static int ns_check(char bmat, int n, la::Which which, int nev, int ncv, int lworkl, int mode,
                    int ishift, int mxiter) {
    int ierr = 0;
    if (n <= 0) ierr = -1;
    else if (nev <= 0) ierr = -2;
    else if (ncv <= nev + 1 || ncv > n || ncv > dev::kMaxNcv) ierr = -3;
    else if (mxiter <= 0) ierr = -4;
    else if (which != la::Which::LM && which != la::Which::SM && which != la::Which::LR &&
             which != la::Which::SR && which != la::Which::LI && which != la::Which::SI)
        ierr = -5;
    else if (bmat != 'I' && bmat != 'G') ierr = -6;
    else if (lworkl < 3 * ncv * ncv + 6 * ncv) ierr = -7;
    else if (mode < 1 || mode > 4) ierr = -10;
    else if (mode == 1 && bmat == 'G') ierr = -11;
    else if (ishift < 0 || ishift > 1) ierr = -12;
    return ierr;
}

// The *aupd driver shared by dsaupd (ns = false, SRC/dsaupd.f:408-690) and
// dnaupd (ns = true, SRC/dnaupd.f:400-693): argument checks and workl layout
// at ido = 0, then resume the solve coroutine until it needs the caller.
//
// R = float (ssaupd/snaupd): the n-length data live in fp32; the ncv-sized host
// work runs in double on a shadow of workl that is copied (rounded) into the
// caller's float workl at every return, and the user shifts of ido = 3 are read
// back from it.
template <class R>
static void sym_aupd(int* ido, const char* bmat, int n, const char* which, int nev, double* tol,
                     R* resid, int ncv, R* v, int ldv, int* iparam, int* ipntr, R* workd,
                     R* workl, int lworkl, int* info, const dev::Csr* csr, int max_cycles = -1,
                     const DistOp* dist = nullptr, bool ns = false, dev::DShift* shift = nullptr,
                     dev::DGen* gen = nullptr) {
    constexpr bool kShadow = !std::is_same_v<R, double>;
    if (dist) csr = dist->A;
    if (shift) csr = shift->A;  // mode 3 free run: OP = (A - sigma I)^{-1} on the device
    if (gen) csr = gen->A;      // modes 2-5, bmat = 'G': OP and B on the device
    if (kShadow && csr) {  // the float family: reverse communication (no device-CSR OP)
        *info = -9999;
        *ido = 99;
        return;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    auto& g_sym = registry<R>();
    SolverT<R>* S = nullptr;
    const int wlen = ns ? 3 * ncv * ncv + 6 * ncv : ncv * ncv + 8 * ncv;
    auto wl_out = [&]() {  // shadow -> caller's workl
        if constexpr (kShadow)
            for (int t = 0; t < wlen; ++t) workl[t] = (R)S->wshadow[t];
    };
    if (*ido == 0) {
        g_stats = Stats{};  // dstats (SRC/dstats.f)
        const la::Which w = la::parse_which(which);
        const int ishift = iparam[0], mxiter = iparam[2], mode = iparam[6];
        int ierr = ns ? ns_check(bmat[0], n, w, nev, ncv, lworkl, mode, ishift, mxiter)
                      : sym_check(bmat[0], n, w, nev, ncv, lworkl, mode, ishift, mxiter);
        // a device OP serves mode 1 (OP = A), or mode 3 through the device solve
        // (symmetric only: CG); bmat = 'I'
        // (dnaupd: a nonsymmetric A needs the general solve, BiCGStab)
        if (gen) {  // the operator pair fixes the mode (bmat = 'G'); dnaupd: modes 2, 3
            // (a complex-shift pair: dnaupd's modes 3 / 4 only)
            if (dist || bmat[0] != 'G' || mode != gen->mode || gen->n != n ||
                (ns && mode != 2 && mode != 3 && !(gen->cshift && mode == 4)) ||
                (!ns && gen->cshift))
                ierr = (ierr ? ierr : -11);
        } else if (csr && ((shift ? mode != 3 || dist ||
                                        (ns && shift->method != dev::kDShiftBicgstab &&
                                         shift->method != dev::kDShiftTridiag)
                                  : mode != 1) ||
                           bmat[0] != 'I' || csr->n != n)) {
            ierr = (ierr ? ierr : -11);
        }
        if (dist && dist->nloc != n) ierr = (ierr ? ierr : -1);
        if (ierr != 0) {
            *info = ierr;
            *ido = 99;
            return;
        }
        if (*tol <= 0.0) *tol = Prec<R>::eps;
        g_sym.erase(v);  // a previous solve on the same V is abandoned: finish it first
        auto up = std::make_unique<SolverT<R>>();
        S = up.get();
        S->bmat = bmat[0];
        S->which = w;
        S->n = n;
        S->ncv = ncv;
        S->mode = mode;
        S->ishift = ishift;
        S->mxiter = mxiter;
        S->nev0 = nev;
        S->np = ncv - nev;
        S->lworkl = lworkl;
        S->info = *info;
        double* wl = reinterpret_cast<double*>(workl);
        if constexpr (kShadow) {
            S->wshadow.assign((size_t)wlen, 0.0);
            wl = S->wshadow.data();
        }
        std::memset(workl, 0, sizeof(R) * (size_t)wlen);
        if (!ns) {  // workl layout (SRC/dsaupd.f:566-595)
            S->ih = 0;
            S->iritz = S->ih + 2 * ncv;
            S->ibounds = S->iritz + ncv;
            S->iq = S->ibounds + ncv;
            S->iw = S->iq + ncv * ncv;
            const int next = S->iw + 3 * ncv;
            ipntr[3] = next + 1;
            ipntr[4] = S->ih + 1;
            ipntr[5] = S->iritz + 1;
            ipntr[6] = S->ibounds + 1;
            ipntr[10] = S->iw + 1;
        } else {  // workl layout (SRC/dnaupd.f:494-520)
            S->arnoldi = true;
            S->ih = 0;
            S->iritz = S->ih + ncv * ncv;
            S->iritzi = S->iritz + ncv;
            S->ibounds = S->iritzi + ncv;
            S->iq = S->ibounds + ncv;
            S->iw = S->iq + ncv * ncv;
            const int next = S->iw + ncv * ncv + 3 * ncv;
            ipntr[3] = next + 1;
            ipntr[4] = S->ih + 1;
            ipntr[5] = S->iritz + 1;
            ipntr[6] = S->iritzi + 1;
            ipntr[7] = S->ibounds + 1;
            ipntr[13] = S->iw + 1;
        }
        S->n_global = dist ? dist->n_global : n;
        if (S->a.attach(n, ncv, resid, v, ldv, workd) != 0 ||
            dev::ws_create(S->ws, n, ncv, S->a.stream) != hipSuccess) {
            *info = -9999;
            *ido = 99;
            return;
        }
        S->a.defq = S->ws.defq;  // (a.sync() launches what is still deferred)
        if (csr) {
            S->free_run = true;
            S->csr = csr;
            S->shift = shift;
            S->gen = gen;
        }
        if (dist) {
            S->dist = dist;
            S->dist_gen = dist->comm_gen;
            S->row0 = dist->row0;
        }
        S->tol = *tol;
        S->iparam = iparam;
        S->ipntr = ipntr;
        S->workl = wl;
        if (ns) S->ws.hld = ncv;
        S->root.emplace(ns ? S->run_ns() : S->run());
        start_root(*S->root, S->ctx);
        g_sym[v] = std::move(up);
    } else {
        auto it = g_sym.find(v);
        if (it == g_sym.end()) {
            *info = -9999;
            *ido = 99;
            return;
        }
        S = it->second.get();
        // the decomposition this solve started on must still be the caller's:
        // a distribution that was freed and rebuilt (PARPACK rebinding to
        // another communicator) may even reuse the address, so the generation
        // of its communicator is checked too
        if (S->dist != dist || (dist && dist->comm && !comm_alive(dist->comm, S->dist_gen))) {
            g_sym.erase(it);
            *info = -9999;
            *ido = 99;
            return;
        }
        S->tol = *tol;  // the ICB passes tol by value on every call (SRC/icbads.F90:14)
        S->iparam = iparam;
        S->ipntr = ipntr;
        const RciReq& r = S->ctx.req;
        if constexpr (kShadow) {
            if (r.ido == 3) {  // the caller's shifts (real parts, then imaginary for dnaupd)
                const int cnt = (ns ? 2 : 1) * iparam[7];
                for (int t = 0; t < cnt; ++t) S->wshadow[S->iw + t] = (double)workl[S->iw + t];
            }
        } else {
            S->workl = workl;
        }
        // bring the caller's results of the previous request into HBM
        if (r.ido == -1 || r.ido == 1 || r.ido == 2) {
            S->a.h2d_workd(r.y, n);
            if (r.ido == 1 && S->mode == 2 && !S->arnoldi) S->a.h2d_workd(r.x, n);
        }
    }
    if (csr) S->pause_budget = max_cycles;
    // a failed collective (RCCL / transport error) ends the solve with
    // info = -9999 at the next return to the caller: the ranks' sums no longer
    // agree.  So does a failed HIP call of this solve (the sticky S->a.err: a
    // copy, an enqueue, or a kernel fault surfacing at a sync).  Both are
    // local observations -- a rank keeps joining the collectives after its own
    // failure, so the ranks stay in step -- and on a multi-rank solve the ranks
    // agree (one flag allreduce) before any of them leaves, so every rank ends
    // at the same return.
    auto broken = [&]() {
        bool bad = S->a.err.bad() || (S->dist && comm_failed(S->dist->comm));
        if (S->dist && comm_size(S->dist->comm) > 1) bad = !dist_all_ok(S->dist->comm, !bad);
        if (!bad) return false;
        (void)hipStreamSynchronize(S->a.stream);
        *info = -9999;
        *ido = 99;
        g_sym.erase(v);
        return true;
    };
    for (;;) {
        S->ctx.leaf.resume();
        if (S->ctx.done) break;
        const RciReq r = S->ctx.req;
        // (the park below drains the stream first, then checks)
        if (r.ido != -1 && r.ido != 1 && r.ido != SolverT<R>::kPauseIdo && broken()) return;
        if (S->gen && (r.ido == -1 || r.ido == 1 || r.ido == 2)) {
            // generalized modes: OP*x (mode 2 also writes A x back over x) and
            // B*x on the device; x, y are the request's device pointers, or its
            // workd slices
            if constexpr (!kShadow) {
                double* W = S->a.d_workd;
                const double* xp = S->op_x ? S->op_x : W + r.x;
                double* yp = S->op_y ? S->op_y : W + r.y;
                const double* bxp = (r.ido == 1 && r.bx >= 0) ? W + r.bx : nullptr;
                dev::flush_deferred_finalize(S->ws.defq, S->a.stream);
                // (dnaupd's mode 2 has no x <- A x write-back: dndrv3.f:215-240)
                const int rc = dev::dgen_apply(*S->gen, S->a.stream, r.ido, xp, yp, bxp,
                                               S->arnoldi ? nullptr : W + r.x);
                if (rc < 0) {  // a solve missed its tolerance: OP is not what was asked
                    S->a.sync();
                    *info = -9999;
                    *ido = 99;
                    g_sym.erase(v);
                    return;
                }
            }
            continue;
        }
        if (S->free_run && (r.ido == -1 || r.ido == 1)) {
            // kernel-mode timing (the SpMV kernels' own execution, as rocprofv3 reports
            // it); a row-distributed SpMV also holds its halo exchange: marker mode
            const double by = dev::csr_bytes(*S->csr);
            if (S->dist && S->x_ready) {
                // overlapped: halo + SpMV on op_stream once the update pass has
                // written x, concurrent with that pass's allreduce + finalize on
                // a.stream (p2p communicator); a.stream waits for y
                S->x_ready = false;
                hipStream_t so = S->op_stream;
                bool ok = hipStreamWaitEvent(so, S->x_ev, 0) == hipSuccess;
                dev::prof_begin(dev::kProfSpmv, so);
                if constexpr (!kShadow) dist_spmv(*S->dist, so, S->op_x, S->op_y, true);
                dev::prof_end(dev::kProfSpmv, so, by);
                ok = ok && hipEventRecord(S->y_ev, so) == hipSuccess &&
                     hipStreamWaitEvent(S->a.stream, S->y_ev, 0) == hipSuccess;
                if (!ok) {  // cannot order the streams: finish here, serialised
                    (void)hipStreamSynchronize(so);
                }
                continue;
            }
            if constexpr (!kShadow) {
                if (S->shift) {  // mode 3 (bmat = 'I': B x = x for ido = 1 too)
                    // the solve's deferred finalize does not ride in the solver's
                    // products: launch it here, ahead of them in stream order
                    dev::flush_deferred_finalize(S->ws.defq, S->a.stream);
                    if (dev::dshift_apply(*S->shift, S->a.stream, S->op_x, S->op_y, nullptr) < 0) {
                        // the solve broke down or missed its tolerance: OP is not
                        // what the caller asked for, so the Lanczos run stops
                        S->a.sync();
                        *info = -9999;
                        *ido = 99;
                        g_sym.erase(v);
                        return;
                    }
                    continue;
                }
            }
            if (S->dist) dev::prof_begin(dev::kProfSpmv, S->a.stream);
            else dev::prof_arm(dev::kProfSpmv, S->a.stream);
            if constexpr (!kShadow) {
                if (S->dist) dist_spmv(*S->dist, S->a.stream, S->op_x, S->op_y, false, S->ws.defq);
                else dev::csr_spmv(S->a.stream, *S->csr, S->op_x, S->op_y, S->ws.defq);
            }
            if (S->dist) dev::prof_end(dev::kProfSpmv, S->a.stream, by);
            else dev::prof_disarm(dev::kProfSpmv, by);
            // (an SpMV form that cannot carry it has launched it; nothing may
            // leave this request with a finalize still pending)
            dev::flush_deferred_finalize(S->ws.defq, S->a.stream);
            continue;
        }
        if (r.ido == SolverT<R>::kPauseIdo) {  // cycle budget spent: park
            // the caller may free or reuse its arrays before resuming: drain
            S->a.sync();
            if (broken()) return;
            *ido = r.ido;
            return;
        }
        // hand the request to the caller
        if ((r.ido == -1 || r.ido == 1) && broken()) return;
        if (r.ido == -1 || r.ido == 1 || r.ido == 2) {
            S->a.d2h_workd(r.x, n);
            if (r.ido == 1 && r.bx >= 0 && S->mode >= 3) S->a.d2h_workd(r.bx, n);
            ipntr[0] = (int)(r.x + 1);
            ipntr[1] = (int)(r.y + 1);
            if (r.bx >= 0) ipntr[2] = (int)(r.bx + 1);
        }
        S->a.sync();
        wl_out();
        *ido = r.ido;
        return;
    }
    // ido = 99: dsaupd post-processing (SRC/dsaupd.f:613-627)
    if (broken()) return;
    *ido = 99;
    iparam[2] = S->mxiter;
    iparam[4] = S->np;
    iparam[8] = g_stats.nopx;
    iparam[9] = g_stats.nbx;
    iparam[10] = g_stats.nrorth;
    int inf = S->info;
    if (inf >= 0 && inf == 2) inf = 3;
    *info = inf;
    S->a.download_all();
    S->a.sync();
    if (S->a.err.bad()) *info = -9999;
    wl_out();
    g_sym.erase(v);
}

}  // namespace ahip

using namespace ahip;

extern "C" {

void dsaupd_c(int* ido, char const* bmat, int n, char const* which, int nev, double tol,
              double* resid, int ncv, double* v, int ldv, int* iparam, int* ipntr, double* workd,
              double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, &tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, nullptr);
}

void dnaupd_c(int* ido, char const* bmat, int n, char const* which, int nev, double tol,
              double* resid, int ncv, double* v, int ldv, int* iparam, int* ipntr, double* workd,
              double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, &tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, nullptr, -1, nullptr, true);
}

void dnaupd_(int* ido, char const* bmat, int* n, char const* which, int* nev, double* tol,
             double* resid, int* ncv, double* v, int* ldv, int* iparam, int* ipntr, double* workd,
             double* workl, int* lworkl, int* info, size_t, size_t) {
    sym_aupd(ido, bmat, *n, which, *nev, tol, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl,
             *lworkl, info, nullptr, -1, nullptr, true);
}

// single-precision family (ICB/arpack.h:16,18; SRC/ssaupd.f, SRC/snaupd.f): fp32
// n-length data and kernels, tol <= 0 -> slamch('EpsMach')
void ssaupd_c(int* ido, char const* bmat, int n, char const* which, int nev, float tol,
              float* resid, int ncv, float* v, int ldv, int* iparam, int* ipntr, float* workd,
              float* workl, int lworkl, int* info) {
    double t = tol;
    sym_aupd(ido, bmat, n, which, nev, &t, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, nullptr);
}

void snaupd_c(int* ido, char const* bmat, int n, char const* which, int nev, float tol,
              float* resid, int ncv, float* v, int ldv, int* iparam, int* ipntr, float* workd,
              float* workl, int lworkl, int* info) {
    double t = tol;
    sym_aupd(ido, bmat, n, which, nev, &t, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, nullptr, -1, nullptr, true);
}

void ssaupd_(int* ido, char const* bmat, int* n, char const* which, int* nev, float* tol,
             float* resid, int* ncv, float* v, int* ldv, int* iparam, int* ipntr, float* workd,
             float* workl, int* lworkl, int* info, size_t, size_t) {
    double t = *tol;
    sym_aupd(ido, bmat, *n, which, *nev, &t, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl,
             *lworkl, info, nullptr);
    *tol = (float)t;
}

void snaupd_(int* ido, char const* bmat, int* n, char const* which, int* nev, float* tol,
             float* resid, int* ncv, float* v, int* ldv, int* iparam, int* ipntr, float* workd,
             float* workl, int* lworkl, int* info, size_t, size_t) {
    double t = *tol;
    sym_aupd(ido, bmat, *n, which, *nev, &t, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl,
             *lworkl, info, nullptr, -1, nullptr, true);
    *tol = (float)t;
}

void arpack_hip_dnaupd_csr_cycles(const arpack_hip_csr* A, int max_cycles, int* ido,
                                  char const* bmat, int n, char const* which, int nev, double* tol,
                                  double* resid, int ncv, double* v, int ldv, int* iparam,
                                  int* ipntr, double* workd, double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, ahip_csr_view(A), max_cycles, nullptr, true);
}

void dsaupd_(int* ido, char const* bmat, int* n, char const* which, int* nev, double* tol,
             double* resid, int* ncv, double* v, int* ldv, int* iparam, int* ipntr, double* workd,
             double* workl, int* lworkl, int* info, size_t, size_t) {
    sym_aupd(ido, bmat, *n, which, *nev, tol, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl,
             *lworkl, info, nullptr);
}

void arpack_hip_dsaupd_csr(const arpack_hip_csr* A, int* ido, char const* bmat, int n,
                           char const* which, int nev, double tol, double* resid, int ncv,
                           double* v, int ldv, int* iparam, int* ipntr, double* workd,
                           double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, &tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, ahip_csr_view(A));
}

void arpack_hip_dsaupd_csr_cycles(const arpack_hip_csr* A, int max_cycles, int* ido,
                                  char const* bmat, int n, char const* which, int nev, double* tol,
                                  double* resid, int ncv, double* v, int ldv, int* iparam,
                                  int* ipntr, double* workd, double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, ahip_csr_view(A), max_cycles);
}

// ---- shift-invert on the device (dsaupd mode 3, dshift.hip) ----------------
struct arpack_hip_dshift {
    ahip::dev::DShift S;
};

struct arpack_hip_dgen {
    ahip::dev::DGen G;
};

int arpack_hip_dgen_create(arpack_hip_dgen** out, const arpack_hip_csr* A, const arpack_hip_csr* B,
                           int mode, double sigma, double rtol, int maxit, int method) {
    if (!out || !(rtol > 0.0) || maxit < 1 || method < ahip::dev::kDShiftCg ||
        method > ahip::dev::kDShiftTridiag)
        return -1;
    auto* D = new arpack_hip_dgen;
    const int rc = ahip::dev::dgen_create(D->G, A, B, mode, sigma, rtol, maxit, method);
    if (rc != 0) {
        delete D;
        return rc;
    }
    *out = D;
    return 0;
}

// dnaupd's complex shifts (modes 3 / 4 with sigmai != 0): OP = Re / Im of
// inv[A - sigma M] M, the complex solve by BiCGStab (method 0) or the direct
// tridiagonal solve (method 1)
int arpack_hip_dgen_create_cshift(arpack_hip_dgen** out, const arpack_hip_csr* A,
                                  const arpack_hip_csr* B, int mode, double sigmar, double sigmai,
                                  double rtol, int maxit, int method) {
    if (!out || !(rtol > 0.0) || maxit < 1) return -1;
    auto* D = new arpack_hip_dgen;
    const int rc = ahip::dev::dgen_create_cshift(D->G, A, B, mode, sigmar, sigmai, rtol, maxit, method);
    if (rc != 0) {
        delete D;
        return rc;
    }
    *out = D;
    return 0;
}

void arpack_hip_dgen_destroy(arpack_hip_dgen* D) {
    if (!D) return;
    ahip::dev::dgen_destroy(D->G);
    delete D;
}

int arpack_hip_dgen_stats(const arpack_hip_dgen* D, long long* solves, long long* iters,
                          long long* fails, double* max_relres) {
    if (!D) return -1;
    if (D->G.cshift) {
        const auto& Z = *D->G.ZS;
        *solves = Z.n_solves;
        *iters = Z.n_iters;
        *fails = Z.n_fail;
        *max_relres = Z.max_relres;
        return 0;
    }
    const ahip::dev::DShift& S = D->G.S;
    *solves = S.n_solves;
    *iters = S.n_iters;
    *fails = S.n_fail;
    *max_relres = S.max_relres;
    return 0;
}

void arpack_hip_dsaupd_gen(arpack_hip_dgen* D, int* ido, char const* bmat, int n, char const* which,
                           int nev, double* tol, double* resid, int ncv, double* v, int ldv,
                           int* iparam, int* ipntr, double* workd, double* workl, int lworkl,
                           int* info) {
    if (!D) {
        *info = -9999;
        *ido = 99;
        return;
    }
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, nullptr, -1, nullptr, false, nullptr, &D->G);
}

// dnaupd's generalized modes on the device (bmat = 'G'; mode 2, or mode 3 with
// the real shift the operator pair was made with; dneupd_c then takes
// sigmar = sigma, sigmai = 0)
void arpack_hip_dnaupd_gen(arpack_hip_dgen* D, int* ido, char const* bmat, int n, char const* which,
                           int nev, double* tol, double* resid, int ncv, double* v, int ldv,
                           int* iparam, int* ipntr, double* workd, double* workl, int lworkl,
                           int* info) {
    if (!D) {
        *info = -9999;
        *ido = 99;
        return;
    }
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, nullptr, -1, nullptr, true, nullptr, &D->G);
}

int arpack_hip_dshift_create(arpack_hip_dshift** out, const arpack_hip_csr* A, double sigma,
                             double rtol, int maxit) {
    if (!out || !A || !(rtol > 0.0) || maxit < 1) return -1;
    auto* D = new arpack_hip_dshift;
    if (ahip::dev::dshift_create(D->S, ahip_csr_view(A), sigma, rtol, maxit) != 0) {
        delete D;
        return -2;
    }
    *out = D;
    return 0;
}

int arpack_hip_dshift_set_method(arpack_hip_dshift* D, int method) {
    if (!D || method < ahip::dev::kDShiftCg || method > ahip::dev::kDShiftTridiag) return -1;
    ahip::dev::dshift_tridiag_free(D->S);
    if (method == ahip::dev::kDShiftTridiag && ahip::dev::dshift_tridiag_factor(D->S) != 0) return -1;
    D->S.method = method;
    D->S.chunk = 8;  // the previous method's iteration count says nothing here
    return 0;
}

void arpack_hip_dshift_destroy(arpack_hip_dshift* D) {
    if (!D) return;
    ahip::dev::dshift_destroy(D->S);
    delete D;
}

int arpack_hip_dshift_solve(arpack_hip_dshift* D, const double* x, double* y, double* relres) {
    if (!D || !x || !y || x == y) return -2;
    return ahip::dev::dshift_apply(D->S, nullptr, x, y, relres);
}

int arpack_hip_dshift_stats(const arpack_hip_dshift* D, long long* solves, long long* iters,
                            long long* failures, double* max_relres, double* ms,
                            double* bytes_per_iter) {
    if (!D) return -1;
    const auto& S = D->S;
    if (solves) *solves = S.n_solves;
    if (iters) *iters = S.n_iters;
    if (failures) *failures = S.n_fail;
    if (max_relres) *max_relres = S.max_relres;
    if (ms) *ms = S.ms_total;
    if (bytes_per_iter) *bytes_per_iter = ahip::dev::dshift_iter_bytes(S);
    return 0;
}

void arpack_hip_dsaupd_shift(arpack_hip_dshift* D, int* ido, char const* bmat, int n,
                             char const* which, int nev, double* tol, double* resid, int ncv,
                             double* v, int ldv, int* iparam, int* ipntr, double* workd,
                             double* workl, int lworkl, int* info) {
    if (!D) {
        *info = -9999;
        *ido = 99;
        return;
    }
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, nullptr, -1, nullptr, false, &D->S);
}

// dnaupd in mode 3 with a real shift, OP = (A - sigma I)^{-1} by the device
// BiCGStab (arpack_hip_dshift_set_method(S, 2)); dneupd_c with sigmar = sigma,
// sigmai = 0 then gives the eigenvalues of A
void arpack_hip_dnaupd_shift(arpack_hip_dshift* D, int* ido, char const* bmat, int n,
                             char const* which, int nev, double* tol, double* resid, int ncv,
                             double* v, int ldv, int* iparam, int* ipntr, double* workd,
                             double* workl, int lworkl, int* info) {
    if (!D) {
        *info = -9999;
        *ido = 99;
        return;
    }
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, nullptr, -1, nullptr, true, &D->S);
}

// Row-block distributed solve (PARPACK's pdsaupd decomposition, n = LOCAL rows):
// each rank calls this with its slice of resid/V/workd; see dist.hpp.
void arpack_hip_pdsaupd_csr_cycles(const arpack_hip_dist* D, int max_cycles, int* ido,
                                   char const* bmat, int n, char const* which, int nev,
                                   double* tol, double* resid, int ncv, double* v, int ldv,
                                   int* iparam, int* ipntr, double* workd, double* workl,
                                   int lworkl, int* info) {
    const DistOp* d = ahip_dist_view(D);
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, d->A, max_cycles, d);
}

// Nonsymmetric twin (PARPACK/SRC/MPI/pdnaupd.f decomposition).
void arpack_hip_pdnaupd_csr_cycles(const arpack_hip_dist* D, int max_cycles, int* ido,
                                   char const* bmat, int n, char const* which, int nev,
                                   double* tol, double* resid, int ncv, double* v, int ldv,
                                   int* iparam, int* ipntr, double* workd, double* workl,
                                   int lworkl, int* info) {
    const DistOp* d = ahip_dist_view(D);
    sym_aupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             info, d->A, max_cycles, d, true);
}

// PARPACK-style RCI (ICB/parpack.h:20 pdsaupd_c, :26 pdnaupd_c): n = LOCAL rows,
// the communicator is the engine's RCCL one (the decomposition handle from
// arpack_hip_dist_rows); the caller's OP acts on its rows.  tol by value.
void arpack_hip_pdsaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, double tol, double* resid, int ncv,
                          double* v, int ldv, int* iparam, int* ipntr, double* workd,
                          double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, &tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, nullptr, -1, ahip_dist_view(D), false);
}

void arpack_hip_pdnaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, double tol, double* resid, int ncv,
                          double* v, int ldv, int* iparam, int* ipntr, double* workd,
                          double* workl, int lworkl, int* info) {
    sym_aupd(ido, bmat, n, which, nev, &tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, nullptr, -1, ahip_dist_view(D), true);
}

// fp32 PARPACK-style RCI (ICB/parpack.h:17 pssaupd_c, :23 psnaupd_c): the float
// engine on a row decomposition; reductions in fp64 and allreduced as for pd*.
void arpack_hip_pssaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, float tol, float* resid, int ncv, float* v,
                          int ldv, int* iparam, int* ipntr, float* workd, float* workl,
                          int lworkl, int* info) {
    double t = tol;
    sym_aupd(ido, bmat, n, which, nev, &t, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, nullptr, -1, ahip_dist_view(D), false);
}
void arpack_hip_psnaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, float tol, float* resid, int ncv, float* v,
                          int ldv, int* iparam, int* ipntr, float* workd, float* workl,
                          int lworkl, int* info) {
    double t = tol;
    sym_aupd(ido, bmat, n, which, nev, &t, resid, ncv, v, ldv, iparam, ipntr, workd, workl,
             lworkl, info, nullptr, -1, ahip_dist_view(D), true);
}

// PARPACK's start vector for info = 0 (PARPACK/SRC/MPI/pdgetv0.f:234-245)
int arpack_hip_dist_set_seed_mode(arpack_hip_dist* D, int mode) {
    if (!D || (mode != 0 && mode != 1)) return -1;
    const_cast<DistOp*>(ahip_dist_view(D))->seed_mode = mode;
    return 0;
}

void arpack_hip_fault_inject(long k) { fault_inject(k); }
void arpack_hip_set_deterministic(int on) { set_deterministic(on != 0); }
int arpack_hip_deterministic(void) { return deterministic() ? 1 : 0; }

void arpack_hip_profile(int enable) { dev::prof_enable(enable != 0); }

int arpack_hip_profile_read(double* ms, double* bytes, long long* count, int nclass) {
    dev::ProfStat st[dev::kProfClasses];
    dev::prof_collect(st);
    const int k = nclass < dev::kProfClasses ? nclass : dev::kProfClasses;
    for (int c = 0; c < k; ++c) {
        ms[c] = st[c].ms;
        bytes[c] = st[c].bytes;
        count[c] = st[c].count;
    }
    return dev::kProfClasses;
}

void sstats_c(void) { g_stats = Stats{}; }
// dstatn / cstatn (SRC/dstatn.f, SRC/cstatn.f): the same counters; the family
// timers they also clear read 0 in this build (see stat_c)
void sstatn_c(void) { g_stats = Stats{}; }
void cstatn_c(void) { g_stats = Stats{}; }

void stat_c(int* nopx, int* nbx, int* nrorth, int* nitref, int* nrstrt, float* tsaupd,
            float* tsaup2, float* tsaitr, float* tseigt, float* tsgets, float* tsapps,
            float* tsconv, float* tnaupd, float* tnaup2, float* tnaitr, float* tneigh,
            float* tngets, float* tnapps, float* tnconv, float* tcaupd, float* tcaup2,
            float* tcaitr, float* tceigh, float* tcgets, float* tcapps, float* tcconv,
            float* tmvopx, float* tmvbx, float* tgetv0, float* titref, float* trvec) {
    *nopx = g_stats.nopx;
    *nbx = g_stats.nbx;
    *nrorth = g_stats.nrorth;
    *nitref = g_stats.nitref;
    *nrstrt = g_stats.nrstrt;
    // the reference's default build links second_NONE.f: every timer reads 0
    for (float* t : {tsaupd, tsaup2, tsaitr, tseigt, tsgets, tsapps, tsconv, tnaupd, tnaup2, tnaitr,
                     tneigh, tngets, tnapps, tnconv, tcaupd, tcaup2, tcaitr, tceigh, tcgets, tcapps,
                     tcconv, tmvopx, tmvbx, tgetv0, titref, trvec})
        if (t) *t = 0.0f;
}

void debug_c(int, int, int, int, int, int, int, int, int, int, int, int, int, int, int, int, int,
             int, int, int, int, int, int, int) {
    // message levels only affect printing (debug.h); printing is out of scope
}

const char* arpack_hip_version(void) { return "arpack-hip 0.1 (gfx950, arpack-ng 3.9.1 ICB)"; }

int arpack_hip_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return c;
}

// PCI bus id ("dddd:bb:dd.f") of a device: bench.py reports which GPU every rank
// of a multi-GPU run drove
int arpack_hip_device_pci_bus_id(int device, char* buf, int len) {
    if (!buf || len < 13) return -1;
    if (hipDeviceGetPCIBusId(buf, len, device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return 0;
}

void arpack_hip_set_stream(void* stream) { g_stream = (hipStream_t)stream; }

void* arpack_hip_malloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
    return p;
}
void arpack_hip_free(void* p) {
    if (p) (void)hipFree(p);
}
// Both complete before they return: hipMemset and a device-to-device
// hipMemcpy may still be in flight on the null stream when they return, and the
// engine's non-blocking stream does not order against it (a memset of a fresh
// Z landed after dseupd had written it: zero rows on one rank of an 8-process
// rehearsal).
int arpack_hip_memcpy(void* dst, const void* src, size_t bytes) {
    return hipMemcpy(dst, src, bytes, hipMemcpyDefault) == hipSuccess &&
                   hipStreamSynchronize(nullptr) == hipSuccess
               ? 0
               : -1;
}
int arpack_hip_memset(void* dst, int value, size_t bytes) {
    return hipMemset(dst, value, bytes) == hipSuccess && hipStreamSynchronize(nullptr) == hipSuccess
               ? 0
               : -1;
}
int arpack_hip_synchronize(void) { return hipDeviceSynchronize() == hipSuccess ? 0 : -1; }

// ---- host kit exports (CPU-testable) ----
int arpack_hip_kit_dstqrb(int n, double* d, double* e, double* z, double* work) {
    return la::stqrb(n, d, e, z, work);
}
int arpack_hip_kit_dsteqr(int n, double* d, double* e, double* z, int ldz, double* work) {
    return la::steqr(n, d, e, z, n, ldz, work, false);
}
void arpack_hip_kit_dlartg(double f, double g, double* c, double* s, double* r) {
    la::lartg(f, g, *c, *s, *r);
}
void arpack_hip_kit_dsortr(char const* which, int apply, int n, double* x1, double* x2) {
    la::dsortr(la::parse_which(which), apply != 0, n, x1, x2);
}
void arpack_hip_kit_dsapps_host(int kev, int np, const double* shift, double* h, int ldh, double* q,
                                int ldq) {
    la::dsapps_host(kev, np, shift, h, ldh, q, ldq);
}
// The device start-vector generators (dgetv0/sgetv0's dlarnv/slarnv) on a
// caller device buffer: prec 'd' (double*) or 's' (float*); iseed updated.
int arpack_hip_larnv_device(char prec, int* iseed, int64_t n, void* x) {
    dev::Workspace ws;
    hipStream_t st = nullptr;
    if (hipStreamCreate(&st) != hipSuccess) return -1;
    if (dev::ws_create(ws, n, 2, st) != hipSuccess) {
        (void)hipStreamDestroy(st);
        return -1;
    }
    const uint64_t s0 = seed48_from_iseed(iseed);
    const uint64_t s1 = prec == 's' ? dev::larnv_uniform(ws, n, s0, (float*)x)
                                    : dev::larnv_uniform(ws, n, s0, (double*)x);
    const int rc = hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
    iseed_from_seed48(s1, iseed);
    dev::ws_destroy(ws);
    (void)hipStreamDestroy(st);
    return rc;
}

void arpack_hip_kit_dlarnv(int* iseed, int n, double* x) {
    // host reference of the device generator (same arithmetic)
    uint64_t s = seed48_from_iseed(iseed);
    const uint64_t mask = (1ull << 48) - 1, a = 33952834046453ull;
    for (int i = 0; i < n; ++i) {
        s = (s * a) & mask;
        x[i] = 2.0 * ((double)s * 0x1p-48) - 1.0;
    }
    iseed_from_seed48(s, iseed);
}

// host slarnv(idist=2) with slaruv's redraw rule (the device generator's fallback)
void arpack_hip_kit_slarnv(int* iseed, int n, float* x) {
    const uint64_t s = dev::slarnv_host(n, seed48_from_iseed(iseed), x);
    iseed_from_seed48(s, iseed);
}

double arpack_hip_kit_dnrm2(int n, const double* x) { return la::nrm2(n, x, 1); }
void arpack_hip_kit_dlanv2(double* a, double* b, double* c, double* d, double* rt1r, double* rt1i,
                           double* rt2r, double* rt2i, double* cs, double* sn) {
    la::lanv2(*a, *b, *c, *d, *rt1r, *rt1i, *rt2r, *rt2i, *cs, *sn);
}
int arpack_hip_kit_dlahqr(int wantt, int wantz, int n, int ilo, int ihi, double* h, int ldh,
                          double* wr, double* wi, int iloz, int ihiz, double* z, int ldz) {
    return la::lahqr(wantt != 0, wantz != 0, n, ilo, ihi, h, ldh, wr, wi, iloz, ihiz, z, ldz);
}
int arpack_hip_kit_dtrevc(char howmny, int* select, int n, const double* t, int ldt, double* vr,
                          int ldvr, double* work) {
    return la::trevc_right(howmny, select, n, t, ldt, vr, ldvr, work);
}
void arpack_hip_kit_dsortc(char const* which, int apply, int n, double* xr, double* xi, double* y) {
    la::dsortc(la::parse_which(which), apply != 0, n, xr, xi, y);
}
void arpack_hip_kit_dngets(int ishift, char const* which, int* kev, int* np, double* ritzr,
                           double* ritzi, double* bounds) {
    la::dngets(ishift, la::parse_which(which), *kev, *np, ritzr, ritzi, bounds);
}
int arpack_hip_kit_dneigh(double rnorm, int n, const double* h, int ldh, double* ritzr,
                          double* ritzi, double* bounds, double* q, int ldq, double* workl) {
    return la::dneigh(rnorm, n, h, ldh, ritzr, ritzi, bounds, q, ldq, workl);
}
int arpack_hip_kit_dnapps_host(int kev, int np, const double* shiftr, const double* shifti,
                               double* h, int ldh, double* q, int ldq, double* workl,
                               int64_t nglob) {
    return la::dnapps_host(kev, np, shiftr, shifti, h, ldh, q, ldq, workl, nglob);
}

int arpack_hip_kit_dtrsen(const int* select, int n, double* t, int ldt, double* q, int ldq,
                          double* wr, double* wi, int* m) {
    std::vector<double> work(n > 0 ? n : 1);
    return la::trsen(select, n, t, ldt, q, ldq, wr, wi, *m, work.data());
}

}  // extern "C"
