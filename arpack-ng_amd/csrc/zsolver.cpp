// Complex implicitly restarted Arnoldi (znaupd family), re-hosted as
// coroutines over the complex device kernels (zkernels.hip).
//
// Reference map:
//   ZSolver::run     SRC/znaup2.f  (restart loop)
//   ZSolver::naitr   SRC/znaitr.f  (Arnoldi step, CGS + DGKS with zgemv 'C')
//   ZSolver::getv0   SRC/zgetv0.f  (zlarnv start vector, restart vector)
//   host             zneigh / zngets / zsortc / znapps chase (zdense.cpp)
//   z_aupd           SRC/znaupd.f  (checks, workl layout, iparam)
//   z_eupd           SRC/zneupd.f  (Schur form, ztrsen, Ritz vectors)
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "../../include/arpack_hip.h"
#include "dist.hpp"
#include "zengine.hpp"
#include "zgen.hpp"
#include "zsolve.hpp"

const ahip::DistOp* ahip_dist_view(const arpack_hip_dist* D);

namespace ahip {

// folded complex steps enqueued by this process (arpack_hip_zfold_steps: tests)
static std::atomic<long long> g_zfold_steps{0};

using cd = std::complex<double>;

template <class R>
ZSolverT<R>::~ZSolverT() {
    // no kernel of this solve may still be writing the caller's arrays
    if (a.stream) (void)hipStreamSynchronize(a.stream);
    root.reset();
    zdev::ws_destroy(ws);
    a.release();
}

template <class R>
bool ZSolverT<R>::check_halt() {
    bool bad = a.err.bad();
    if (dist && comm_size(dist->comm) > 1) bad = !dist_all_ok(dist->comm, !bad);
    halted = halted || bad;
    return halted;
}

template <class R>
RciAwait ZSolverT<R>::rci(int ido, int64_t x, int64_t y, int64_t bx) {
    op_x = nullptr;
    op_y = nullptr;
    return RciAwait{&ctx, RciReq{ido, x, y, bx}};
}

template <class R>
RciAwait ZSolverT<R>::op(int ido, int64_t x, int64_t y, int64_t bx) {
    op_x = wd(x);
    op_y = wd(y);
    return RciAwait{&ctx, RciReq{ido, x, y, bx}};
}

template <class R>
RciAwait ZSolverT<R>::op_raw(R* x, int64_t y) {
    op_x = x;
    op_y = wd(y);
    return RciAwait{&ctx, RciReq{1, -1, y, -1}};
}

template <class R>
double ZSolverT<R>::cnorm(const R* x) {
    cd s;
    zdev::dots(ws, n, 0, a.d_v, ldc(), x, x, &s);
    return std::sqrt(std::fabs(s.real()));
}

// zgetv0 (SRC/zgetv0.f): start vector in range(OP), B-orthogonal to V(:,1:j-1)
template <class R>
Task ZSolverT<R>::getv0(bool initv, int j, int itry, int& ierr) {
    const int64_t nn = n;
    ierr = 0;
    if (!initv) {  // zlarnv(idist=2): re/im pairs of one dlaruv stream
        dev::Workspace tmp;
        tmp.stream = a.stream;
        constexpr char fam = std::is_same_v<R, double> ? 'z' : 'c';
        if (dist && dist->seed_mode == 1) {  // PARPACK/SRC/MPI/pzgetv0.f:231-242: per rank
            uint64_t& sd = pgetv0_seed(fam, comm_rank(dist->comm));
            sd = dev::larnv_uniform(tmp, 2 * nn, sd, a.d_resid, 0, 128);
        } else {  // one stream, this rank's slice of 2 n_global reals
            uint64_t& sd = getv0_seed(fam);
            const uint64_t s1 = dev::larnv_uniform(tmp, 2 * nn, sd, a.d_resid, 2 * row0, 128);
            sd = dist ? lcg_advance(sd, 2 * (uint64_t)n_global) : s1;
        }
    }
    if (itry == 1) {
        g_stats.nopx += 1;
        dev::copy(a.stream, 2 * nn, a.d_resid, wd(0));
        co_await op(-1, 0, nn, -1);
        dev::copy(a.stream, 2 * nn, wd(nn), a.d_resid);
    } else if (bmat == 'G') {
        dev::copy(a.stream, 2 * nn, a.d_resid, wd(nn));
    }
    double rnorm0;
    if (bmat == 'G') {
        g_stats.nbx += 1;
        if (itry == 1) dev::copy(a.stream, 2 * nn, a.d_resid, wd(nn));
        co_await rci(2, nn, 0);
        cd s;
        zdev::dots(ws, nn, 0, a.d_v, ldc(), wd(0), a.d_resid, &s);
        rnorm0 = std::sqrt(std::abs(s));
    } else {
        dev::copy(a.stream, 2 * nn, a.d_resid, wd(0));
        rnorm0 = cnorm(a.d_resid);
    }
    rnorm = rnorm0;
    if (j == 1) co_return;
    std::vector<cd> c(j);
    for (int iter = 0;;) {
        zdev::dots<R>(ws, nn, j - 1, a.d_v, ldc(), wd(0), nullptr, c.data());
        zdev::update(ws, nn, j - 1, a.d_v, ldc(), c.data(), a.d_resid, a.d_resid);
        if (bmat == 'G') {
            g_stats.nbx += 1;
            dev::copy(a.stream, 2 * nn, a.d_resid, wd(nn));
            co_await rci(2, nn, 0);
            cd s;
            zdev::dots(ws, nn, 0, a.d_v, ldc(), wd(0), a.d_resid, &s);
            rnorm = std::sqrt(std::abs(s));
        } else {
            dev::copy(a.stream, 2 * nn, a.d_resid, wd(0));
            rnorm = cnorm(a.d_resid);
        }
        if (rnorm > 0.717 * rnorm0) break;
        ++iter;
        if (iter <= 5) {
            rnorm0 = rnorm;
            continue;
        }
        dev::fill(a.stream, 2 * nn, 0.0, a.d_resid);
        rnorm = 0.0;
        ierr = -1;
        break;
    }
    co_return;
}

template <class R>
void ZSolverT<R>::read_state() {
    a.ck(hipMemcpyAsync(ws.st_host, ws.st, sizeof(dev::LzState), hipMemcpyDeviceToHost, a.stream));
    a.sync();
}

template <class R>
void ZSolverT<R>::write_state() {
    a.ck(hipMemcpyAsync(ws.st, ws.st_host, sizeof(dev::LzState), hipMemcpyHostToDevice, a.stream));
}

// The second DGKS sweep of step j (SRC/znaitr.f:730-780, gated on the device
// decision), its finalize, and the give-up zeroing of r.
template <class R>
void ZSolverT<R>::dgks2_tail(int j, int rstart) {
    zdev::step_update(ws, (int64_t)n, j, a.d_v, ldc(), 2, a.d_resid, a.d_resid, true, 2);
    zdev::step_finalize(ws, j + 1, dev::kFinDgks2, j, rstart, 2);
    zdev::step_zero_if(ws, (int64_t)n, a.d_resid);
}

// znaitr for bmat = 'I' with the device-resident step (zstep.hip): every
// reduction and 0.717 decision stays on the device; the free-running form
// (OP = a device complex CSR) enqueues the whole extension and reads the state
// once, the RCI form once per step (where it returns to the caller anyway).  A
// second DGKS sweep in the free-running form parks the rest of the extension
// (st.abort = 2) and is finished here, as in the real engine.
//
// Folded steps (free-running mode 1, ncv <= kZFoldMax + 1; AHIP_ZFOLD=0
// disables), as the real engine's (sym.cpp): step j-1's DGKS sweep is not a
// pass of its own.  Its update pass leaves r (before the sweep) in resid, OP
// runs on r, and step j's first pass (k_zfold_dots, reads only) forms r' = r -
// V s in registers, rebuilds A r' from A r with the Arnoldi relation, and sums
// step j's CGS coefficients and r'^H r' (step j-1's deferred refinement
// check); the second pass (k_zfold_update) forms them again, stores v_j =
// r'/||r'|| and r_j.  Two V passes a step instead of three (config 5 in mode 1
// takes the sweep at every step), no k_zs_place pass, one finalize fewer.
// The first step of a cycle (V(:,k+1) from the restart) and the last one
// (no next step to carry its sweep) take the unfolded form.
template <class R>
Task ZSolverT<R>::naitr_dev(int k, int npk, int& iinfo) {
    const int64_t nn = n;
    const int64_t ipj = 0, irj = nn, ivj = 2 * nn;
    const int ldh = ncv;
    cd* h = workl + ih;
    const bool free_run = csr != nullptr;
    static const bool zfold_env = [] {
        const char* e = getenv("AHIP_ZFOLD");
        return !(e && e[0] == '0');
    }();
    // exact OP only (A r' = A r - A V s): mode 1 with the device CSR -- not the
    // shift-invert's iterative solve
    const bool fold_ok = std::is_same_v<R, double> && zfold_env && free_run && mode == 1 &&
                         ncv <= zdev::kZFoldMax + 1;
    iinfo = 0;
    dev::LzState& sh = *ws.st_host;
    sh.rnorm = rnorm;  // the host's rnorm (zgetv0, or after znapps) seeds the state
    sh.abort = 0;
    sh.dgks = 0;
    sh.zero = 0;
    sh.fold = 0;
    write_state();
    if (fold_ok && k > 0) {
        // H(:, 1:k) after znapps for the fold's t = H s (the device records hold
        // only this cycle's new steps): columns into hcol, the real nonnegative
        // subdiagonals (SRC/znapps.f:405-415) into rec
        std::vector<cd> hc((size_t)k * ncv, cd(0.0));
        std::vector<double> rc((size_t)k, 0.0);
        for (int c = 0; c < k; ++c) {
            for (int i = 0; i <= c; ++i) hc[(size_t)c * ncv + i] = h[i + (size_t)c * ldh];
            if (c > 0) rc[c] = h[c + (size_t)(c - 1) * ldh].real();
        }
        a.ck(hipMemcpyAsync(ws.hcol, hc.data(), sizeof(cd) * hc.size(), hipMemcpyHostToDevice, a.stream));
        a.ck(hipMemcpyAsync(ws.rec, rc.data(), sizeof(double) * rc.size(), hipMemcpyHostToDevice,
                            a.stream));
        a.sync();  // (the staging vectors are about to go)
    }
    bool restart_pending = !(rnorm > 0.0);
    bool folded = false;  // step j's passes form v_j from resid (step j-1's raw r)
    int rstart_j = -1;
    int j = k + 1;
    for (;;) {
        while (j <= k + npk) {
            int rstart = 0;
            if (restart_pending) {  // restart with a vector orthogonal to V (znaitr.f:373-422)
                g_stats.nrstrt += 1;
                int itry = 1, ierr = 0;
                for (;;) {
                    co_await getv0(false, j, itry, ierr);
                    if (ierr >= 0) break;
                    if (++itry <= 3) continue;
                    iinfo = j - 1;
                    co_return;
                }
                restart_pending = false;
                folded = false;
                rstart = 1;
                rstart_j = j;
                sh.abort = 0;
                sh.rnorm = rnorm;
                write_state();
            }
            g_stats.nopx += 1;
            if (folded) {
                // OP on the raw residual, then the two fold passes (see above)
                co_await op_raw(a.d_resid, irj);
                g_zfold_steps.fetch_add(1, std::memory_order_relaxed);
                if constexpr (std::is_same_v<R, double>) {
                    zdev::step_fold_dots(ws, nn, j, a.d_v, ldc(), a.d_resid, wd(irj));
                    zdev::step_finalize(ws, j + 1, dev::kFinCgsFolded, j, rstart, -1);
                    zdev::step_fold_update(ws, nn, j, a.d_v, ldc(), wd(irj), a.d_resid);
                }
            } else {
                // v_j = r / rnorm; the OP input workd(ivj) and, as the reference
                // keeps it, workd(ipj) = B v_j = v_j (znaitr.f:453-476)
                zdev::step_place(ws, nn, a.d_resid, col(j), wd(ivj), free_run ? nullptr : wd(ipj),
                                 Prec<R>::safmin, j);
                co_await op(1, ivj, irj, ipj);
                const R* w = wd(irj);
                // h(1:j,j) = V^H w, wnorm (znaitr.f:545-577)
                zdev::step_dots(ws, nn, j, a.d_v, ldc(), w, -1);
                zdev::step_finalize(ws, j + 1, dev::kFinCgs, j, rstart, -1);
                // r = w - V h with the partials of [V^H r ; r^H r] (znaitr.f:585-640)
                zdev::step_update(ws, nn, j, a.d_v, ldc(), 0, w, a.d_resid, true, -1);
            }
            const bool next_folded = fold_ok && j < k + npk && j <= zdev::kZFoldMax;
            if (next_folded) {
                // the DGKS decision; a sweep's coefficients s, t = H s and st.fold
                // go to the next step's passes (znaitr.f:651-690)
                zdev::step_finalize(ws, j + 1, dev::kFinPostCgsFold, j, rstart, -1);
                folded = true;
            } else {
                zdev::step_finalize(ws, j + 1, dev::kFinPostCgs, j, rstart, -1);
                // DGKS sweeps, each gated on the device decision (znaitr.f:651-780)
                zdev::step_update(ws, nn, j, a.d_v, ldc(), 1, a.d_resid, a.d_resid, true, 1);
                const bool lazy = free_run;
                zdev::step_finalize(ws, j + 1, lazy ? dev::kFinDgks1Lazy : dev::kFinDgks1, j, rstart, 1);
                if (!lazy) dgks2_tail(j, rstart);
                folded = false;
            }
            ++j;
            if (!free_run) {
                read_state();
                rnorm = sh.rnorm;
                if (!(rnorm > 0.0)) restart_pending = true;
            }
        }
        read_state();
        // a park inside a folded cycle leaves resid = r of the step before the
        // parked one, BEFORE its DGKS sweep when st.fold (the sweep was taken)
        const bool was_folded = folded || sh.fold;
        folded = false;  // a resumed cycle restarts with a formed v_j
        auto unfold = [&](int jprev) {  // resid = r' = r - V(:,1:jprev) s
            if (fold_ok && sh.fold)
                zdev::step_update(ws, nn, jprev, a.d_v, ldc(), 1, a.d_resid, a.d_resid, false, -1);
        };
        if (sh.abort == 2) {  // step abort_j needs its second DGKS sweep
            const int ja = sh.abort_j;
            g_stats.nopx -= (k + npk) - ja;  // the later steps were skipped
            const bool parked_by_fold = fold_ok && was_folded && ja < k + npk && sh.fold;
            sh.abort = 0;
            write_state();
            if (parked_by_fold) {
                // parked by step ja+1's kFinCgsFolded: r' was formed only in
                // registers and the second sweep's coefficients V^H r' not summed
                unfold(ja);
                zdev::step_dots(ws, nn, ja, a.d_v, ldc(), a.d_resid, -1);
                zdev::step_finalize(ws, ja + 1, dev::kFinFoldCoef2, ja, ja == rstart_j ? 1 : 0, -1);
            }
            sh.fold = 0;
            write_state();
            dgks2_tail(ja, ja == rstart_j ? 1 : 0);
            j = ja + 1;
            continue;
        }
        if (sh.abort == 3) {  // folded step abort_j: rnorm outside the raw range --
            const int ja = sh.abort_j;  // redo it with v_j formed
            g_stats.nopx -= (k + npk) - ja + 1;
            sh.abort = 0;
            write_state();
            unfold(ja - 1);  // r' of step ja-1
            sh.fold = 0;
            write_state();
            j = ja;
            continue;
        }
        if (sh.abort) {  // rnorm == 0 at step abort_j: restart there
            const int ja = sh.abort_j;
            g_stats.nopx -= (k + npk) - ja + 1;
            sh.fold = 0;
            write_state();
            j = ja;
            restart_pending = true;
            continue;
        }
        break;
    }
    rnorm = sh.rnorm;
    g_stats.nrorth += sh.nrorth;
    g_stats.nitref += sh.nitref;
    sh.nrorth = sh.nitref = 0;
    write_state();
    // H(:, k+1 : k+npk) from the device records: h(1:j,j) and h(j,j-1)
    {
        std::vector<cd> hc((size_t)ncv * npk);
        std::vector<double> beta((size_t)(k + npk));
        a.ck(hipMemcpyAsync(hc.data(), ws.hcol + 2 * (size_t)k * ncv, sizeof(cd) * hc.size(),
                             hipMemcpyDeviceToHost, a.stream));
        a.ck(hipMemcpyAsync(beta.data(), ws.rec, sizeof(double) * beta.size(), hipMemcpyDeviceToHost,
                             a.stream));
        a.sync();
        for (int jj = k + 1; jj <= k + npk; ++jj) {
            cd* colh = h + (size_t)(jj - 1) * ldh;
            std::memcpy(static_cast<void*>(colh), hc.data() + (size_t)(jj - 1 - k) * ncv,
                        sizeof(cd) * jj);
            if (jj > 1) h[(jj - 1) + (size_t)(jj - 2) * ldh] = cd(beta[jj - 1], 0.0);
        }
    }
    co_return;
}

// znaitr: extend a k-step Arnoldi factorization to k+npk steps (host-driven
// decisions: bmat = 'G', where every B*r is a reverse-communication request).
template <class R>
Task ZSolverT<R>::naitr(int k, int npk, int& iinfo) {
    const int64_t nn = n;
    const int64_t ipj = 0, irj = nn, ivj = 2 * nn;
    const int ldh = ncv;
    cd* h = workl + ih;
    const double unfl = Prec<R>::safmin;
    iinfo = 0;
    std::vector<cd> c(ncv + 1);
    static const bool dev_steps = [] {  // AHIP_ZHOST=1: the host-driven step for bmat = 'I' too
        const char* e = getenv("AHIP_ZHOST");
        return !(e && e[0] == '1');
    }();
    // the device finalize stages 2 doubles per complex slot in dynamic LDS
    // (16 (j+1) B, 64 KB a workgroup): wider bases take the host-driven step
    static const int dev_max_ncv = [] {  // AHIP_ZDEV_MAXNCV: test hook for the switch
        const char* e = getenv("AHIP_ZDEV_MAXNCV");
        const int v = e ? atoi(e) : 0;
        return v > 0 && v < zdev::kMaxDevStepNcv ? v : zdev::kMaxDevStepNcv;
    }();
    // (a row-distributed solve takes the host-driven step: its reductions are
    // the allreduced dots of zdev::dots, PARPACK/SRC/MPI/pznaitr.f:580-763)
    if (bmat == 'I' && dev_steps && ncv <= dev_max_ncv && !dist) {
        co_await naitr_dev(k, npk, iinfo);
        if (iinfo > 0) co_return;
    } else
    for (int j = k + 1; j <= k + npk; ++j) {
        double betaj = rnorm;
        if (!(rnorm > 0.0)) {  // restart with a vector orthogonal to V (SRC/znaitr.f:373-422)
            betaj = 0.0;
            g_stats.nrstrt += 1;
            int itry = 1, ierr = 0;
            for (;;) {
                co_await getv0(false, j, itry, ierr);
                if (ierr >= 0) break;
                if (++itry <= 3) continue;
                iinfo = j - 1;
                co_return;
            }
        }
        // v_j = r / rnorm (and workd(ipj) for bmat = 'G') (SRC/znaitr.f:434-450)
        dev::copy(a.stream, 2 * nn, a.d_resid, col(j));
        if (rnorm >= unfl) {
            const double t = 1.0 / rnorm;
            dev::scal(a.stream, 2 * nn, t, col(j));
            dev::scal(a.stream, 2 * nn, t, wd(ipj));
        } else {
            double mul[4];
            const int nm = la::lascl_factors(rnorm, 1.0, mul);
            for (int q = 0; q < nm; ++q) {
                dev::scal(a.stream, 2 * nn, mul[q], col(j));
                dev::scal(a.stream, 2 * nn, mul[q], wd(ipj));
            }
        }
        g_stats.nopx += 1;
        dev::copy(a.stream, 2 * nn, col(j), wd(ivj));
        co_await op(1, ivj, irj, ipj);
        dev::copy(a.stream, 2 * nn, wd(irj), a.d_resid);
        double wnorm;
        if (bmat == 'G') {
            g_stats.nbx += 1;
            co_await rci(2, irj, ipj);
            cd s;
            zdev::dots(ws, nn, 0, a.d_v, ldc(), wd(ipj), a.d_resid, &s);
            wnorm = std::sqrt(std::abs(s));
        } else {
            dev::copy(a.stream, 2 * nn, a.d_resid, wd(ipj));
            wnorm = cnorm(a.d_resid);
        }
        // CGS: h(1:j,j) = V' B r ; r -= V h (SRC/znaitr.f:567-590)
        zdev::dots<R>(ws, nn, j, a.d_v, ldc(), wd(ipj), nullptr, c.data());
        for (int i = 0; i < j; ++i) h[i + (size_t)(j - 1) * ldh] = c[i];
        zdev::update(ws, nn, j, a.d_v, ldc(), c.data(), a.d_resid, a.d_resid);
        if (j > 1) h[(j - 1) + (size_t)(j - 2) * ldh] = cd(betaj, 0.0);
        auto bnorm = [&]() -> Task {  // rnorm of the current resid (with its RCI for 'G')
            if (bmat == 'G') {
                g_stats.nbx += 1;
                dev::copy(a.stream, 2 * nn, a.d_resid, wd(irj));
                co_await rci(2, irj, ipj);
                cd s;
                zdev::dots(ws, nn, 0, a.d_v, ldc(), wd(ipj), a.d_resid, &s);
                rnorm = std::sqrt(std::abs(s));
            } else {
                dev::copy(a.stream, 2 * nn, a.d_resid, wd(ipj));
                rnorm = cnorm(a.d_resid);
            }
        };
        co_await bnorm();
        if (!(rnorm > 0.717 * wnorm)) {  // DGKS (SRC/znaitr.f:651-780)
            g_stats.nrorth += 1;
            for (int iter = 0;;) {
                const double rprev = rnorm;
                zdev::dots<R>(ws, nn, j, a.d_v, ldc(), wd(ipj), nullptr, c.data());
                zdev::update(ws, nn, j, a.d_v, ldc(), c.data(), a.d_resid, a.d_resid);
                for (int i = 0; i < j; ++i) h[i + (size_t)(j - 1) * ldh] += c[i];
                co_await bnorm();
                if (rnorm > 0.717 * rprev) break;
                g_stats.nitref += 1;
                ++iter;
                if (iter <= 1) continue;
                dev::fill(a.stream, 2 * nn, 0.0, a.d_resid);
                rnorm = 0.0;
                break;
            }
        }
    }
    // negligible subdiagonals (SRC/znaitr.f:812-830)
    const double ulp = 2.0 * Prec<R>::eps, smlnum = Prec<R>::safmin * ((double)n / ulp);
    const int kp = k + npk;
    for (int i = std::max(1, k); i <= kp - 1; ++i) {
        double tst1 = zla::cabs1(h[(i - 1) + (size_t)(i - 1) * ldh]) + zla::cabs1(h[i + (size_t)i * ldh]);
        if (tst1 == 0.0) tst1 = zla::lanhs1(kp, h, ldh);
        cd& sub = h[i + (size_t)(i - 1) * ldh];
        if (std::fabs(sub.real()) <= std::max(ulp * tst1, smlnum)) sub = 0.0;
    }
    co_return;
}

template <class R>
Task ZSolverT<R>::run() {
    using la::Which;
    const double eps23 = std::pow(Prec<R>::eps, 2.0 / 3.0);
    int nev = nev0;
    const int np0 = np, kplusp = nev0 + np0;
    int nconv = 0, iter = 0;
    const bool initv = (info != 0);
    info = 0;
    cd* h = workl + ih;
    cd* ritz = workl + iritz;
    cd* bounds = workl + ibounds;
    cd* wl = workl + iw;
    cd* q = workl + iq;
    int ierr = 0, sinfo = 0;
    if (initv) a.upload_resid();
    co_await getv0(initv, 1, 1, ierr);
    if (check_halt()) goto fault;
    if (rnorm == 0.0) {
        info = -9;
        goto done;
    }
    co_await naitr(0, nev, sinfo);
    if (check_halt()) goto fault;
    if (sinfo > 0) {
        np = sinfo;
        mxiter = iter;
        info = -9999;
        goto fail;
    }
    for (;;) {  // SRC/znaup2.f main loop
        ++iter;
        np = kplusp - nev;
        co_await naitr(nev, np, sinfo);
        if (check_halt()) goto fault;
        if (sinfo > 0) {
            np = sinfo;
            mxiter = iter;
            info = -9999;
            goto fail;
        }
        if (zla::zneigh(rnorm, kplusp, h, ncv, ritz, bounds, q, ncv, wl) != 0) {
            info = -8;
            goto fail;
        }
        nev = nev0;
        np = np0;
        std::memcpy(wl + kplusp * kplusp, ritz, sizeof(cd) * kplusp);
        std::memcpy(wl + kplusp * kplusp + kplusp, bounds, sizeof(cd) * kplusp);
        zla::zngets(ishift, which, nev, np, ritz, bounds);
        nconv = 0;
        for (int i = 0; i < nev; ++i) {
            const double rtemp = std::max(eps23, la::lapy2(ritz[np + i].real(), ritz[np + i].imag()));
            if (la::lapy2(bounds[np + i].real(), bounds[np + i].imag()) <= tol * rtemp) ++nconv;
        }
        {
            const int nptemp = np;
            for (int j = 0; j < nptemp; ++j)
                if (bounds[j] == cd(0.0)) {
                    --np;
                    ++nev;
                }
        }
        if (nconv >= nev0 || iter > mxiter || np == 0) {
            h[2] = cd(rnorm, 0.0);  // h(3,1) (SRC/znaup2.f:566)
            Which wp = which;
            switch (which) {
                case Which::LM: wp = Which::SM; break;
                case Which::SM: wp = Which::LM; break;
                case Which::LR: wp = Which::SR; break;
                case Which::SR: wp = Which::LR; break;
                case Which::LI: wp = Which::SI; break;
                case Which::SI: wp = Which::LI; break;
                default: break;
            }
            zla::zsortc(wp, true, kplusp, ritz, bounds);
            for (int j = 0; j < nev0; ++j)
                bounds[j] /= std::max(eps23, la::lapy2(ritz[j].real(), ritz[j].imag()));
            zla::zsortc(Which::LM, true, nev0, bounds, ritz);
            for (int j = 0; j < nev0; ++j)
                bounds[j] *= std::max(eps23, la::lapy2(ritz[j].real(), ritz[j].imag()));
            zla::zsortc(which, true, nconv, ritz, bounds);
            if (iter > mxiter && nconv < nev0) info = 1;
            if (np == 0 && nconv < nev0) info = 2;
            np = nconv;
            goto done;
        } else if (nconv < nev0 && ishift == 1) {
            const int nevbef = nev;
            nev += std::min(nconv, np / 2);
            if (nev == 1 && kplusp >= 6) nev = kplusp / 2;
            else if (nev == 1 && kplusp > 3) nev = 2;
            np = kplusp - nev;
            if (nevbef < nev) zla::zngets(ishift, which, nev, np, ritz, bounds);
        }
        if (ishift == 0) {
            iparam[7] = np;
            co_await rci(3, -1, -1);
            std::memcpy(ritz, wl, sizeof(cd) * np);
        }
        {   // znapps: chase on the host, V*Q and resid update on the device
            zla::znapps_host(nev, np, ritz, h, ncv, q, ncv, wl, n_global);
            const int kev = nev;
            const bool next = h[kev + (size_t)(kev - 1) * ncv].real() > 0.0;
            const int nz = kev + (next ? 1 : 0);
            std::vector<cd> M((size_t)kplusp * nz);
            for (int cc = 0; cc < nz; ++cc)
                for (int r = 0; r < kplusp; ++r) M[(size_t)cc * kplusp + r] = q[r + (size_t)cc * ncv];
            zdev::gemm(ws, n, a.d_v, ldc(), kplusp, nz, M.data(), a.d_v, ldc());
            const cd sigmak = q[(kplusp - 1) + (size_t)(kev - 1) * ncv];
            const cd betak = h[kev + (size_t)(kev - 1) * ncv];
            zdev::axpby(ws, n, sigmak, a.d_resid, betak, next ? col(kev + 1) : nullptr);
        }
        if (bmat == 'G') {
            g_stats.nbx += 1;
            dev::copy(a.stream, 2 * (int64_t)n, a.d_resid, wd(n));
            co_await rci(2, n, 0);
            cd s;
            zdev::dots(ws, n, 0, a.d_v, ldc(), wd(0), a.d_resid, &s);
            rnorm = std::sqrt(la::lapy2(s.real(), s.imag()));
        } else {
            dev::copy(a.stream, 2 * (int64_t)n, a.d_resid, wd(0));
            rnorm = cnorm(a.d_resid);
        }  // (a failure here is caught by the next cycle's check)
    }
done:
    mxiter = iter;
    goto fail;
fault:  // a failed HIP call: the device state is not trustworthy (see sym.cpp)
    mxiter = iter;
    info = -9999;
fail:
    iparam[2] = mxiter;
    co_return;
}

// ---------------------------------------------------------------- drivers ---
template class ZSolverT<double>;
template class ZSolverT<float>;

static std::mutex g_zmu;
template <class R>
static std::unordered_map<const void*, std::unique_ptr<ZSolverT<R>>>& zregistry() {
    static std::unordered_map<const void*, std::unique_ptr<ZSolverT<R>>> m;
    return m;
}

// znaupd (R = double) and cnaupd (R = float: complex64 n-length data, complex128
// host work on a shadow of workl rounded into the caller's at every return).
template <class R>
static void z_aupd(int* ido, const char* bmat, int n, const char* which, int nev, double* tol,
                   std::complex<R>* resid, int ncv, std::complex<R>* v, int ldv, int* iparam,
                   int* ipntr, std::complex<R>* workd, std::complex<R>* workl, int lworkl,
                   R* rwork, int* info, const zdev::ZCsr* csr, zdev::ZShift* zs = nullptr,
                   const DistOp* dist = nullptr, zdev::ZGen* gen = nullptr) {
    constexpr bool kShadow = !std::is_same_v<R, double>;
    if (zs) csr = zs->A;  // free-running shift-invert: OP = (A - sigma I)^{-1} on the device
    if (kShadow && (csr || gen)) {
        *info = -9999;
        *ido = 99;
        return;
    }
    std::lock_guard<std::mutex> lk(g_zmu);
    auto& g_z = zregistry<R>();
    ZSolverT<R>* S = nullptr;
    const int wlen = 3 * ncv * ncv + 5 * ncv;
    auto wl_out = [&]() {
        if constexpr (kShadow)
            for (int t = 0; t < wlen; ++t) workl[t] = std::complex<R>(S->wshadow[t]);
    };
    if (*ido == 0) {
        g_stats = Stats{};
        const la::Which w = la::parse_which(which);
        const int ishift = iparam[0], mxiter = iparam[2], mode = iparam[6];
        int ierr = 0;  // SRC/znaupd.f:473-505
        if (n <= 0) ierr = -1;
        else if (nev <= 0) ierr = -2;
        else if (ncv <= nev || ncv > n || ncv > dev::kMaxNcv) ierr = -3;
        else if (mxiter <= 0) ierr = -4;
        else if (w != la::Which::LM && w != la::Which::SM && w != la::Which::LR &&
                 w != la::Which::SR && w != la::Which::LI && w != la::Which::SI)
            ierr = -5;
        else if (bmat[0] != 'I' && bmat[0] != 'G') ierr = -6;
        else if (lworkl < 3 * ncv * ncv + 5 * ncv) ierr = -7;
        else if (mode < 1 || mode > 3) ierr = -10;
        else if (mode == 1 && bmat[0] == 'G') ierr = -11;
        if (csr && ((zs ? mode != 3 || bmat[0] != 'I' : mode != 1) || csr->n != n))
            ierr = ierr ? ierr : -11;
        if (dist && (csr || dist->nloc != n)) ierr = ierr ? ierr : -1;
        // generalized modes on the device: the operator pair fixes mode and n
        if (gen && (bmat[0] != 'G' || mode != gen->mode || gen->n != n || csr || dist))
            ierr = ierr ? ierr : -11;
        if (ierr != 0) {
            *info = ierr;
            *ido = 99;
            return;
        }
        if (*tol <= 0.0) *tol = Prec<R>::eps;
        g_z.erase(v);  // a previous solve on the same V is abandoned: finish it first
        auto up = std::make_unique<ZSolverT<R>>();
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
        std::memset(static_cast<void*>(workl), 0, sizeof(std::complex<R>) * (size_t)wlen);
        cd* wl = reinterpret_cast<cd*>(workl);
        if constexpr (kShadow) {
            S->wshadow.assign((size_t)wlen, cd(0.0));
            wl = S->wshadow.data();
        }
        S->ih = 0;  // SRC/znaupd.f:541-555
        S->iritz = S->ih + ncv * ncv;
        S->ibounds = S->iritz + ncv;
        S->iq = S->ibounds + ncv;
        S->iw = S->iq + ncv * ncv;
        const int next = S->iw + ncv * ncv + 3 * ncv;
        ipntr[3] = next + 1;
        ipntr[4] = S->ih + 1;
        ipntr[5] = S->iritz + 1;
        ipntr[6] = S->iq + 1;
        ipntr[7] = S->ibounds + 1;
        ipntr[13] = S->iw + 1;
        if (S->a.attach(2 * (int64_t)n, ncv, reinterpret_cast<R*>(resid), reinterpret_cast<R*>(v),
                        2 * ldv, reinterpret_cast<R*>(workd)) != 0 ||
            zdev::ws_create(S->ws, n, ncv, S->a.stream) != hipSuccess) {
            *info = -9999;
            *ido = 99;
            return;
        }
        S->ws.err = &S->a.err;
        S->csr = csr;
        S->gen = gen;
        S->n_global = dist ? dist->n_global : n;
        if (dist) {  // row block of a distributed solve (PARPACK's pznaupd)
            S->dist = dist;
            S->dist_gen = dist->comm_gen;
            S->row0 = dist->row0;
            S->ws.comm = dist->comm;
        }
        S->tol = *tol;
        S->iparam = iparam;
        S->ipntr = ipntr;
        S->workl = wl;
        S->rwork = nullptr;  // the engine needs no real workspace (zneigh's is internal)
        (void)rwork;
        S->root.emplace(S->run());
        start_root(*S->root, S->ctx);
        g_z[v] = std::move(up);
    } else {
        auto it = g_z.find(v);
        if (it == g_z.end()) {
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
            g_z.erase(it);
            *info = -9999;
            *ido = 99;
            return;
        }
        S->tol = *tol;
        S->iparam = iparam;
        S->ipntr = ipntr;
        const RciReq& r = S->ctx.req;
        if constexpr (kShadow) {
            if (r.ido == 3)  // the caller's shifts at workl(ipntr(14))
                for (int t = 0; t < iparam[7]; ++t) S->wshadow[S->iw + t] = cd(workl[S->iw + t]);
        } else {
            S->workl = reinterpret_cast<cd*>(workl);
        }
        if (r.ido == -1 || r.ido == 1 || r.ido == 2) S->a.h2d_workd(2 * r.y, 2 * (int64_t)n);
    }
    // a failed collective or HIP call: info = -9999 (see sym_aupd)
    // (agreed across the ranks first, as in sym_aupd)
    auto comm_broken = [&]() {
        bool bad = S->a.err.bad() || (S->dist && comm_failed(S->dist->comm));
        if (S->dist && comm_size(S->dist->comm) > 1) bad = !dist_all_ok(S->dist->comm, !bad);
        if (!bad) return false;
        (void)hipStreamSynchronize(S->a.stream);
        *info = -9999;
        *ido = 99;
        g_z.erase(v);
        return true;
    };
    for (;;) {
        S->ctx.leaf.resume();
        if (S->ctx.done) break;
        const RciReq r = S->ctx.req;
        // free-running OP requests stay on the device: no agreement per product
        if (!(S->csr && (r.ido == -1 || r.ido == 1)) && comm_broken()) return;
        if (S->gen && (r.ido == -1 || r.ido == 1 || r.ido == 2)) {
            // generalized modes: OP*x and B*x on the device, on the request's
            // workd slices in HBM (complex offsets; bx: M x at ido = 1, mode 3)
            if constexpr (!kShadow) {
                double* W = reinterpret_cast<double*>(S->a.d_workd);
                const double* bx = (r.ido == 1 && r.bx >= 0) ? W + 2 * r.bx : nullptr;
                if (zdev::zgen_apply(*S->gen, S->a.stream, r.ido, W + 2 * r.x, W + 2 * r.y, bx) < 0) {
                    // a solve missed its tolerance (or a HIP error): OP is not
                    // what was asked, so the Arnoldi run stops
                    S->a.sync();
                    *info = -9999;
                    *ido = 99;
                    g_z.erase(v);
                    return;
                }
            }
            continue;
        }
        if (S->csr && (r.ido == -1 || r.ido == 1)) {
            if constexpr (!kShadow) {
                if (!zs) {
                    zdev::zcsr_spmv(S->a.stream, *S->csr, S->op_x, S->op_y);
                } else if (zdev::zshift_apply(*zs, S->a.stream, S->op_x, S->op_y, nullptr) < 0) {
                    // mode 3 (bmat = 'I': B x = x for ido = 1 too): the solve broke
                    // down or missed its tolerance -- OP is not what the
                    // caller asked for, so the Arnoldi run stops
                    S->a.sync();
                    *info = -9999;
                    *ido = 99;
                    g_z.erase(v);
                    return;
                }
            }
            continue;
        }
        if (r.ido == -1 || r.ido == 1 || r.ido == 2) {
            S->a.d2h_workd(2 * r.x, 2 * (int64_t)n);
            if (r.ido == 1 && r.bx >= 0 && S->mode == 3) S->a.d2h_workd(2 * r.bx, 2 * (int64_t)n);
            ipntr[0] = (int)(r.x + 1);
            ipntr[1] = (int)(r.y + 1);
            if (r.bx >= 0) ipntr[2] = (int)(r.bx + 1);
        }
        S->a.sync();
        wl_out();
        *ido = r.ido;
        return;
    }
    if (comm_broken()) return;
    *ido = 99;  // SRC/znaupd.f:585-600
    iparam[2] = S->mxiter;
    iparam[4] = S->np;
    iparam[8] = g_stats.nopx;
    iparam[9] = g_stats.nbx;
    iparam[10] = g_stats.nrorth;
    int inf = S->info;
    if (inf == 2) inf = 3;
    *info = inf;
    S->a.download_all();
    S->a.sync();
    if (S->a.err.bad()) *info = -9999;
    wl_out();
    g_z.erase(v);
}

// zneupd (SRC/zneupd.f): Schur form of H, ztrsen reordering, V <- V*Qh and
// Z = V(:,1:nconv) * X (ztrevc eigenvectors of T) on the device.
// R = float (cneupd): complex128 host work on shadows of workl, d and workev.
template <class R>
static int z_eupd(bool rvec, char howmny, std::complex<R>* d_out, std::complex<R>* z, int ldz,
                  cd sigma, std::complex<R>* workev_out, char bmat, int n, const char* which_s,
                  int nev, double tol, std::complex<R>* resid, int ncv, std::complex<R>* v,
                  int ldv, int* iparam, int* ipntr, std::complex<R>* workd,
                  std::complex<R>* workl_in, int lworkl) {
    using la::Which;
    using CT = std::complex<R>;
    constexpr bool kShadow = !std::is_same_v<R, double>;
    cd* workl = reinterpret_cast<cd*>(workl_in);
    cd* d = reinterpret_cast<cd*>(d_out);
    cd* workev = reinterpret_cast<cd*>(workev_out);
    std::vector<cd> sh[3];  // workl, d, workev
    if constexpr (kShadow) {
        sh[0].assign(workl_in, workl_in + (lworkl > 0 ? lworkl : 0));
        sh[1].assign((size_t)(nev > 0 ? nev : 0), cd(0.0));
        sh[2].assign(2 * (size_t)(ncv > 0 ? ncv : 0), cd(0.0));
        workl = sh[0].data();
        d = sh[1].data();
        workev = sh[2].data();
    }
    struct Back {
        std::vector<cd>* sh;
        CT* out[3];
        ~Back() {
            if constexpr (kShadow)
                for (int k = 0; k < 3; ++k)
                    for (size_t t = 0; t < sh[k].size(); ++t) out[k][t] = CT(sh[k][t]);
        }
    } back{sh, {workl_in, d_out, workev_out}};
    const int mode = iparam[6];
    int nconv = iparam[4];
    const double eps23 = std::pow(Prec<R>::eps, 2.0 / 3.0);
    const Which which = la::parse_which(which_s);
    int ierr = 0;
    if (nconv <= 0) ierr = -14;
    else if (n <= 0) ierr = -1;
    else if (nev <= 0) ierr = -2;
    else if (ncv <= nev || ncv > n) ierr = -3;
    else if (which != Which::LM && which != Which::SM && which != Which::LR && which != Which::SR &&
             which != Which::LI && which != Which::SI)
        ierr = -5;
    else if (bmat != 'I' && bmat != 'G') ierr = -6;
    else if (lworkl < 3 * ncv * ncv + 4 * ncv) ierr = -7;
    else if ((howmny != 'A' && howmny != 'P' && howmny != 'S') && rvec) ierr = -13;
    else if (howmny == 'S') ierr = -12;
    enum { REGULR, SHIFTI } type = REGULR;
    if (mode == 1 || mode == 2) type = REGULR;
    else if (mode == 3) type = SHIFTI;
    else ierr = -10;
    if (mode == 1 && bmat == 'G') ierr = -11;
    if (ierr != 0) return ierr;
    // workl layout (SRC/zneupd.f:458-480)
    const int ih = ipntr[4] - 1, iritz = ipntr[5] - 1, ibounds = ipntr[7] - 1;
    const int ldh = ncv, ldq = ncv;
    const int iheig = ibounds + ldh, ihbds = iheig + ldh, iuptri = ihbds + ldh;
    const int invsub = iuptri + ldh * ncv;
    ipntr[8] = iheig + 1;
    ipntr[10] = ihbds + 1;
    ipntr[11] = iuptri + 1;
    ipntr[12] = invsub + 1;
    const int irz = ipntr[13] - 1 + ncv * ncv, ibd = irz + ncv;
    const double rnorm = workl[ih + 2].real();
    workl[ih + 2] = 0.0;
    cd* T = workl + iuptri;
    cd* Qs = workl + invsub;
    std::vector<int> sel(ncv, 0);
    std::vector<cd> Qh, X;
    if (rvec) {
        bool reord = false;
        for (int j = 0; j < ncv; ++j) workl[ibounds + j] = (double)(j + 1);
        zla::zngets(0, which, nev, ncv - nev, workl + irz, workl + ibounds);
        int numcnv = 0;
        for (int j = 1; j <= ncv; ++j) {
            const cd rz = workl[irz + ncv - j];
            const double rtemp = std::max(eps23, la::lapy2(rz.real(), rz.imag()));
            const int jj = (int)workl[ibounds + ncv - j].real();
            const cd bd = workl[ibd + jj - 1];
            if (numcnv < nconv && la::lapy2(bd.real(), bd.imag()) <= tol * rtemp) {
                sel[jj - 1] = 1;
                ++numcnv;
                if (jj > nconv) reord = true;
            }
        }
        if (numcnv != nconv) return -15;
        std::memcpy(static_cast<void*>(T), workl + ih, sizeof(cd) * ldh * ncv);
        for (int j = 0; j < ncv; ++j)
            for (int i = 0; i < ncv; ++i) Qs[i + (size_t)j * ldq] = (i == j) ? 1.0 : 0.0;
        if (zla::lahqr(true, true, ncv, 1, ncv, T, ldh, workl + iheig, 1, ncv, Qs, ldq) != 0) return -8;
        if (reord) {
            int nconv2 = 0;
            zla::trsen(sel.data(), ncv, T, ldh, Qs, ldq, workl + iheig, nconv2);
            if (nconv2 < nconv) nconv = nconv2;
        }
        for (int j = 0; j < ncv; ++j) workl[ihbds + j] = Qs[(ncv - 1) + (size_t)j * ldq];
        if (type == REGULR) std::memcpy(static_cast<void*>(d), workl + iheig, sizeof(cd) * nconv);
        std::vector<cd> work(ncv + 1);
        zla::geqr2(ncv, nconv, Qs, ldq, workev, workev + ncv);
        Qh.assign((size_t)ncv * ncv, 0.0);
        for (int j = 0; j < ncv; ++j) Qh[(size_t)j * ncv + j] = 1.0;
        zla::unm2r_ln(ncv, ncv, nconv, Qs, ldq, workev, Qh.data(), ncv, work.data());
        for (int j = 0; j < nconv; ++j)
            if (Qs[j + (size_t)j * ldq].real() < 0.0) {
                for (int cc = 0; cc < nconv; ++cc) T[j + (size_t)cc * ldq] = -T[j + (size_t)cc * ldq];
                for (int r = 0; r < nconv; ++r) T[r + (size_t)j * ldq] = -T[r + (size_t)j * ldq];
            }
        if (howmny == 'A') {
            for (int j = 0; j < ncv; ++j) sel[j] = j < nconv;
            std::vector<cd> tw(2 * ncv);
            zla::trevc_right('S', sel.data(), ncv, T, ldq, Qs, ldq, tw.data());
            for (int j = 0; j < nconv; ++j) {
                cd* cj = Qs + (size_t)j * ldq;
                const double s = 1.0 / zla::dznrm2(ncv, cj, 1);
                for (int r = 0; r < ncv; ++r) cj[r] *= s;
                cd dot = 0.0;  // zzdotc(j, ihbds, 1, col j, 1)
                for (int r = 0; r <= j; ++r) dot += std::conj(workl[ihbds + r]) * cj[r];
                workev[j] = dot;
            }
            std::memcpy(static_cast<void*>(workl + ihbds), workev, sizeof(cd) * nconv);
            X.assign((size_t)nconv * nconv, 0.0);  // upper triangular eigenvector block
            for (int cc = 0; cc < nconv; ++cc)
                for (int r = 0; r <= cc; ++r) X[r + (size_t)cc * nconv] = Qs[r + (size_t)cc * ldq];
        }
    } else {
        std::memcpy(static_cast<void*>(d), workl + iritz, sizeof(cd) * nconv);
        std::memcpy(static_cast<void*>(workl + iheig), workl + iritz, sizeof(cd) * nconv);
        std::memcpy(static_cast<void*>(workl + ihbds), workl + ibounds, sizeof(cd) * nconv);
    }
    if (rvec)
        for (int k = 0; k < ncv; ++k) workl[ihbds + k] *= rnorm;
    if (type != REGULR) {
        for (int k = 0; k < ncv; ++k) {
            const cd t = workl[iheig + k];
            workl[ihbds + k] = workl[ihbds + k] / t / t;
        }
        for (int k = 0; k < nconv; ++k) d[k] = 1.0 / workl[iheig + k] + sigma;
    }
    if (!rvec) return 0;
    std::vector<cd> wpur;
    if (howmny == 'A' && type == SHIFTI) {
        wpur.assign(nconv, 0.0);
        for (int j = 0; j < nconv; ++j)
            if (workl[iheig + j] != cd(0.0)) wpur[j] = Qs[(ncv - 1) + (size_t)j * ldq] / workl[iheig + j];
        std::memcpy(static_cast<void*>(workev), wpur.data(), sizeof(cd) * nconv);
    }
    // ---- device: V <- V*Qh ; Z = V(:,1:nconv) * X (+ resid w^T)
    ArraysT<R> a;
    if (a.attach(2 * (int64_t)n, ncv, reinterpret_cast<R*>(resid), reinterpret_cast<R*>(v), 2 * ldv,
                 reinterpret_cast<R*>(workd)) != 0)
        return -9999;
    zdev::Ws ws;
    if (zdev::ws_create(ws, n, ncv, a.stream) != hipSuccess) {
        a.release();
        return -9999;
    }
    ws.err = &a.err;
    if (a.host_mode) {
        a.ck(hipMemcpy2DAsync(a.d_v, sizeof(R) * a.d_ld, v, sizeof(CT) * ldv, sizeof(CT) * n, ncv,
                               hipMemcpyHostToDevice, a.stream));
        a.upload_resid();
    }
    const int64_t ldc = a.d_ld / 2;
    zdev::gemm(ws, n, a.d_v, ldc, ncv, ncv, Qh.data(), a.d_v, ldc);
    const bool zdevp = is_device_pointer(z);
    // a device Z the caller may still be writing on another stream (V / resid /
    // workd in device memory are ordered at attach): complete it first
    if (zdevp && a.host_mode) a.ck(hipDeviceSynchronize());
    R* zd = nullptr;
    int64_t ldzd = ldc;
    if (zdevp) {
        zd = reinterpret_cast<R*>(z);
        ldzd = ldz;
    } else {
        if (hipMalloc(&zd, sizeof(CT) * (size_t)ldc * nconv) != hipSuccess) {
            zdev::ws_destroy(ws);
            a.release();
            return -9999;
        }
    }
    if (howmny == 'A') {
        zdev::gemm(ws, n, a.d_v, ldc, nconv, nconv, X.data(), zd, ldzd);
        if (type == SHIFTI) zdev::ger(ws, n, nconv, a.d_resid, wpur.data(), zd, ldzd);
    } else if (zd != a.d_v) {
        a.ck(hipMemcpy2DAsync(zd, sizeof(CT) * ldzd, a.d_v, sizeof(R) * a.d_ld, sizeof(CT) * n, nconv,
                               hipMemcpyDeviceToDevice, a.stream));
    }
    // V first, then Z: a caller may pass Z = V (the reference's drivers do)
    if (a.host_mode)
        a.ck(hipMemcpy2DAsync(v, sizeof(CT) * ldv, a.d_v, sizeof(R) * a.d_ld, sizeof(CT) * n, ncv,
                               hipMemcpyDeviceToHost, a.stream));
    if (!zdevp) {
        a.ck(hipMemcpy2DAsync(z, sizeof(CT) * ldz, zd, sizeof(CT) * ldc, sizeof(CT) * n, nconv,
                               hipMemcpyDeviceToHost, a.stream));
    }
    a.sync();
    if (!zdevp) (void)hipFree(zd);
    zdev::ws_destroy(ws);
    const bool bad = a.err.bad();  // a failed copy or a kernel fault of this call
    a.release();
    return bad ? -9999 : 0;
}

}  // namespace ahip

// ---------------------------------------------------------------- C-ABI -----
struct arpack_hip_zcsr {
    ahip::zdev::ZCsr A;
};

const ahip::zdev::ZCsr* ahip_zcsr_view(const arpack_hip_zcsr* Z) { return Z ? &Z->A : nullptr; }

using ahip::cd;

extern "C" {

void znaupd_c(int* ido, char const* bmat, int n, char const* which, int nev, double tol, a_dcomplex* resid,
              int ncv, a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int lworkl,
              double* rwork, int* info) {
    ahip::z_aupd(ido, bmat, n, which, nev, &tol, (cd*)resid, ncv, (cd*)v, ldv, iparam, ipntr, (cd*)workd,
                 (cd*)workl, lworkl, rwork, info, nullptr);
}

void znaupd_(int* ido, char const* bmat, int* n, char const* which, int* nev, double* tol, a_dcomplex* resid,
             int* ncv, a_dcomplex* v, int* ldv, int* iparam, int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int* lworkl,
             double* rwork, int* info, size_t, size_t) {
    ahip::z_aupd(ido, bmat, *n, which, *nev, tol, (cd*)resid, *ncv, (cd*)v, *ldv, iparam, ipntr,
                 (cd*)workd, (cd*)workl, *lworkl, rwork, info, nullptr);
}

void zneupd_c(int rvec, char const* howmny, int const* select, a_dcomplex* d, a_dcomplex* z, int ldz, a_dcomplex sigma,
              a_dcomplex* workev, char const* bmat, int n, char const* which, int nev, double tol, a_dcomplex* resid,
              int ncv, a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int lworkl,
              double* rwork, int* info) {
    (void)select;
    (void)rwork;
    const cd s(__real__ sigma, __imag__ sigma);
    *info = ahip::z_eupd(rvec != 0, howmny[0], (cd*)d, (cd*)z, ldz, s, (cd*)workev, bmat[0], n, which, nev,
                         tol, (cd*)resid, ncv, (cd*)v, ldv, iparam, ipntr, (cd*)workd, (cd*)workl, lworkl);
}

void zneupd_(int* rvec, char const* howmny, int* select, a_dcomplex* d, a_dcomplex* z, int* ldz, a_dcomplex* sigma,
             a_dcomplex* workev, char const* bmat, int* n, char const* which, int* nev, double* tol, a_dcomplex* resid,
             int* ncv, a_dcomplex* v, int* ldv, int* iparam, int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int* lworkl,
             double* rwork, int* info, size_t, size_t, size_t) {
    (void)select;
    (void)rwork;
    const cd s = *reinterpret_cast<const cd*>(sigma);
    *info = ahip::z_eupd(*rvec != 0, howmny[0], (cd*)d, (cd*)z, *ldz, s, (cd*)workev, bmat[0], *n, which,
                         *nev, *tol, (cd*)resid, *ncv, (cd*)v, *ldv, iparam, ipntr, (cd*)workd, (cd*)workl,
                         *lworkl);
}

// ---- complex64 family (ICB/arpack.h:10-11; SRC/cnaupd.f, SRC/cneupd.f) ----
typedef std::complex<float> cf;

void cnaupd_c(int* ido, char const* bmat, int n, char const* which, int nev, float tol,
              a_fcomplex* resid, int ncv, a_fcomplex* v, int ldv, int* iparam, int* ipntr,
              a_fcomplex* workd, a_fcomplex* workl, int lworkl, float* rwork, int* info) {
    double t = tol;
    ahip::z_aupd<float>(ido, bmat, n, which, nev, &t, (cf*)resid, ncv, (cf*)v, ldv, iparam, ipntr,
                        (cf*)workd, (cf*)workl, lworkl, rwork, info, nullptr);
}

void cnaupd_(int* ido, char const* bmat, int* n, char const* which, int* nev, float* tol,
             a_fcomplex* resid, int* ncv, a_fcomplex* v, int* ldv, int* iparam, int* ipntr,
             a_fcomplex* workd, a_fcomplex* workl, int* lworkl, float* rwork, int* info, size_t,
             size_t) {
    double t = *tol;
    ahip::z_aupd<float>(ido, bmat, *n, which, *nev, &t, (cf*)resid, *ncv, (cf*)v, *ldv, iparam,
                        ipntr, (cf*)workd, (cf*)workl, *lworkl, rwork, info, nullptr);
    *tol = (float)t;
}

void cneupd_c(int rvec, char const* howmny, int const* select, a_fcomplex* d, a_fcomplex* z,
              int ldz, a_fcomplex sigma, a_fcomplex* workev, char const* bmat, int n,
              char const* which, int nev, float tol, a_fcomplex* resid, int ncv, a_fcomplex* v,
              int ldv, int* iparam, int* ipntr, a_fcomplex* workd, a_fcomplex* workl, int lworkl,
              float* rwork, int* info) {
    (void)select;
    (void)rwork;
    const cd s(__real__ sigma, __imag__ sigma);
    *info = ahip::z_eupd<float>(rvec != 0, howmny[0], (cf*)d, (cf*)z, ldz, s, (cf*)workev, bmat[0],
                                n, which, nev, tol, (cf*)resid, ncv, (cf*)v, ldv, iparam, ipntr,
                                (cf*)workd, (cf*)workl, lworkl);
}

void cneupd_(int* rvec, char const* howmny, int* select, a_fcomplex* d, a_fcomplex* z, int* ldz,
             a_fcomplex* sigma, a_fcomplex* workev, char const* bmat, int* n, char const* which,
             int* nev, float* tol, a_fcomplex* resid, int* ncv, a_fcomplex* v, int* ldv,
             int* iparam, int* ipntr, a_fcomplex* workd, a_fcomplex* workl, int* lworkl,
             float* rwork, int* info, size_t, size_t, size_t) {
    (void)select;
    (void)rwork;
    const cf sg = *reinterpret_cast<const cf*>(sigma);
    *info = ahip::z_eupd<float>(*rvec != 0, howmny[0], (cf*)d, (cf*)z, *ldz, cd(sg), (cf*)workev,
                                bmat[0], *n, which, *nev, *tol, (cf*)resid, *ncv, (cf*)v, *ldv,
                                iparam, ipntr, (cf*)workd, (cf*)workl, *lworkl);
}

// ---- complex host kit exports (CPU-testable; tests/test_kit_z.py) ----
int arpack_hip_kit_zlahqr(int n, a_dcomplex* h, int ldh, a_dcomplex* w, a_dcomplex* z, int ldz) {
    return ahip::zla::lahqr(true, true, n, 1, n, (cd*)h, ldh, (cd*)w, 1, n, (cd*)z, ldz);
}
int arpack_hip_kit_ztrevc(char howmny, int* select, int n, a_dcomplex* t, int ldt, a_dcomplex* vr,
                          int ldvr) {
    std::vector<cd> work(2 * (size_t)n + 1);
    return ahip::zla::trevc_right(howmny, select, n, (cd*)t, ldt, (cd*)vr, ldvr, work.data());
}
int arpack_hip_kit_ztrsen(const int* select, int n, a_dcomplex* t, int ldt, a_dcomplex* q, int ldq,
                          a_dcomplex* w, int* m) {
    return ahip::zla::trsen(select, n, (cd*)t, ldt, (cd*)q, ldq, (cd*)w, *m);
}
void arpack_hip_kit_zsortc(char const* which, int apply, int n, a_dcomplex* x, a_dcomplex* y) {
    ahip::zla::zsortc(ahip::la::parse_which(which), apply != 0, n, (cd*)x, (cd*)y);
}
void arpack_hip_kit_zngets(int ishift, char const* which, int kev, int np, a_dcomplex* ritz,
                           a_dcomplex* bounds) {
    ahip::zla::zngets(ishift, ahip::la::parse_which(which), kev, np, (cd*)ritz, (cd*)bounds);
}
int arpack_hip_kit_zneigh(double rnorm, int n, const a_dcomplex* h, int ldh, a_dcomplex* ritz,
                          a_dcomplex* bounds, a_dcomplex* q, int ldq) {
    std::vector<cd> wk((size_t)n * n + 2 * (size_t)n + 1);
    return ahip::zla::zneigh(rnorm, n, (const cd*)h, ldh, (cd*)ritz, (cd*)bounds, (cd*)q, ldq, wk.data());
}
void arpack_hip_kit_znapps_host(int kev, int np, const a_dcomplex* shift, a_dcomplex* h, int ldh,
                                a_dcomplex* q, int ldq, int64_t nglob) {
    std::vector<cd> wk((size_t)kev + np + 1);
    ahip::zla::znapps_host(kev, np, (const cd*)shift, (cd*)h, ldh, (cd*)q, ldq, wk.data(), nglob);
}

int arpack_hip_zcsr_create(arpack_hip_zcsr** out, int64_t n, int64_t nnz, const int64_t* rowptr,
                           const int32_t* col, const double* val) {
    auto* Z = new arpack_hip_zcsr;
    int64_t* rp = nullptr;
    int32_t* c = nullptr;
    double* v = nullptr;
    if (hipMalloc(&rp, sizeof(int64_t) * (n + 1)) || hipMalloc(&c, sizeof(int32_t) * (nnz ? nnz : 1)) ||
        hipMalloc(&v, sizeof(double) * 2 * (nnz ? nnz : 1)) ||
        hipMemcpy(rp, rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDefault) ||
        (nnz && (hipMemcpy(c, col, sizeof(int32_t) * nnz, hipMemcpyDefault) ||
                 hipMemcpy(v, val, sizeof(double) * 2 * nnz, hipMemcpyDefault)))) {
        (void)hipFree(rp);
        (void)hipFree(c);
        (void)hipFree(v);
        delete Z;
        return -1;
    }
    Z->A.n = n;
    Z->A.nnz = nnz;
    Z->A.rowptr = rp;
    Z->A.col = c;
    Z->A.val = v;
    Z->A.owned = true;
    // XCD column split when it pays; optional: if it cannot be built (e.g. no
    // memory for the slices) it is freed and the wave-per-row kernel serves A
    (void)ahip::zdev::zcsr_build_split(Z->A);
    *out = Z;
    return 0;
}

int arpack_hip_gen_zrandom(arpack_hip_zcsr** out, int64_t n, int per_row, uint32_t seed, double dshift) {
    auto* Z = new arpack_hip_zcsr;
    if (ahip::zdev::gen_zrandom(Z->A, n, per_row, seed, dshift) != 0) {
        delete Z;
        return -1;
    }
    (void)ahip::zdev::zcsr_build_split(Z->A);  // optional, as in arpack_hip_zcsr_create
    *out = Z;
    return 0;
}

void arpack_hip_zcsr_destroy(arpack_hip_zcsr* Z) {
    if (!Z) return;
    ahip::zdev::zcsr_free_split(Z->A);
    if (Z->A.owned) {
        (void)hipFree((void*)Z->A.rowptr);
        (void)hipFree((void*)Z->A.col);
        (void)hipFree((void*)Z->A.val);
    }
    delete Z;
}

int arpack_hip_zcsr_info(const arpack_hip_zcsr* Z, int64_t* n, int64_t* nnz) {
    *n = Z->A.n;
    *nnz = Z->A.nnz;
    return 0;
}

int arpack_hip_zcsr_tile_info(const arpack_hip_zcsr* Z, int* form, int64_t* stored) {
    const auto& A = Z->A;
    *form = !A.split ? 0 : !A.tile ? 1 : A.t_pk ? 3 : 2;
    *stored = A.tile ? A.t_stored : A.nnz;
    return 0;
}

int arpack_hip_zcsr_download(const arpack_hip_zcsr* Z, int64_t* rowptr, int32_t* col, double* val) {
    const auto& A = Z->A;
    if (hipMemcpy(rowptr, A.rowptr, sizeof(int64_t) * (A.n + 1), hipMemcpyDeviceToHost) ||
        hipMemcpy(col, A.col, sizeof(int32_t) * A.nnz, hipMemcpyDeviceToHost) ||
        hipMemcpy(val, A.val, sizeof(double) * 2 * A.nnz, hipMemcpyDeviceToHost))
        return -1;
    return 0;
}

int arpack_hip_zcsr_spmv(const arpack_hip_zcsr* Z, const double* x, double* y) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;  // the caller's x (see csr_spmv)
    ahip::zdev::zcsr_spmv(nullptr, Z->A, x, y);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

void arpack_hip_znaupd_zcsr(const arpack_hip_zcsr* Z, int* ido, char const* bmat, int n, char const* which,
                            int nev, double* tol, a_dcomplex* resid, int ncv, a_dcomplex* v, int ldv, int* iparam,
                            int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int lworkl, double* rwork, int* info) {
    ahip::z_aupd(ido, bmat, n, which, nev, tol, (cd*)resid, ncv, (cd*)v, ldv, iparam, ipntr, (cd*)workd,
                 (cd*)workl, lworkl, rwork, info, &Z->A);
}

// ---- PARPACK-style complex RCI (ICB/parpack.h:30-33 pcnaupd_c / pznaupd_c
//      with n = LOCAL rows; PARPACK/SRC/MPI/pznaupd.f decomposition) ----
void arpack_hip_pznaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, double tol, a_dcomplex* resid, int ncv,
                          a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd,
                          a_dcomplex* workl, int lworkl, double* rwork, int* info) {
    ahip::z_aupd(ido, bmat, n, which, nev, &tol, (cd*)resid, ncv, (cd*)v, ldv, iparam, ipntr,
                 (cd*)workd, (cd*)workl, lworkl, rwork, info, nullptr, nullptr, ahip_dist_view(D));
}
void arpack_hip_pcnaupd_c(const arpack_hip_dist* D, int* ido, char const* bmat, int n,
                          char const* which, int nev, float tol, a_fcomplex* resid, int ncv,
                          a_fcomplex* v, int ldv, int* iparam, int* ipntr, a_fcomplex* workd,
                          a_fcomplex* workl, int lworkl, float* rwork, int* info) {
    double t = tol;
    ahip::z_aupd<float>(ido, bmat, n, which, nev, &t, (cf*)resid, ncv, (cf*)v, ldv, iparam, ipntr,
                        (cf*)workd, (cf*)workl, lworkl, rwork, info, nullptr, nullptr,
                        ahip_dist_view(D));
}
// p[cz]neupd (PARPACK/SRC/MPI/pzneupd.f): no collective -- the Schur / Ritz
// work is replicated host work and the n-length products are row-local
void arpack_hip_pzneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, a_dcomplex* d, a_dcomplex* z, int ldz,
                          a_dcomplex sigma, a_dcomplex* workev, char const* bmat, int n,
                          char const* which, int nev, double tol, a_dcomplex* resid, int ncv,
                          a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd,
                          a_dcomplex* workl, int lworkl, double* rwork, int* info) {
    (void)D;
    zneupd_c(rvec, howmny, select, d, z, ldz, sigma, workev, bmat, n, which, nev, tol, resid, ncv,
             v, ldv, iparam, ipntr, workd, workl, lworkl, rwork, info);
}
void arpack_hip_pcneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, a_fcomplex* d, a_fcomplex* z, int ldz,
                          a_fcomplex sigma, a_fcomplex* workev, char const* bmat, int n,
                          char const* which, int nev, float tol, a_fcomplex* resid, int ncv,
                          a_fcomplex* v, int ldv, int* iparam, int* ipntr, a_fcomplex* workd,
                          a_fcomplex* workl, int lworkl, float* rwork, int* info) {
    (void)D;
    cneupd_c(rvec, howmny, select, d, z, ldz, sigma, workev, bmat, n, which, nev, tol, resid, ncv,
             v, ldv, iparam, ipntr, workd, workl, lworkl, rwork, info);
}

// ---- device shift-invert operator (zsolve.hip) ----
struct arpack_hip_zshift {
    ahip::zdev::ZShift S;
};

int arpack_hip_zshift_create(arpack_hip_zshift** out, const arpack_hip_zcsr* A, double sigma_re,
                             double sigma_im, double rtol, int maxit) {
    if (!out || !A || !(rtol > 0.0) || maxit < 1) return -1;
    auto* Z = new arpack_hip_zshift;
    if (ahip::zdev::zshift_create(Z->S, &A->A, cd(sigma_re, sigma_im), rtol, maxit) != 0) {
        delete Z;
        return -2;
    }
    *out = Z;
    return 0;
}

void arpack_hip_zshift_destroy(arpack_hip_zshift* Z) {
    if (!Z) return;
    ahip::zdev::zshift_destroy(Z->S);
    delete Z;
}

// 0: BiCGStab (the default), 1: a direct solve of a tridiagonal A - sigma I
// (zgttrf on the host, the triangular solves as device scans, ztri.hip)
int arpack_hip_zshift_set_method(arpack_hip_zshift* Z, int method) {
    if (!Z || method < 0 || method > 1) return -1;
    ahip::zdev::zshift_tridiag_free(Z->S);  // (method 0 again)
    if (method == 1) return ahip::zdev::zshift_tridiag_factor(Z->S) == 0 ? 0 : -1;
    return 0;
}

int arpack_hip_zshift_solve(arpack_hip_zshift* Z, const double* x, double* y, double* relres) {
    if (!Z || !x || !y || x == y) return -2;  // as arpack_hip_dshift_solve
    return ahip::zdev::zshift_apply(Z->S, nullptr, x, y, relres);
}

int arpack_hip_zshift_stats(const arpack_hip_zshift* Z, long long* solves, long long* iters,
                            long long* failures, double* max_relres, double* ms,
                            double* bytes_per_iter) {
    if (!Z) return -1;
    const auto& S = Z->S;
    if (solves) *solves = S.n_solves;
    if (iters) *iters = S.n_iters;
    if (failures) *failures = S.n_fail;
    if (max_relres) *max_relres = S.max_relres;
    if (ms) *ms = S.ms_total;
    if (bytes_per_iter) *bytes_per_iter = ahip::zdev::zshift_iter_bytes(S);
    return 0;
}

void arpack_hip_znaupd_zshift(arpack_hip_zshift* Z, int* ido, char const* bmat, int n,
                              char const* which, int nev, double* tol, a_dcomplex* resid, int ncv,
                              a_dcomplex* v, int ldv, int* iparam, int* ipntr, a_dcomplex* workd,
                              a_dcomplex* workl, int lworkl, double* rwork, int* info) {
    ahip::z_aupd(ido, bmat, n, which, nev, tol, (cd*)resid, ncv, (cd*)v, ldv, iparam, ipntr,
                 (cd*)workd, (cd*)workl, lworkl, rwork, info, nullptr, &Z->S);
}

long long arpack_hip_zfold_steps(void) { return ahip::g_zfold_steps.load(); }

// ---- znaupd's generalized modes on the device (zgen.cpp) ----
struct arpack_hip_zgen {
    ahip::zdev::ZGen G;
};

int arpack_hip_zgen_create(arpack_hip_zgen** out, const arpack_hip_zcsr* A, const arpack_hip_zcsr* M,
                           int mode, double sigma_re, double sigma_im, double rtol, int maxit) {
    if (!out || !(rtol > 0.0) || maxit < 1) return -1;
    auto* Z = new arpack_hip_zgen;
    const int rc = ahip::zdev::zgen_create(Z->G, A, M, mode, cd(sigma_re, sigma_im), rtol, maxit);
    if (rc != 0) {
        delete Z;
        return rc;
    }
    *out = Z;
    return 0;
}

// 0: BiCGStab on C (the default), 1: the direct tridiagonal solve of C
// (ztri.hip; A and M tridiagonal, as zndrv4.f's pair it factors with zgttrf)
int arpack_hip_zgen_set_method(arpack_hip_zgen* Z, int method) {
    if (!Z || method < 0 || method > 1) return -1;
    ahip::zdev::zshift_tridiag_free(Z->G.S);
    if (method == 1) return ahip::zdev::zshift_tridiag_factor(Z->G.S) == 0 ? 0 : -1;
    return 0;
}

void arpack_hip_zgen_destroy(arpack_hip_zgen* Z) {
    if (!Z) return;
    ahip::zdev::zgen_destroy(Z->G);
    delete Z;
}

int arpack_hip_zgen_stats(const arpack_hip_zgen* Z, long long* solves, long long* iters,
                          long long* failures, double* max_relres) {
    if (!Z) return -1;
    const auto& S = Z->G.S;
    if (solves) *solves = S.n_solves;
    if (iters) *iters = S.n_iters;
    if (failures) *failures = S.n_fail;
    if (max_relres) *max_relres = S.max_relres;
    return 0;
}

void arpack_hip_znaupd_gen(arpack_hip_zgen* Z, int* ido, char const* bmat, int n, char const* which,
                           int nev, double* tol, a_dcomplex* resid, int ncv, a_dcomplex* v, int ldv,
                           int* iparam, int* ipntr, a_dcomplex* workd, a_dcomplex* workl, int lworkl,
                           double* rwork, int* info) {
    if (!Z) {
        *info = -9999;
        *ido = 99;
        return;
    }
    ahip::z_aupd(ido, bmat, n, which, nev, tol, (cd*)resid, ncv, (cd*)v, ldv, iparam, ipntr,
                 (cd*)workd, (cd*)workl, lworkl, rwork, info, nullptr, nullptr, nullptr, &Z->G);
}

}  // extern "C"
