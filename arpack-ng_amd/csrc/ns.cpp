// Nonsymmetric implicitly restarted Arnoldi: the dnaup2 restart loop re-hosted
// as a coroutine over the shared device step machinery (sym.cpp: getv0 and the
// Arnoldi step, which records h(1:j,j) on the device when `arnoldi` is set).
//
// Reference map:
//   Solver::run_ns   SRC/dnaup2.f:179-846   (restart loop, nev adaptation)
//   Solver::saitr    SRC/dnaitr.f:209-840   (Arnoldi step; CGS + DGKS)
//   Solver::napps    SRC/dnapps.f:143-649   (shifts on H host-side, V*Q on device)
//   la::dneigh/dngets/dnconv/dsortc          (SRC/dneigh.f, dngets.f, dnconv.f, dsortc.f)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "engine.hpp"

namespace ahip {

template <class R>
Task SolverT<R>::run_ns() {
    using la::Which;
    // ---- dnaup2 initialisation (SRC/dnaup2.f:272-317)
    const double eps23 = std::pow(eps, 2.0 / 3.0);
    int nev = nev0;
    const int np0 = np;
    const int kplusp = nev0 + np0;
    int nconv = 0, iter = 0, numcnv = nev;
    const bool initv = (info != 0);
    info = 0;
    double* h = workl + ih;
    double* ritzr = workl + iritz;
    double* ritzi = workl + iritzi;
    double* bounds = workl + ibounds;
    double* wl = workl + iw;
    int ierr = 0, sinfo = 0;

    if (initv) a.upload_resid();
    co_await getv0(initv, 1, 1, ierr);
    if (check_halt()) goto fault;
    if (rnorm == 0.0) {
        info = -9;
        goto done;
    }
    ws.st_host->rnorm = rnorm;
    ws.st_host->abort = 0;
    write_state();

    co_await saitr(0, nev, sinfo);
    if (halted) goto fault;
    if (sinfo > 0) {
        np = sinfo;
        mxiter = iter;
        info = -9999;
        goto fail;
    }

    for (;;) {  // MAIN ARNOLDI ITERATION LOOP (SRC/dnaup2.f:385-822)
        if (pause_budget == 0) co_await rci(kPauseIdo, -1, -1);
        if (pause_budget > 0) --pause_budget;
        ++iter;
        np = kplusp - nev;
        co_await saitr(nev, np, sinfo);
        if (halted) goto fault;
        if (sinfo > 0) {
            np = sinfo;
            mxiter = iter;
            info = -9999;
            goto fail;
        }
        // Ritz values of H and their error bounds (SRC/dnaup2.f:447-462)
        if (la::dneigh(rnorm, kplusp, h, ncv, ritzr, ritzi, bounds, workl + iq, ncv, wl) != 0) {
            info = -8;
            goto fail;
        }
        std::memcpy(wl + kplusp * kplusp, ritzr, sizeof(double) * kplusp);
        std::memcpy(wl + kplusp * kplusp + kplusp, ritzi, sizeof(double) * kplusp);
        std::memcpy(wl + kplusp * kplusp + 2 * kplusp, bounds, sizeof(double) * kplusp);
        nev = nev0;
        np = np0;
        numcnv = nev;
        la::dngets(ishift, which, nev, np, ritzr, ritzi, bounds);
        if (nev == nev0 + 1) numcnv = nev0 + 1;
        std::memcpy(wl + 2 * np, bounds + np, sizeof(double) * nev);
        nconv = la::dnconv(nev, ritzr + np, ritzi + np, wl + 2 * np, tol, eps);
        {
            const int nptemp = np;
            for (int j = 0; j < nptemp; ++j)
                if (bounds[j] == 0.0) {
                    --np;
                    ++nev;
                }
        }
        if (nconv >= numcnv || iter > mxiter || np == 0) {
            // prepare to exit (SRC/dnaup2.f:546-650)
            h[2] = rnorm;  // h(3,1): rnorm for dneupd
            Which wp = Which::SR;
            switch (which) {
                case Which::LM: wp = Which::SR; break;
                case Which::SM: wp = Which::LR; break;
                case Which::LR: wp = Which::SM; break;
                case Which::SR: wp = Which::LM; break;
                case Which::LI: wp = Which::SM; break;
                case Which::SI: wp = Which::LM; break;
                default: break;
            }
            la::dsortc(wp, true, kplusp, ritzr, ritzi, bounds);
            switch (which) {
                case Which::LM: wp = Which::SM; break;
                case Which::SM: wp = Which::LM; break;
                case Which::LR: wp = Which::SR; break;
                case Which::SR: wp = Which::LR; break;
                case Which::LI: wp = Which::SI; break;
                case Which::SI: wp = Which::LI; break;
                default: break;
            }
            la::dsortc(wp, true, kplusp, ritzr, ritzi, bounds);
            for (int j = 0; j < numcnv; ++j)
                bounds[j] /= std::max(eps23, la::lapy2(ritzr[j], ritzi[j]));
            la::dsortc(Which::LR, true, numcnv, bounds, ritzr, ritzi);
            for (int j = 0; j < numcnv; ++j)
                bounds[j] *= std::max(eps23, la::lapy2(ritzr[j], ritzi[j]));
            la::dsortc(which, true, nconv, ritzr, ritzi, bounds);
            if (iter > mxiter && nconv < numcnv) info = 1;
            if (np == 0 && nconv < numcnv) info = 2;
            np = nconv;
            goto done;
        } else if (nconv < numcnv && ishift == 1) {
            // anti-stagnation: grow nev (SRC/dnaup2.f:652-688, incl. the kplusp-2 cap)
            const int nevbef = nev;
            nev += std::min(nconv, np / 2);
            if (nev == 1 && kplusp >= 6) nev = kplusp / 2;
            else if (nev == 1 && kplusp > 3) nev = 2;
            if (nev > kplusp - 2) nev = kplusp - 2;
            np = kplusp - nev;
            if (nevbef < nev) la::dngets(ishift, which, nev, np, ritzr, ritzi, bounds);
        }
        if (ishift == 0) {  // user shifts: real parts at workl(ipntr(14)), imag after
            iparam[7] = np;
            co_await rci(3, -1, -1);
            std::memcpy(ritzr, wl, sizeof(double) * np);
            std::memcpy(ritzi, wl + np, sizeof(double) * np);
        }
        {
            // shifts on H (host), then V*Q and the residual update (device)
            double* q = workl + iq;
            std::vector<double> wk(ncv);
            const int kp_now = nev + np;
            nev = la::dnapps_host(nev, np, ritzr, ritzi, h, ncv, q, ncv, wk.data(), n_global);
            if (np > 0) {
                // dnapps: sigmak = q(kplusp, kev), betak = h(kev+1, kev) with the
                // (possibly incremented) kev (SRC/dnapps.f:583-640)
                const double sigmak = q[(kp_now - 1) + (size_t)(nev - 1) * ncv];
                const double betak = h[nev + (size_t)(nev - 1) * ncv];
                vq_device(nev, kp_now, sigmak, betak);
            }
        }
        // B-norm of the updated residual (SRC/dnaup2.f:769-805)
        if (bmat == 'G') {
            g_stats.nbx += 1;
            dev::copy(a.stream, n, a.d_resid, a.d_workd + n);
            co_await rci(2, n, 0);
            dev::dots(ws, n, 0, a.d_v, a.d_ld, a.d_workd, a.d_resid, -1);
            fin(1, dev::kFinNorm, 0, 0, -1);
        } else {
            fin(1, dev::kFinNorm, 0, 0, -1);  // r'r partials came with V*Q
        }
        if (free_run && bmat != 'G') {  // the next cycle queues behind V*Q (see run())
            rnorm_stale = true;
            continue;
        }
        read_state();  // (a failure here is caught by the next cycle's check)
        rnorm = ws.st_host->rnorm;
    }
done:
    mxiter = iter;
    nev0 = numcnv;
    goto fail;
fault:  // a failed HIP call: the device state is not trustworthy (see sym.cpp)
    mxiter = iter;
    info = -9999;
fail:
    if (ybuf) dev::copy(a.stream, n, ybuf, a.d_workd + n);  // workd(irj) = the last OP x (saitr)
    iparam[2] = mxiter;
    co_return;
}

template Task SolverT<double>::run_ns();
template Task SolverT<float>::run_ns();

}  // namespace ahip
