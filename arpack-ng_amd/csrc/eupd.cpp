// dseupd: Ritz values / Ritz vectors from the final Lanczos factorization
// (SRC/dseupd.f:218-867).  The ncv-sized work (dsgets re-selection, dsteqr,
// spectral transforms, Householder QR of the eigenvector matrix) is done on
// the host in the caller's workl exactly as the reference lays it out; the
// n-length products are device kernels: V <- V * (H_1 ... H_nconv) as ONE
// tall-skinny GEMM (the reference applies nconv rank-1 reflectors with
// dorm2r, SRC/dseupd.f:742-746), Z = V(:,1:nconv), and the rank-1
// purification Z += resid * w' for the spectral-transform modes (:840-857).
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../../include/arpack_hip.h"
#include "engine.hpp"

namespace ahip {

// R = float (sseupd): the ncv-sized work runs in double on a shadow of the
// caller's float workl (copied back, rounded, on return), d is rounded at the end.
template <class R>
static int sym_eupd(int rvec, char howmny, int* select, R* d_out, R* z, int ldz, double sigma,
                    char bmat, int n, const char* which_s, int nev, double tol, R* resid, int ncv,
                    R* v, int ldv, int* iparam, int* ipntr, R* workd, R* workl_in, int lworkl,
                    const DistOp* dist = nullptr) {
    using la::Which;
    constexpr bool kShadow = !std::is_same_v<R, double>;
    std::vector<double> wsh, dsh;
    double* workl = reinterpret_cast<double*>(workl_in);
    double* d = reinterpret_cast<double*>(d_out);
    if constexpr (kShadow) {
        wsh.assign(workl_in, workl_in + (lworkl > 0 ? lworkl : 0));
        dsh.assign((size_t)(nev > 0 ? nev : 0) + 1, 0.0);
        workl = wsh.data();
        d = dsh.data();
    }
    struct Back {  // float family: results back into the caller's arrays
        std::vector<double>&wsh, &dsh;
        R *workl_in, *d_out;
        int nd;
        ~Back() {
            if constexpr (kShadow) {
                for (size_t t = 0; t < wsh.size(); ++t) workl_in[t] = (R)wsh[t];
                for (int t = 0; t < nd && t < (int)dsh.size(); ++t) d_out[t] = (R)dsh[t];
            }
        }
    } back{wsh, dsh, workl_in, d_out, iparam[4]};
    const int mode = iparam[6];
    const int nconv = iparam[4];
    if (nconv == 0) return 0;
    const Which which = la::parse_which(which_s);
    int ierr = 0;
    if (nconv <= 0) ierr = -14;
    if (n <= 0) ierr = -1;
    if (nev <= 0) ierr = -2;
    if (ncv <= nev || ncv > n) ierr = -3;
    if (which != Which::LM && which != Which::SM && which != Which::LA && which != Which::SA &&
        which != Which::BE)
        ierr = -5;
    if (bmat != 'I' && bmat != 'G') ierr = -6;
    if ((howmny != 'A' && howmny != 'P' && howmny != 'S') && rvec) ierr = -15;
    if (rvec && howmny == 'S') ierr = -16;
    if (rvec && lworkl < ncv * ncv + 8 * ncv) ierr = -7;
    enum { REGULR, SHIFTI, BUCKLE, CAYLEY } type = REGULR;
    if (mode == 1 || mode == 2) type = REGULR;
    else if (mode == 3) type = SHIFTI;
    else if (mode == 4) type = BUCKLE;
    else if (mode == 5) type = CAYLEY;
    else ierr = -10;
    if (mode == 1 && bmat == 'G') ierr = -11;
    if (nev == 1 && which == Which::BE) ierr = -12;
    if (ierr != 0) return ierr;

    // workl layout (SRC/dseupd.f:437-468), 0-based
    const int ih = ipntr[4] - 1, iritz = ipntr[5] - 1, ibounds = ipntr[6] - 1;
    const int ldh = ncv, ldq = ncv;
    const int ihd = ibounds + ldh, ihb = ihd + ldh, iq = ihb + ldh, iw = iq + ldh * ncv;
    const int next = iw + 2 * ncv;
    ipntr[3] = next + 1;
    ipntr[7] = ihd + 1;
    ipntr[8] = ihb + 1;
    ipntr[9] = iq + 1;
    const int irz = ipntr[10] - 1 + ncv, ibd = irz + ncv;
    const double eps23 = std::pow(Prec<R>::eps, 2.0 / 3.0);
    const double rnorm = workl[ih];

    // device context (V, resid, workd may be host or device memory)
    ArraysT<R> a;
    if (a.attach(n, ncv, resid, v, ldv, workd) != 0) return -9999;
    dev::Workspace ws;
    if (dev::ws_create(ws, n, ncv, a.stream) != hipSuccess) {
        a.release();
        return -9999;
    }
    struct Guard {
        ArraysT<R>& a;
        dev::Workspace& ws;
        ~Guard() {
            dev::ws_destroy(ws);
            a.release();
        }
    } guard{a, ws};
    if (a.host_mode) {
        a.ck(hipMemcpy2DAsync(a.d_v, sizeof(R) * a.d_ld, v, sizeof(R) * ldv,
                               sizeof(R) * n, ncv, hipMemcpyHostToDevice, a.stream));
        a.upload_resid();
        a.ck(hipMemcpyAsync(a.d_workd, workd, sizeof(R) * n, hipMemcpyHostToDevice, a.stream));
    }
    double bnorm2 = rnorm;
    if (bmat == 'G') {  // dnrm2(n, workd, 1); pdnorm2 over the ranks (pdseupd.f:456)
        dev::dots(ws, n, 0, a.d_v, a.d_ld, a.d_workd, a.d_workd, -1);
        if (dist && dist->comm) {
            dev::finalize(ws, 1, dev::kFinRaw, 0, 0, -1);
            if (comm_allreduce_sum(dist->comm, ws.sums, 1, a.stream) != 0) return -9999;
            dev::finalize(ws, 1, dev::kFinNorm, 0, 0, -1, true);
        } else {
            dev::finalize(ws, 1, dev::kFinNorm, 0, 0, -1);
        }
        a.ck(hipMemcpyAsync(ws.st_host, ws.st, sizeof(dev::LzState), hipMemcpyDeviceToHost, a.stream));
        a.sync();
        if (a.err.bad()) return -9999;
        bnorm2 = ws.st_host->rnorm;
    }

    std::vector<int> sel(ncv, 0);
    if (rvec) {
        bool reord = false;
        for (int j = 0; j < ncv; ++j) workl[ibounds + j] = j + 1;
        const int np = ncv - nev;
        la::dsgets(0, which, nev, np, workl + irz, workl + ibounds, workl);
        int numcnv = 0;
        for (int j = 1; j <= ncv; ++j) {
            const double temp1 = std::max(eps23, std::fabs(workl[irz + ncv - j]));
            const int jj = (int)workl[ibounds + ncv - j];
            if (numcnv < nconv && workl[ibd + jj - 1] <= tol * temp1) {
                sel[jj - 1] = 1;
                ++numcnv;
                if (jj > nconv) reord = true;
            }
        }
        if (numcnv != nconv) return -17;
        std::memcpy(workl + ihb, workl + ih + 1, sizeof(double) * (ncv - 1));
        std::memcpy(workl + ihd, workl + ih + ldh, sizeof(double) * ncv);
        if (la::steqr(ncv, workl + ihd, workl + ihb, workl + iq, ncv, ldq, workl + iw, false) != 0)
            return -8;
        if (reord) {  // move the selected Ritz pairs to the front (SRC/dseupd.f:587-617)
            int lp = 0, rp = ncv - 1;
            if (ncv > 1) {
                do {
                    if (sel[lp]) {
                        ++lp;
                    } else if (!sel[rp]) {
                        --rp;
                    } else {
                        std::swap(workl[ihd + lp], workl[ihd + rp]);
                        for (int i = 0; i < ncv; ++i)
                            std::swap(workl[iq + ncv * lp + i], workl[iq + ncv * rp + i]);
                        ++lp;
                        --rp;
                    }
                } while (lp < rp);
            }
        }
        std::memcpy(d, workl + ihd, sizeof(double) * nconv);
    } else {
        std::memcpy(d, workl + iritz, sizeof(double) * nconv);
        std::memcpy(workl + ihd, workl + iritz, sizeof(double) * ncv);
    }
    if (select) for (int j = 0; j < ncv; ++j) select[j] = sel[j];

    if (type == REGULR) {
        if (rvec) la::dsesrt(Which::LA, true, nconv, d, ncv, workl + iq, ldq);
        else std::memcpy(workl + ihb, workl + ibounds, sizeof(double) * ncv);
    } else {
        std::memcpy(workl + iw, workl + ihd, sizeof(double) * ncv);
        for (int k = 0; k < ncv; ++k) {
            double& t = workl[ihd + k];
            if (type == SHIFTI) t = 1.0 / t + sigma;
            else if (type == BUCKLE) t = sigma * t / (t - 1.0);
            else t = sigma * (t + 1.0) / (t - 1.0);
        }
        std::memcpy(d, workl + ihd, sizeof(double) * nconv);
        la::dsortr(Which::LA, true, nconv, workl + ihd, workl + iw);
        if (rvec) {
            la::dsesrt(Which::LA, true, nconv, d, ncv, workl + iq, ldq);
        } else {
            std::memcpy(workl + ihb, workl + ibounds, sizeof(double) * ncv);
            for (int k = 0; k < ncv; ++k) workl[ihb + k] *= bnorm2 / rnorm;
            la::dsortr(Which::LA, true, nconv, d, workl + ihb);
        }
    }

    const bool zdev = is_device_pointer(z);
    // a device Z the caller may still be writing on another stream (V / resid /
    // workd in device memory are ordered at attach): complete it first
    if (zdev && a.host_mode) a.ck(hipDeviceSynchronize());
    // M is the source of an asynchronous copy from pageable memory: it lives
    // until the a.sync() below (a run of 8 processes on one GPU read it freed)
    std::vector<double> M;
    if (rvec && howmny == 'A') {
        std::vector<double> work(ncv + 1);
        la::geqr2(ncv, nconv, workl + iq, ldq, workl + iw + ncv, work.data());
        // M = H_1 ... H_nconv * I(:, 1:nconv)  (ncv x nconv), then V <- V*M on device
        M.assign((size_t)ncv * nconv, 0.0);
        for (int j = 0; j < nconv; ++j) M[(size_t)j * ncv + j] = 1.0;
        la::orm2r('L', 'N', ncv, nconv, nconv, workl + iq, ldq, workl + iw + ncv, M.data(), ncv,
                  work.data());
        a.ck(hipMemcpyAsync(ws.q, M.data(), sizeof(double) * M.size(), hipMemcpyHostToDevice, a.stream));
        dev::vq_gemm(ws, n, a.d_v, a.d_ld, ncv, nconv, a.d_v, a.d_ld);
        // last row of Q for the Ritz estimates (SRC/dseupd.f:752-765)
        for (int j = 0; j < ncv - 1; ++j) workl[ihb + j] = 0.0;
        workl[ihb + ncv - 1] = 1.0;
        la::orm2r('L', 'T', ncv, 1, nconv, workl + iq, ldq, workl + iw + ncv, workl + ihb, ncv,
                  work.data());
        for (int j = 0; j < nconv; ++j) workl[iw + ncv + j] = workl[ihb + j];
    }
    if (type == REGULR && rvec) {
        for (int j = 0; j < ncv; ++j) workl[ihb + j] = rnorm * std::fabs(workl[ihb + j]);
    } else if (type != REGULR && rvec) {
        for (int k = 0; k < ncv; ++k) workl[ihb + k] *= bnorm2;
        for (int k = 0; k < ncv; ++k) {
            double& t = workl[ihb + k];
            const double wk = workl[iw + k];
            if (type == SHIFTI) t = std::fabs(t) / (wk * wk);
            else if (type == BUCKLE) t = sigma * std::fabs(t) / ((wk - 1.0) * (wk - 1.0));
            else t = std::fabs(t / wk * (wk - 1.0));
        }
    }
    if (rvec && (type == SHIFTI || type == CAYLEY)) {
        for (int k = 0; k < nconv; ++k) workl[iw + k] = workl[iw + ncv + k] / workl[iw + k];
    } else if (rvec && type == BUCKLE) {
        for (int k = 0; k < nconv; ++k) workl[iw + k] = workl[iw + ncv + k] / (workl[iw + k] - 1.0);
    }
    if (rvec && howmny == 'A') {
        // Z := V(:,1:nconv) (+ resid * w' purification for the transform modes)
        R* zd = nullptr;
        int64_t ldzd = a.d_ld;
        if (zdev) {
            zd = z;
            ldzd = ldz;
            a.ck(hipMemcpy2DAsync(zd, sizeof(R) * ldz, a.d_v, sizeof(R) * a.d_ld,
                                   sizeof(R) * n, nconv, hipMemcpyDeviceToDevice, a.stream));
        } else {
            if (hipMallocAsync(&zd, sizeof(R) * (size_t)a.d_ld * nconv, a.stream) != hipSuccess) {
                a.sync();  // (the pending copies read M)
                return -9999;
            }
            a.ck(hipMemcpyAsync(zd, a.d_v, sizeof(R) * (size_t)a.d_ld * nconv,
                                 hipMemcpyDeviceToDevice, a.stream));
        }
        if (type != REGULR) {
            a.ck(hipMemcpyAsync(ws.coef, workl + iw, sizeof(double) * nconv, hipMemcpyHostToDevice,
                                 a.stream));
            dev::ger_cols(a.stream, n, nconv, a.d_resid, ws.coef, zd, ldzd);
        }
        // V first, then Z: with Z = V (the reference's drivers pass v for z) the
        // purified Ritz vectors must be what V(:,1:nconv) holds on return
        if (a.host_mode)  // the reference leaves V * Q in V (dorm2r in place)
            a.ck(hipMemcpy2DAsync(v, sizeof(R) * ldv, a.d_v, sizeof(R) * a.d_ld,
                                   sizeof(R) * n, nconv, hipMemcpyDeviceToHost, a.stream));
        if (!zdev) {
            a.ck(hipMemcpy2DAsync(z, sizeof(R) * ldz, zd, sizeof(R) * a.d_ld,
                                   sizeof(R) * n, nconv, hipMemcpyDeviceToHost, a.stream));
            (void)hipFreeAsync(zd, a.stream);
        }
    }
    a.sync();  // a failed copy or a kernel fault of this call: -9999
    return a.err.bad() ? -9999 : 0;
}

}  // namespace ahip

const ahip::DistOp* ahip_dist_view(const arpack_hip_dist* D);

extern "C" {

// PARPACK's pdseupd_c (ICB/parpack.h:21): dseupd on this rank's rows; the
// only collective is the B-norm of B*resid for bmat = 'G' (pdseupd.f:456).
void arpack_hip_pdseupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, double* d, double* z, int ldz, double sigma,
                          char const* bmat, int n, char const* which, int nev, double tol,
                          double* resid, int ncv, double* v, int ldv, int* iparam, int* ipntr,
                          double* workd, double* workl, int lworkl, int* info) {
    (void)select;
    *info = ahip::sym_eupd(rvec != 0, howmny[0], nullptr, d, z, ldz, sigma, bmat[0], n, which, nev,
                           tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
                           ahip_dist_view(D));
}

void dseupd_c(int rvec, char const* howmny, int const* select, double* d, double* z, int ldz,
              double sigma, char const* bmat, int n, char const* which, int nev, double tol,
              double* resid, int ncv, double* v, int ldv, int* iparam, int* ipntr, double* workd,
              double* workl, int lworkl, int* info) {
    (void)select;  // intent(in) in the ICB (SRC/icbads.F90:46): a local copy is used
    *info = ahip::sym_eupd(rvec != 0, howmny[0], nullptr, d, z, ldz, sigma, bmat[0], n, which, nev,
                           tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl);
}

void dseupd_(int* rvec, char const* howmny, int* select, double* d, double* z, int* ldz,
             double* sigma, char const* bmat, int* n, char const* which, int* nev, double* tol,
             double* resid, int* ncv, double* v, int* ldv, int* iparam, int* ipntr, double* workd,
             double* workl, int* lworkl, int* info, size_t, size_t, size_t) {
    *info = ahip::sym_eupd(*rvec != 0, howmny[0], select, d, z, *ldz, *sigma, bmat[0], *n, which,
                           *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl);
}

// single-precision family (ICB/arpack.h:19; SRC/sseupd.f)
// pss: the fp32 family on a row distribution (ICB/parpack.h:17-18)
void arpack_hip_psseupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, float* d, float* z, int ldz, float sigma,
                          char const* bmat, int n, char const* which, int nev, float tol,
                          float* resid, int ncv, float* v, int ldv, int* iparam, int* ipntr,
                          float* workd, float* workl, int lworkl, int* info) {
    (void)select;
    *info = ahip::sym_eupd(rvec != 0, howmny[0], nullptr, d, z, ldz, sigma, bmat[0], n, which, nev,
                           tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
                           ahip_dist_view(D));
}
void sseupd_c(int rvec, char const* howmny, int const* select, float* d, float* z, int ldz,
              float sigma, char const* bmat, int n, char const* which, int nev, float tol,
              float* resid, int ncv, float* v, int ldv, int* iparam, int* ipntr, float* workd,
              float* workl, int lworkl, int* info) {
    (void)select;
    *info = ahip::sym_eupd(rvec != 0, howmny[0], nullptr, d, z, ldz, sigma, bmat[0], n, which, nev,
                           tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl);
}

void sseupd_(int* rvec, char const* howmny, int* select, float* d, float* z, int* ldz,
             float* sigma, char const* bmat, int* n, char const* which, int* nev, float* tol,
             float* resid, int* ncv, float* v, int* ldv, int* iparam, int* ipntr, float* workd,
             float* workl, int* lworkl, int* info, size_t, size_t, size_t) {
    *info = ahip::sym_eupd(*rvec != 0, howmny[0], select, d, z, *ldz, *sigma, bmat[0], *n, which,
                           *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl);
}

}  // extern "C"
