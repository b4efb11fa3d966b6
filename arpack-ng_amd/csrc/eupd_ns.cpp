// dneupd: Ritz values / Ritz (or Schur) vectors of the nonsymmetric Arnoldi
// factorization (SRC/dneupd.f:185-1071).  The ncv-sized work runs on the host
// in the caller's workl exactly as the reference lays it out (dngets
// re-selection, dlahqr Schur form, dtrsen reordering, dgeqr2 of the Schur
// vectors, dtrevc eigenvectors of T, Ritz estimates, spectral transform); the
// n-length products become two device GEMMs:
//   V <- V * Qh           (the reference's dorm2r on V, :734-736)
//   Z  = V(:,1:nconv) * Qx*R (its dorm2r + dtrmm on Z, :893-903)
// with Qh / Qx formed explicitly from the host Householder reflectors, plus the
// rank-1 purification Z += resid * w' in shift-invert mode (:1019-1059).
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../../include/arpack_hip.h"
#include "engine.hpp"

namespace ahip {

// R = float (sneupd): ncv-sized work in double on shadows of workl, dr, di and
// workev, rounded back into the caller's arrays on return.
template <class R>
static int ns_eupd(bool rvec, char howmny, int* select_out, R* dr_out, R* di_out, R* z, int ldz,
                   double sigmar, double sigmai, R* workev_out, char bmat, int n,
                   const char* which_s, int nev, double tol, R* resid, int ncv, R* v, int ldv,
                   int* iparam, int* ipntr, R* workd, R* workl_in, int lworkl) {
    using la::Which;
    constexpr bool kShadow = !std::is_same_v<R, double>;
    double* workl = reinterpret_cast<double*>(workl_in);
    double* dr = reinterpret_cast<double*>(dr_out);
    double* di = reinterpret_cast<double*>(di_out);
    double* workev = reinterpret_cast<double*>(workev_out);
    std::vector<double> sh[4];  // workl, dr, di, workev
    if constexpr (kShadow) {
        sh[0].assign(workl_in, workl_in + (lworkl > 0 ? lworkl : 0));
        sh[1].assign((size_t)(nev > 0 ? nev : 0) + 1, 0.0);
        sh[2].assign((size_t)(nev > 0 ? nev : 0) + 1, 0.0);
        sh[3].assign(3 * (size_t)(ncv > 0 ? ncv : 0), 0.0);
        workl = sh[0].data();
        dr = sh[1].data();
        di = sh[2].data();
        workev = sh[3].data();
    }
    struct Back {
        std::vector<double>* sh;
        R* out[4];
        ~Back() {
            if constexpr (kShadow)
                for (int k = 0; k < 4; ++k)
                    for (size_t t = 0; t < sh[k].size(); ++t) out[k][t] = (R)sh[k][t];
        }
    } back{sh, {workl_in, dr_out, di_out, workev_out}};
    const int mode = iparam[6];
    int nconv = iparam[4];
    const double eps23 = std::pow(Prec<R>::eps, 2.0 / 3.0);
    const Which which = la::parse_which(which_s);
    int ierr = 0;
    if (nconv <= 0) ierr = -14;
    else if (n <= 0) ierr = -1;
    else if (nev <= 0) ierr = -2;
    else if (ncv <= nev + 1 || ncv > n) ierr = -3;
    else if (which != Which::LM && which != Which::SM && which != Which::LR && which != Which::SR &&
             which != Which::LI && which != Which::SI)
        ierr = -5;
    else if (bmat != 'I' && bmat != 'G') ierr = -6;
    else if (lworkl < 3 * ncv * ncv + 6 * ncv) ierr = -7;
    else if ((howmny != 'A' && howmny != 'P' && howmny != 'S') && rvec) ierr = -13;
    else if (howmny == 'S') ierr = -12;
    enum { REGULR, SHIFTI, REALPT, IMAGPT } type = REGULR;
    if (mode == 1 || mode == 2) type = REGULR;
    else if (mode == 3 && sigmai == 0.0) type = SHIFTI;
    else if (mode == 3) type = REALPT;
    else if (mode == 4) type = IMAGPT;
    else ierr = -10;
    if (mode == 1 && bmat == 'G') ierr = -11;
    if (ierr != 0) return ierr;

    // workl layout (SRC/dneupd.f:508-535), 0-based
    const int ih = ipntr[4] - 1, iritzr = ipntr[5] - 1, iritzi = ipntr[6] - 1,
              ibounds = ipntr[7] - 1;
    const int ldh = ncv, ldq = ncv;
    const int iheigr = ibounds + ldh, iheigi = iheigr + ldh, ihbds = iheigi + ldh;
    const int iuptri = ihbds + ldh, invsub = iuptri + ldh * ncv;
    ipntr[8] = iheigr + 1;
    ipntr[9] = iheigi + 1;
    ipntr[10] = ihbds + 1;
    ipntr[11] = iuptri + 1;
    ipntr[12] = invsub + 1;
    const int irr = ipntr[13] - 1 + ncv * ncv, iri = irr + ncv, ibd = iri + ncv;
    const double rnorm = workl[ih + 2];
    workl[ih + 2] = 0.0;
    double* T = workl + iuptri;
    double* Qs = workl + invsub;

    std::vector<int> sel(ncv, 0);
    std::vector<double> Qh, M2;  // explicit Householder products for the device GEMMs
    if (rvec) {
        bool reord = false;
        for (int j = 0; j < ncv; ++j) workl[ibounds + j] = j + 1;
        int np = ncv - nev, kev = nev;
        la::dngets(0, which, kev, np, workl + irr, workl + iri, workl + ibounds);
        int numcnv = 0;
        for (int j = 1; j <= ncv; ++j) {
            const double temp1 = std::max(eps23, la::lapy2(workl[irr + ncv - j], workl[iri + ncv - j]));
            const int jj = (int)workl[ibounds + ncv - j];
            if (numcnv < nconv && workl[ibd + jj - 1] <= tol * temp1) {
                sel[jj - 1] = 1;
                ++numcnv;
                if (jj > nconv) reord = true;
            }
        }
        if (numcnv != nconv) return -15;
        // Schur form of H with Schur vectors (SRC/dneupd.f:622-636)
        std::memcpy(T, workl + ih, sizeof(double) * ldh * ncv);
        for (int j = 0; j < ncv; ++j)
            for (int i = 0; i < ncv; ++i) Qs[i + (size_t)j * ldq] = (i == j) ? 1.0 : 0.0;
        if (la::lahqr(true, true, ncv, 1, ncv, T, ldh, workl + iheigr, workl + iheigi, 1, ncv, Qs,
                      ldq) != 0)
            return -8;
        for (int j = 0; j < ncv; ++j) workl[ihbds + j] = Qs[(ncv - 1) + (size_t)j * ldq];
        if (reord) {  // wanted Ritz values to the leading block (SRC/dneupd.f:659-672)
            int nconv2 = 0;
            const int rc = la::trsen(sel.data(), ncv, T, ldh, Qs, ldq, workl + iheigr,
                                     workl + iheigi, nconv2, workl + ihbds);
            if (nconv2 < nconv) nconv = nconv2;
            if (rc == 1) return 1;
        }
        for (int j = 0; j < ncv; ++j) workl[ihbds + j] = Qs[(ncv - 1) + (size_t)j * ldq];
        if (type == REGULR) {
            std::memcpy(dr, workl + iheigr, sizeof(double) * nconv);
            std::memcpy(di, workl + iheigi, sizeof(double) * nconv);
        }
        // QR of the leading nconv Schur vectors; Qh = H_1 ... H_nconv (SRC/dneupd.f:718-736)
        std::vector<double> work(ncv + 1);
        la::geqr2(ncv, nconv, Qs, ldq, workev, workev + ncv);
        Qh.assign((size_t)ncv * ncv, 0.0);
        for (int j = 0; j < ncv; ++j) Qh[(size_t)j * ncv + j] = 1.0;
        la::orm2r('L', 'N', ncv, ncv, nconv, Qs, ldq, workev, Qh.data(), ncv, work.data());
        // make T consistent with the sign of R's diagonal (SRC/dneupd.f:748-755)
        for (int j = 0; j < nconv; ++j) {
            if (Qs[j + (size_t)j * ldq] < 0.0) {
                for (int c = 0; c < nconv; ++c) T[j + (size_t)c * ldq] = -T[j + (size_t)c * ldq];
                for (int r = 0; r < nconv; ++r) T[r + (size_t)j * ldq] = -T[r + (size_t)j * ldq];
            }
        }
        if (howmny == 'A') {
            // eigenvectors of the leading nconv block of T (SRC/dneupd.f:763-789)
            for (int j = 0; j < ncv; ++j) sel[j] = j < nconv;
            la::trevc_right('S', sel.data(), ncv, T, ldq, Qs, ldq, workev);
            int iconj = 0;
            for (int j = 0; j < nconv; ++j) {
                double* cj = Qs + (size_t)j * ldq;
                if (workl[iheigi + j] == 0.0) {
                    const double s = 1.0 / la::nrm2(ncv, cj, 1);
                    for (int r = 0; r < ncv; ++r) cj[r] *= s;
                } else if (iconj == 0) {
                    const double s = 1.0 / la::lapy2(la::nrm2(ncv, cj, 1), la::nrm2(ncv, cj + ldq, 1));
                    for (int r = 0; r < ncv; ++r) cj[r] *= s;
                    for (int r = 0; r < ncv; ++r) cj[ldq + r] *= s;
                    iconj = 1;
                } else {
                    iconj = 0;
                }
            }
            for (int j = 0; j < nconv; ++j) {  // dgemv('T', ncv, nconv, Qs, ihbds)
                double s = 0.0;
                for (int r = 0; r < ncv; ++r) s += Qs[r + (size_t)j * ldq] * workl[ihbds + r];
                workev[j] = s;
            }
            iconj = 0;
            for (int j = 0; j < nconv; ++j) {
                if (workl[iheigi + j] != 0.0) {
                    if (iconj == 0) {
                        workev[j] = la::lapy2(workev[j], workev[j + 1]);
                        workev[j + 1] = workev[j];
                        iconj = 1;
                    } else {
                        iconj = 0;
                    }
                }
            }
            std::memcpy(workl + ihbds, workev, sizeof(double) * nconv);
            // X = Qx R: Z <- Z*Qx*R (SRC/dneupd.f:881-903); the reflectors vanish
            // below row nconv, so only the leading nconv x nconv block acts
            la::geqr2(ncv, nconv, Qs, ldq, workev, workev + ncv);
            std::vector<double> Qx((size_t)ncv * ncv, 0.0);
            for (int j = 0; j < ncv; ++j) Qx[(size_t)j * ncv + j] = 1.0;
            la::orm2r('L', 'N', ncv, ncv, nconv, Qs, ldq, workev, Qx.data(), ncv, work.data());
            M2.assign((size_t)nconv * nconv, 0.0);  // (Qx R)(1:nconv, 1:nconv), ld nconv
            for (int c = 0; c < nconv; ++c)
                for (int r = 0; r < nconv; ++r) {
                    double s = 0.0;
                    for (int k = 0; k <= c; ++k) s += Qx[r + (size_t)k * ncv] * Qs[k + (size_t)c * ldq];
                    M2[r + (size_t)c * nconv] = s;
                }
        }
    } else {
        std::memcpy(dr, workl + iritzr, sizeof(double) * nconv);
        std::memcpy(di, workl + iritzi, sizeof(double) * nconv);
        std::memcpy(workl + iheigr, workl + iritzr, sizeof(double) * nconv);
        std::memcpy(workl + iheigi, workl + iritzi, sizeof(double) * nconv);
        std::memcpy(workl + ihbds, workl + ibounds, sizeof(double) * nconv);
    }
    if (select_out)
        for (int j = 0; j < ncv; ++j) select_out[j] = sel[j];

    // Ritz estimates and the spectral transformation (SRC/dneupd.f:919-990)
    if (type == REGULR) {
        if (rvec)
            for (int k = 0; k < ncv; ++k) workl[ihbds + k] *= rnorm;
    } else {
        if (type == SHIFTI) {
            if (rvec)
                for (int k = 0; k < ncv; ++k) workl[ihbds + k] *= rnorm;
            for (int k = 0; k < ncv; ++k) {
                const double temp = la::lapy2(workl[iheigr + k], workl[iheigi + k]);
                workl[ihbds + k] = std::fabs(workl[ihbds + k]) / temp / temp;
            }
            for (int k = 0; k < ncv; ++k) {
                const double temp = la::lapy2(workl[iheigr + k], workl[iheigi + k]);
                workl[iheigr + k] = workl[iheigr + k] / temp / temp + sigmar;
                workl[iheigi + k] = -workl[iheigi + k] / temp / temp + sigmai;
            }
        }
        std::memcpy(dr, workl + iheigr, sizeof(double) * nconv);
        std::memcpy(di, workl + iheigi, sizeof(double) * nconv);
    }
    if (!rvec) return 0;

    // purification coefficients (SRC/dneupd.f:1019-1056)
    std::vector<double> wpur;
    if (howmny == 'A' && type == SHIFTI) {
        wpur.assign(nconv, 0.0);
        int iconj = 0;
        for (int j = 0; j < nconv; ++j) {
            const double hr = workl[iheigr + j], hi = workl[iheigi + j];
            const double lastj = Qs[(ncv - 1) + (size_t)j * ldq];
            if (hi == 0.0 && hr != 0.0) {
                wpur[j] = lastj / hr;
            } else if (iconj == 0) {
                const double temp = la::lapy2(hr, hi);
                if (temp != 0.0) {
                    const double lastj1 = Qs[(ncv - 1) + (size_t)(j + 1) * ldq];
                    wpur[j] = (lastj * hr + lastj1 * hi) / temp / temp;
                    wpur[j + 1] = (lastj1 * hr - lastj * hi) / temp / temp;
                }
                iconj = 1;
            } else {
                iconj = 0;
            }
        }
        std::memcpy(workev, wpur.data(), sizeof(double) * nconv);
    }

    // ---- device part: V <- V*Qh, Z = V(:,1:nconv)*M2 (+ resid w')
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
    }
    a.ck(hipMemcpyAsync(ws.q, Qh.data(), sizeof(double) * Qh.size(), hipMemcpyHostToDevice, a.stream));
    dev::vq_gemm(ws, n, a.d_v, a.d_ld, ncv, ncv, a.d_v, a.d_ld);
    const bool zdev = is_device_pointer(z);
    // a device Z the caller may still be writing on another stream (V / resid /
    // workd in device memory are ordered at attach): complete it first
    if (zdev && a.host_mode) a.ck(hipDeviceSynchronize());
    R* zd = nullptr;
    int64_t ldzd = a.d_ld;
    if (zdev) {
        zd = z;
        ldzd = ldz;
    } else {
        if (hipMallocAsync(&zd, sizeof(R) * (size_t)a.d_ld * nconv, a.stream) != hipSuccess) {
            a.sync();  // (the pending copy reads Qh)
            return -9999;
        }
    }
    if (howmny == 'A') {
        a.sync();  // ws.q (Qh) consumed before it is overwritten
        a.ck(hipMemcpyAsync(ws.q, M2.data(), sizeof(double) * M2.size(), hipMemcpyHostToDevice,
                             a.stream));
        dev::vq_gemm(ws, n, a.d_v, a.d_ld, nconv, nconv, zd, ldzd);
        if (type == SHIFTI) {
            a.ck(hipMemcpyAsync(ws.coef, wpur.data(), sizeof(double) * nconv, hipMemcpyHostToDevice,
                                 a.stream));
            dev::ger_cols(a.stream, n, nconv, a.d_resid, ws.coef, zd, ldzd);
        }
    } else if (zd != a.d_v) {  // 'P': Z = the Schur vectors
        a.ck(hipMemcpy2DAsync(zd, sizeof(R) * ldzd, a.d_v, sizeof(R) * a.d_ld,
                               sizeof(R) * n, nconv, hipMemcpyDeviceToDevice, a.stream));
    }
    // V first, then Z: a caller may pass Z = V (the reference's drivers do),
    // and the reference then leaves the Ritz vectors in V(:,1:nconv)
    if (a.host_mode)  // the reference leaves V*Qh (the Schur basis) in V
        a.ck(hipMemcpy2DAsync(v, sizeof(R) * ldv, a.d_v, sizeof(R) * a.d_ld,
                               sizeof(R) * n, ncv, hipMemcpyDeviceToHost, a.stream));
    if (!zdev) {
        a.ck(hipMemcpy2DAsync(z, sizeof(R) * ldz, zd, sizeof(R) * a.d_ld,
                               sizeof(R) * n, nconv, hipMemcpyDeviceToHost, a.stream));
        (void)hipFreeAsync(zd, a.stream);
    }
    a.sync();  // a failed copy or a kernel fault of this call: -9999
    return a.err.bad() ? -9999 : 0;
}

}  // namespace ahip

extern "C" {

// PARPACK's pdneupd_c (ICB/parpack.h:27): pdneupd communicates nothing beyond
// its debug output (PARPACK/SRC/MPI/pdneupd.f), so it is dneupd on this rank's rows.
void arpack_hip_pdneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, double* dr, double* di, double* z, int ldz,
                          double sigmar, double sigmai, double* workev, char const* bmat, int n,
                          char const* which, int nev, double tol, double* resid, int ncv,
                          double* v, int ldv, int* iparam, int* ipntr, double* workd,
                          double* workl, int lworkl, int* info) {
    (void)D;
    (void)select;
    *info = ahip::ns_eupd(rvec != 0, howmny[0], nullptr, dr, di, z, ldz, sigmar, sigmai, workev,
                          bmat[0], n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                          workl, lworkl);
}

void dneupd_c(int rvec, char const* howmny, int const* select, double* dr, double* di, double* z,
              int ldz, double sigmar, double sigmai, double* workev, char const* bmat, int n,
              char const* which, int nev, double tol, double* resid, int ncv, double* v, int ldv,
              int* iparam, int* ipntr, double* workd, double* workl, int lworkl, int* info) {
    (void)select;  // intent(in) in the ICB (SRC/icbadn.F90): a local copy is used
    *info = ahip::ns_eupd(rvec != 0, howmny[0], nullptr, dr, di, z, ldz, sigmar, sigmai, workev,
                          bmat[0], n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                          workl, lworkl);
}

void dneupd_(int* rvec, char const* howmny, int* select, double* dr, double* di, double* z,
             int* ldz, double* sigmar, double* sigmai, double* workev, char const* bmat, int* n,
             char const* which, int* nev, double* tol, double* resid, int* ncv, double* v,
             int* ldv, int* iparam, int* ipntr, double* workd, double* workl, int* lworkl,
             int* info, size_t, size_t, size_t) {
    *info = ahip::ns_eupd(*rvec != 0, howmny[0], select, dr, di, z, *ldz, *sigmar, *sigmai, workev,
                          bmat[0], *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr,
                          workd, workl, *lworkl);
}

// single-precision family (ICB/arpack.h:17; SRC/sneupd.f)
// psn (ICB/parpack.h:23-24): as pdneupd, no collective
void arpack_hip_psneupd_c(const arpack_hip_dist* D, int rvec, char const* howmny,
                          int const* select, float* dr, float* di, float* z, int ldz,
                          float sigmar, float sigmai, float* workev, char const* bmat, int n,
                          char const* which, int nev, float tol, float* resid, int ncv, float* v,
                          int ldv, int* iparam, int* ipntr, float* workd, float* workl,
                          int lworkl, int* info) {
    (void)D;
    (void)select;
    *info = ahip::ns_eupd(rvec != 0, howmny[0], nullptr, dr, di, z, ldz, sigmar, sigmai, workev,
                          bmat[0], n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                          workl, lworkl);
}
void sneupd_c(int rvec, char const* howmny, int const* select, float* dr, float* di, float* z,
              int ldz, float sigmar, float sigmai, float* workev, char const* bmat, int n,
              char const* which, int nev, float tol, float* resid, int ncv, float* v, int ldv,
              int* iparam, int* ipntr, float* workd, float* workl, int lworkl, int* info) {
    (void)select;
    *info = ahip::ns_eupd(rvec != 0, howmny[0], nullptr, dr, di, z, ldz, sigmar, sigmai, workev,
                          bmat[0], n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                          workl, lworkl);
}

void sneupd_(int* rvec, char const* howmny, int* select, float* dr, float* di, float* z, int* ldz,
             float* sigmar, float* sigmai, float* workev, char const* bmat, int* n,
             char const* which, int* nev, float* tol, float* resid, int* ncv, float* v, int* ldv,
             int* iparam, int* ipntr, float* workd, float* workl, int* lworkl, int* info, size_t,
             size_t, size_t) {
    *info = ahip::ns_eupd(*rvec != 0, howmny[0], select, dr, di, z, *ldz, *sigmar, *sigmai, workev,
                          bmat[0], *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr,
                          workd, workl, *lworkl);
}

}  // extern "C"
