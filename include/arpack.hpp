/*
 * arpack.hpp -- the C++ binding of the reference (ICB/arpack.hpp): type-checked
 * overloads arpack::saupd / seupd / naupd / neupd over float, double,
 * std::complex<float> and std::complex<double>, with the option enums
 * arpack::which / bmat / howmny in place of the two-letter codes.
 *
 * Every overload forwards to the C entry point of arpack_hip.h with the
 * reference's argument meaning (SRC/icba*.F90), so C++ callers of arpack-ng
 * build unchanged against libarpack_hip.so. Complex arrays are passed as
 * std::complex<T>* (layout-identical to C99 T _Complex).
 */
#ifndef ARPACK_HIP_ICB_ARPACK_HPP
#define ARPACK_HIP_ICB_ARPACK_HPP

#include <complex>
#include <cstring>
#include <stdexcept>
#include <string>

#include "arpack_hip.h"

namespace arpack {

// enumerator order as ICB/arpack.hpp:10-48
enum class which : int {
    largest_algebraic,   // LA
    smallest_algebraic,  // SA
    largest_magnitude,   // LM
    smallest_magnitude,  // SM
    largest_real,        // LR
    smallest_real,       // SR
    largest_imaginary,   // LI
    smallest_imaginary,  // SI
    both_ends            // BE
};
enum class bmat : int { identity, generalized };
enum class howmny : int { ritz_vectors, schur_vectors, ritz_specified };

namespace detail {
inline char const* code(which w) {
    static char const* const c[] = {"LA", "SA", "LM", "SM", "LR", "SR", "LI", "SI", "BE"};
    return c[static_cast<int>(w)];
}
inline char const* code(bmat b) { return b == bmat::identity ? "I" : "G"; }
inline char const* code(howmny h) {
    static char const* const c[] = {"A", "P", "S"};
    return c[static_cast<int>(h)];
}
inline a_dcomplex* c99(std::complex<double>* p) { return reinterpret_cast<a_dcomplex*>(p); }
inline a_fcomplex* c99(std::complex<float>* p) { return reinterpret_cast<a_fcomplex*>(p); }
template <class C, class T>
inline C c99v(std::complex<T> z) {
    C r;
    std::memcpy(&r, &z, sizeof r);
    return r;
}
}  // namespace detail

// ---- symmetric (dsaupd / ssaupd, dseupd / sseupd) -------------------------------
inline void saupd(a_int& ido, bmat const b, a_int n, which const w, a_int nev, double tol,
                  double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  double* workd, double* workl, a_int lworkl, a_int& info) {
    dsaupd_c(&ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam,
             ipntr, workd, workl, lworkl, &info);
}
inline void saupd(a_int& ido, bmat const b, a_int n, which const w, a_int nev, float tol,
                  float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  float* workd, float* workl, a_int lworkl, a_int& info) {
    ssaupd_c(&ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam,
             ipntr, workd, workl, lworkl, &info);
}
inline void seupd(a_int rvec, howmny const h, a_int* select, double* d, double* z, a_int ldz,
                  double sigma, bmat const b, a_int n, which const w, a_int nev, double tol,
                  double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  double* workd, double* workl, a_int lworkl, a_int& info) {
    dseupd_c(rvec, detail::code(h), select, d, z, ldz, sigma, detail::code(b), n,
             detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             &info);
}
inline void seupd(a_int rvec, howmny const h, a_int* select, float* d, float* z, a_int ldz,
                  float sigma, bmat const b, a_int n, which const w, a_int nev, float tol,
                  float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  float* workd, float* workl, a_int lworkl, a_int& info) {
    sseupd_c(rvec, detail::code(h), select, d, z, ldz, sigma, detail::code(b), n,
             detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
             &info);
}

// ---- real nonsymmetric (dnaupd / snaupd, dneupd / sneupd) -----------------------
inline void naupd(a_int& ido, bmat const b, a_int n, which const w, a_int nev, double tol,
                  double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  double* workd, double* workl, a_int lworkl, a_int& info) {
    dnaupd_c(&ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam,
             ipntr, workd, workl, lworkl, &info);
}
inline void naupd(a_int& ido, bmat const b, a_int n, which const w, a_int nev, float tol,
                  float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  float* workd, float* workl, a_int lworkl, a_int& info) {
    snaupd_c(&ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam,
             ipntr, workd, workl, lworkl, &info);
}
inline void neupd(a_int rvec, howmny const h, a_int* select, double* dr, double* di, double* z,
                  a_int ldz, double sigmar, double sigmai, double* workev, bmat const b, a_int n,
                  which const w, a_int nev, double tol, double* resid, a_int ncv, double* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, double* workd, double* workl,
                  a_int lworkl, a_int& info) {
    dneupd_c(rvec, detail::code(h), select, dr, di, z, ldz, sigmar, sigmai, workev,
             detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr,
             workd, workl, lworkl, &info);
}
inline void neupd(a_int rvec, howmny const h, a_int* select, float* dr, float* di, float* z,
                  a_int ldz, float sigmar, float sigmai, float* workev, bmat const b, a_int n,
                  which const w, a_int nev, float tol, float* resid, a_int ncv, float* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, float* workd, float* workl,
                  a_int lworkl, a_int& info) {
    sneupd_c(rvec, detail::code(h), select, dr, di, z, ldz, sigmar, sigmai, workev,
             detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr,
             workd, workl, lworkl, &info);
}

// ---- complex (znaupd / cnaupd, zneupd / cneupd) ----------------------------------
inline void naupd(a_int& ido, bmat const b, a_int n, which const w, a_int nev, double tol,
                  std::complex<double>* resid, a_int ncv, std::complex<double>* v, a_int ldv,
                  a_int* iparam, a_int* ipntr, std::complex<double>* workd,
                  std::complex<double>* workl, a_int lworkl, double* rwork, a_int& info) {
    znaupd_c(&ido, detail::code(b), n, detail::code(w), nev, tol, detail::c99(resid), ncv,
             detail::c99(v), ldv, iparam, ipntr, detail::c99(workd), detail::c99(workl), lworkl,
             rwork, &info);
}
inline void naupd(a_int& ido, bmat const b, a_int n, which const w, a_int nev, float tol,
                  std::complex<float>* resid, a_int ncv, std::complex<float>* v, a_int ldv,
                  a_int* iparam, a_int* ipntr, std::complex<float>* workd,
                  std::complex<float>* workl, a_int lworkl, float* rwork, a_int& info) {
    cnaupd_c(&ido, detail::code(b), n, detail::code(w), nev, tol, detail::c99(resid), ncv,
             detail::c99(v), ldv, iparam, ipntr, detail::c99(workd), detail::c99(workl), lworkl,
             rwork, &info);
}
inline void neupd(a_int rvec, howmny const h, a_int* select, std::complex<double>* d,
                  std::complex<double>* z, a_int ldz, std::complex<double> sigma,
                  std::complex<double>* workev, bmat const b, a_int n, which const w, a_int nev,
                  double tol, std::complex<double>* resid, a_int ncv, std::complex<double>* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, std::complex<double>* workd,
                  std::complex<double>* workl, a_int lworkl, double* rwork, a_int& info) {
    zneupd_c(rvec, detail::code(h), select, detail::c99(d), detail::c99(z), ldz,
             detail::c99v<a_dcomplex>(sigma), detail::c99(workev), detail::code(b), n,
             detail::code(w), nev, tol, detail::c99(resid), ncv, detail::c99(v), ldv, iparam,
             ipntr, detail::c99(workd), detail::c99(workl), lworkl, rwork, &info);
}
inline void neupd(a_int rvec, howmny const h, a_int* select, std::complex<float>* d,
                  std::complex<float>* z, a_int ldz, std::complex<float> sigma,
                  std::complex<float>* workev, bmat const b, a_int n, which const w, a_int nev,
                  float tol, std::complex<float>* resid, a_int ncv, std::complex<float>* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, std::complex<float>* workd,
                  std::complex<float>* workl, a_int lworkl, float* rwork, a_int& info) {
    cneupd_c(rvec, detail::code(h), select, detail::c99(d), detail::c99(z), ldz,
             detail::c99v<a_fcomplex>(sigma), detail::c99(workev), detail::code(b), n,
             detail::code(w), nev, tol, detail::c99(resid), ncv, detail::c99(v), ldv, iparam,
             ipntr, detail::c99(workd), detail::c99(workl), lworkl, rwork, &info);
}

}  // namespace arpack

#endif
