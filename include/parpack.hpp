/*
 * parpack.hpp -- the C++ binding of PARPACK (reference: ICB/parpack.hpp): the
 * arpack::saupd / seupd / naupd / neupd overloads of arpack.hpp with the MPI
 * communicator (Fortran handle, MPI_Comm_c2f) as first argument, forwarding to
 * the C entry points of parpack.h (libparpack_hip.so) with the reference's
 * argument meaning; n is the number of rows this process owns.
 */
#ifndef ARPACK_HIP_ICB_PARPACK_HPP
#define ARPACK_HIP_ICB_PARPACK_HPP

#include "arpack.hpp"
#include "parpack.h"

namespace arpack {

// ---- symmetric (p[sd]saupd / p[sd]seupd) ----------------------------------------
inline void saupd(MPI_Fint comm, a_int& ido, bmat const b, a_int n, which const w, a_int nev,
                  double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
                  a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int& info) {
    pdsaupd_c(comm, &ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv,
              iparam, ipntr, workd, workl, lworkl, &info);
}
inline void saupd(MPI_Fint comm, a_int& ido, bmat const b, a_int n, which const w, a_int nev,
                  float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
                  a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int& info) {
    pssaupd_c(comm, &ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv,
              iparam, ipntr, workd, workl, lworkl, &info);
}
inline void seupd(MPI_Fint comm, a_int rvec, howmny const h, a_int* select, double* d, double* z,
                  a_int ldz, double sigma, bmat const b, a_int n, which const w, a_int nev,
                  double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
                  a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int& info) {
    pdseupd_c(comm, rvec, detail::code(h), select, d, z, ldz, sigma, detail::code(b), n,
              detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
              &info);
}
inline void seupd(MPI_Fint comm, a_int rvec, howmny const h, a_int* select, float* d, float* z,
                  a_int ldz, float sigma, bmat const b, a_int n, which const w, a_int nev,
                  float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
                  a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int& info) {
    psseupd_c(comm, rvec, detail::code(h), select, d, z, ldz, sigma, detail::code(b), n,
              detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
              &info);
}

// ---- real nonsymmetric (p[sd]naupd / p[sd]neupd) --------------------------------
inline void naupd(MPI_Fint comm, a_int& ido, bmat const b, a_int n, which const w, a_int nev,
                  double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
                  a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int& info) {
    pdnaupd_c(comm, &ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv,
              iparam, ipntr, workd, workl, lworkl, &info);
}
inline void naupd(MPI_Fint comm, a_int& ido, bmat const b, a_int n, which const w, a_int nev,
                  float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
                  a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int& info) {
    psnaupd_c(comm, &ido, detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv,
              iparam, ipntr, workd, workl, lworkl, &info);
}
inline void neupd(MPI_Fint comm, a_int rvec, howmny const h, a_int* select, double* dr,
                  double* di, double* z, a_int ldz, double sigmar, double sigmai, double* workev,
                  bmat const b, a_int n, which const w, a_int nev, double tol, double* resid,
                  a_int ncv, double* v, a_int ldv, a_int* iparam, a_int* ipntr, double* workd,
                  double* workl, a_int lworkl, a_int& info) {
    pdneupd_c(comm, rvec, detail::code(h), select, dr, di, z, ldz, sigmar, sigmai, workev,
              detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr,
              workd, workl, lworkl, &info);
}
inline void neupd(MPI_Fint comm, a_int rvec, howmny const h, a_int* select, float* dr, float* di,
                  float* z, a_int ldz, float sigmar, float sigmai, float* workev, bmat const b,
                  a_int n, which const w, a_int nev, float tol, float* resid, a_int ncv, float* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, float* workd, float* workl,
                  a_int lworkl, a_int& info) {
    psneupd_c(comm, rvec, detail::code(h), select, dr, di, z, ldz, sigmar, sigmai, workev,
              detail::code(b), n, detail::code(w), nev, tol, resid, ncv, v, ldv, iparam, ipntr,
              workd, workl, lworkl, &info);
}

// ---- complex (p[cz]naupd / p[cz]neupd) ------------------------------------------
inline void naupd(MPI_Fint comm, a_int& ido, bmat const b, a_int n, which const w, a_int nev,
                  double tol, std::complex<double>* resid, a_int ncv, std::complex<double>* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, std::complex<double>* workd,
                  std::complex<double>* workl, a_int lworkl, double* rwork, a_int& info) {
    pznaupd_c(comm, &ido, detail::code(b), n, detail::code(w), nev, tol, detail::c99(resid), ncv,
              detail::c99(v), ldv, iparam, ipntr, detail::c99(workd), detail::c99(workl), lworkl,
              rwork, &info);
}
inline void naupd(MPI_Fint comm, a_int& ido, bmat const b, a_int n, which const w, a_int nev,
                  float tol, std::complex<float>* resid, a_int ncv, std::complex<float>* v,
                  a_int ldv, a_int* iparam, a_int* ipntr, std::complex<float>* workd,
                  std::complex<float>* workl, a_int lworkl, float* rwork, a_int& info) {
    pcnaupd_c(comm, &ido, detail::code(b), n, detail::code(w), nev, tol, detail::c99(resid), ncv,
              detail::c99(v), ldv, iparam, ipntr, detail::c99(workd), detail::c99(workl), lworkl,
              rwork, &info);
}
inline void neupd(MPI_Fint comm, a_int rvec, howmny const h, a_int* select,
                  std::complex<double>* d, std::complex<double>* z, a_int ldz,
                  std::complex<double> sigma, std::complex<double>* workev, bmat const b, a_int n,
                  which const w, a_int nev, double tol, std::complex<double>* resid, a_int ncv,
                  std::complex<double>* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  std::complex<double>* workd, std::complex<double>* workl, a_int lworkl,
                  double* rwork, a_int& info) {
    pzneupd_c(comm, rvec, detail::code(h), select, detail::c99(d), detail::c99(z), ldz,
              detail::c99v<a_dcomplex>(sigma), detail::c99(workev), detail::code(b), n,
              detail::code(w), nev, tol, detail::c99(resid), ncv, detail::c99(v), ldv, iparam,
              ipntr, detail::c99(workd), detail::c99(workl), lworkl, rwork, &info);
}
inline void neupd(MPI_Fint comm, a_int rvec, howmny const h, a_int* select,
                  std::complex<float>* d, std::complex<float>* z, a_int ldz,
                  std::complex<float> sigma, std::complex<float>* workev, bmat const b, a_int n,
                  which const w, a_int nev, float tol, std::complex<float>* resid, a_int ncv,
                  std::complex<float>* v, a_int ldv, a_int* iparam, a_int* ipntr,
                  std::complex<float>* workd, std::complex<float>* workl, a_int lworkl,
                  float* rwork, a_int& info) {
    pcneupd_c(comm, rvec, detail::code(h), select, detail::c99(d), detail::c99(z), ldz,
              detail::c99v<a_fcomplex>(sigma), detail::c99(workev), detail::code(b), n,
              detail::code(w), nev, tol, detail::c99(resid), ncv, detail::c99(v), ldv, iparam,
              ipntr, detail::c99(workd), detail::c99(workl), lworkl, rwork, &info);
}

}  // namespace arpack

#endif
