// Host small-dense kit of the COMPLEX Arnoldi cycle (znaupd family): the
// ncv x ncv work the reference hands to LAPACK (zlahqr, ztrevc, ztrsen,
// zgeqr2, zunm2r, zlartg) and ARPACK's own helpers (zsortc, zngets, zneigh,
// the bulge chase of znapps).  Restated from the published LAPACK >= 3.10
// algorithms (zdense.cpp); compared with the image's LAPACK to rounding level
// in tests/test_kit_z.py.  Column-major, 0-based, `ld` = leading dimension.
#pragma once
#include <complex>
#include <cstdint>

#include "dense.hpp"

namespace ahip::zla {

using cd = std::complex<double>;
using la::Which;

inline double cabs1(cd z) { return std::fabs(z.real()) + std::fabs(z.imag()); }
double dznrm2(int n, const cd* x, int incx);
// LAPACK 3.10+ zlartg: c real, s and r complex
void lartg(cd f, cd g, double& c, cd& s, cd& r);
void larfg(int n, cd& alpha, cd* x, int incx, cd& tau);
// H = I - tau v v^H from the Left (C := H C) or the Right (C := C H)
void larf(char side, int m, int n, const cd* v, cd tau, cd* c, int ldc, cd* work);
void geqr2(int m, int n, cd* a, int lda, cd* tau, cd* work);
// zunm2r side='R', trans='N': C(m x n) := C * (H_1 ... H_k)
void unm2r_rn(int m, int n, int k, cd* a, int lda, const cd* tau, cd* c, int ldc, cd* work);
// zunm2r side='L', trans='N': C(m x n) := (H_1 ... H_k) * C
void unm2r_ln(int m, int n, int k, cd* a, int lda, const cd* tau, cd* c, int ldc, cd* work);
int lahqr(bool wantt, bool wantz, int n, int ilo, int ihi, cd* h, int ldh, cd* w, int iloz,
          int ihiz, cd* z, int ldz);
// ztrevc side='R'; howmny 'A' | 'B' | 'S'; work 2n; returns m
int trevc_right(char howmny, int* select, int n, cd* t, int ldt, cd* vr, int ldvr, cd* work);
// ztrsen(job='N', compq='V'); returns info, m
int trsen(const int* select, int n, cd* t, int ldt, cd* q, int ldq, cd* w, int& m);
double lanhs1(int n, const cd* a, int lda);

void zsortc(Which which, bool apply, int n, cd* x, cd* y);
void zngets(int ishift, Which which, int kev, int np, cd* ritz, cd* bounds);
// zneigh (SRC/zneigh.f): workl >= n*n + 2n
int zneigh(double rnorm, int n, const cd* h, int ldh, cd* ritz, cd* bounds, cd* q, int ldq,
           cd* workl);
// znapps bulge chase (SRC/znapps.f): H (ldh), Q (ldq x kplusp) on the host
void znapps_host(int kev, int np, const cd* shift, cd* h, int ldh, cd* q, int ldq, cd* workl,
                 int64_t nglob);

}  // namespace ahip::zla
