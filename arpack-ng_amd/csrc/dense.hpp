// Host small-dense kit: the ncv-sized pieces of the IRL/IRA cycle.
//
// Everything here operates on O(ncv) / O(ncv^2) data that lives in the
// caller's `workl` (host memory), exactly like the reference, where these
// steps cost ~0% of the time (SURVEY.md §1 L1 "host small-dense").  They are
// restated from the published LAPACK algorithms (LAPACK >= 3.10 variants,
// which is what the image's OpenBLAS carries) and from ARPACK's own helpers;
// the shell-sort tie order is cloned exactly because it decides which Ritz
// values become shifts.
//
// Column-major storage, 0-based indices, `ld` = leading dimension.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>

namespace ahip::la {

// dlamch('E') / dlamch('S') as LAPACK >= 3.x computes them for IEEE double:
// eps = epsilon/2 (rounding mode), sfmin = tiny.
constexpr double kEps = DBL_EPSILON * 0.5;
constexpr double kSafmin = DBL_MIN;

double lapy2(double x, double y);
// LAPACK 3.10+ dlartg (la_xlartg): c >= 0, r carries the sign of f.
void lartg(double f, double g, double& c, double& s, double& r);
void lae2(double a, double b, double c, double& rt1, double& rt2);
void laev2(double a, double b, double c, double& rt1, double& rt2, double& cs1,
           double& sn1);
// dlascl('G') on a contiguous vector: x *= cto/cfrom without over/underflow.
void lascl(double cfrom, double cto, int n, double* x);
// The multipliers dlascl applies (at most 4 are ever needed for doubles).
int lascl_factors(double cfrom, double cto, double mul[4]);

// Implicit QL/QR on a symmetric tridiagonal (d[n], e[n-1]).
//  - dstqrb mode (SRC/dstqrb.f): z is ONE row (the last row of the eigenvector
//    matrix), zrows=1, ldz=1, norm 'I';
//  - dsteqr('I') mode (LAPACK): z is n x n, zrows=n, norm 'M'.
// Returns info (0 = ok, >0 = number of unconverged off-diagonals).
int steqr(int n, double* d, double* e, double* z, int zrows, int ldz, double* work,
          bool one_norm_inf);
inline int stqrb(int n, double* d, double* e, double* z, double* work) {
    return steqr(n, d, e, z, 1, 1, work, true);
}

// Householder kit (dseupd / dneupd post-processing).
double nrm2(int n, const double* x, int incx);
void larfg(int n, double& alpha, double* x, int incx, double& tau);
// H = I - tau v v^T applied from the Left (side='L') or Right (side='R') to C(m,n).
void larf(char side, int m, int n, const double* v, int incv, double tau, double* c,
          int ldc, double* work);
void geqr2(int m, int n, double* a, int lda, double* tau, double* work);
// dorm2r for side in {'L','R'}, trans in {'N','T'}.
void orm2r(char side, char trans, int m, int n, int k, double* a, int lda,
           const double* tau, double* c, int ldc, double* work);

// ---------------- ARPACK symmetric helpers (SRC/ds*.f) -----------------------
enum class Which : int { LM = 0, SM, LA, SA, BE, LR, SR, LI, SI, BAD };
Which parse_which(const char* w);

// dsortr (SRC/dsortr.f:59-218): shell sort of x1 by `which`, permuting x2.
void dsortr(Which which, bool apply, int n, double* x1, double* x2);
// dsesrt (SRC/dsesrt.f): shell sort of x, permuting columns of a(na, n).
void dsesrt(Which which, bool apply, int n, double* x, int na, double* a, int lda);
// dsgets (SRC/dsgets.f:93-219)
void dsgets(int ishift, Which which, int kev, int np, double* ritz, double* bounds,
            double* shifts);
// dsconv (SRC/dsconv.f:59-138)
int dsconv(int n, const double* ritz, const double* bounds, double tol, double eps = kEps);
// dseigt (SRC/dseigt.f:87-181): h(ldh,2), returns ierr
int dseigt(double rnorm, int n, const double* h, int ldh, double* eig, double* bounds,
           double* workl);

// Implicit-shift bulge chase of dsapps (SRC/dsapps.f:240-442) on the host:
// updates h(ldh,2) in place and accumulates Q (ldq x kplusp).  The n-length
// V*Q / residual update is done on the device by the caller.
void dsapps_host(int kev, int np, const double* shift, double* h, int ldh, double* q,
                 int ldq);

// ---------------- nonsymmetric kit (dense_ns.cpp) ----------------------------
void lanv2(double& a, double& b, double& c, double& d, double& rt1r, double& rt1i, double& rt2r,
           double& rt2i, double& cs, double& sn);
double lanhs1(int n, const double* a, int lda);
// dlahqr with 1-based ilo/ihi/iloz/ihiz; returns info
int lahqr(bool wantt, bool wantz, int n, int ilo, int ihi, double* h, int ldh, double* wr,
          double* wi, int iloz, int ihiz, double* z, int ldz);
void ladiv(double a, double b, double c, double d, double& p, double& q);
int laln2(int na, int nw, double smin, double ca, const double* a, int lda, double d1, double d2,
          const double* b, int ldb, double wr, double wi, double* x, int ldx, double& scale,
          double& xnorm);
// dtrevc side='R'; howmny 'A' | 'B' | 'S'; work 3n; returns m
int trevc_right(char howmny, int* select, int n, const double* t, int ldt, double* vr, int ldvr,
                double* work);
void dsortc(Which which, bool apply, int n, double* xr, double* xi, double* y);
void dngets(int ishift, Which which, int& kev, int& np, double* ritzr, double* ritzi,
            double* bounds);
int dnconv(int n, const double* ritzr, const double* ritzi, const double* bounds, double tol,
           double eps = kEps);
int dneigh(double rnorm, int n, const double* h, int ldh, double* ritzr, double* ritzi,
           double* bounds, double* q, int ldq, double* workl);
int dnapps_host(int kev, int np, const double* shiftr, const double* shifti, double* h, int ldh,
                double* q, int ldq, double* workl, int64_t nglob);
// Schur reordering for dneupd: dlasy2, dlaexc, dtrexc, dtrsen(job='N', compq='V')
int lasy2(int isgn, int n1, int n2, const double* tl, int ldtl, const double* tr, int ldtr,
          const double* b, int ldb, double& scale, double* x, int ldx, double& xnorm);
int laexc(bool wantq, int n, double* t, int ldt, double* q, int ldq, int j1, int n1, int n2,
          double* work);
int trexc(bool wantq, int n, double* t, int ldt, double* q, int ldq, int& ifst, int& ilst,
          double* work);
int trsen(const int* select, int n, double* t, int ldt, double* q, int ldq, double* wr,
          double* wi, int& m, double* work);

}  // namespace ahip::la
