// Device shift-invert operator of the complex engine: y = (A - sigma I)^{-1} x
// by BiCGStab on the complex CSR operator, every step on the GPU.
//
// This is the caller-side solve of znaupd's mode 3 (SRC/znaupd.f:27, OP =
// inv[A - sigma M] M with M = I), which the reference's example drivers do with
// a banded LU on the host (EXAMPLES/COMPLEX/zndrv2.f:179 zgttrf, :250 zgttrs).
// BASELINE config 5 (random complex CSR, n = 5e5, ~100 nnz a row, diag += 100)
// has no band structure, so the MI355X-native solve is Krylov: BiCGStab with
// the products on the XCD-split SpMV (zsplit.hip) and the vector updates, dot
// products and scalar recurrences in fused kernels whose scalars never leave
// the device (each kernel's blocks reduce the previous kernel's partials
// themselves, in one fixed order, so there is no finalize launch and no host
// round trip inside an iteration).  The host only enqueues iterations in
// chunks and reads a 64-byte state between chunks.
#pragma once
#include <hip/hip_runtime.h>

#include <complex>
#include <cstdint>

#include "zengine.hpp"

namespace ahip::zdev {

// device-resident BiCGStab state (one per solver)
struct BiState {
    int done;       // converged, broke down or hit maxit: later kernels return at once
    int breakdown;  // rhat^H v == 0 or rho == 0 before convergence
    int iters;      // iterations taken when done
    int pad;
    double rho[2][2];   // rho of iteration k at [k & 1] (complex re, im)
    double alpha[2];    // complex
    double omega[2];    // complex
    double bnorm2;      // ||b||^2
    double rnorm2;      // ||r||^2 of the last iteration
};

struct ZShift {
    const ZCsr* A = nullptr;
    std::complex<double> sigma;
    double rtol = 1e-12;
    int maxit = 200;
    int64_t n = 0;
    int nblk = 0;
    double *r = nullptr, *rh = nullptr, *p = nullptr, *v = nullptr, *s = nullptr, *t = nullptr,
           *w = nullptr;           // n complex each
    double* part = nullptr;        // 4 slots x nblk
    BiState* st = nullptr;         // device
    BiState* st_host = nullptr;    // pinned mirror
    int chunk = 4;                 // iterations enqueued before the first state read
    // statistics (host): solves, iterations, SpMVs, failures, worst final residual
    long long n_solves = 0, n_iters = 0, n_fail = 0;
    double max_relres = 0.0;
    double ms_total = 0.0;         // device time of the solves (hipEvents)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // method 1 (zshift_set_tridiag): a DIRECT solve of a tridiagonal A - sigma I
    // (zgttrf restated on the host, the triangular solves as device scans,
    // ztri.hip) -- what EXAMPLES/COMPLEX/zndrv2.f does with zgttrf / zgttrs
    int method = 0;
    double *tri_dl = nullptr, *tri_d = nullptr, *tri_du = nullptr, *tri_du2 = nullptr;  // complex
    int* tri_ipiv = nullptr;
    void* tri_bc = nullptr;        // block composites of the scans
    double* tri_cin = nullptr;     // the state entering each block (2 complex)
};

// 0, or a hipError_t on allocation failure (nothing leaks)
int zshift_create(ZShift& S, const ZCsr* A, std::complex<double> sigma, double rtol, int maxit);
void zshift_destroy(ZShift& S);
// y = (A - sigma I)^{-1} b on `stream` (device pointers, interleaved complex;
// y must not alias b).  Returns the iterations (>= 0) and *relres = ||r|| / ||b||
// of the recursively updated residual, -1 if BiCGStab broke down or did not
// reach rtol within maxit (y then holds the last iterate), -2 on a HIP error.
int zshift_apply(ZShift& S, hipStream_t stream, const double* b, double* y, double* relres);
// method 1: factor A - sigma I (A tridiagonal): 0; -1 not tridiagonal or
// singular; -2 HIP failure.  ztri_free releases the factors (method 0 again).
int zshift_tridiag_factor(ZShift& S);
void zshift_tridiag_free(ZShift& S);
// y = (A - sigma I)^{-1} b by the factors (b, y device, not aliased): 0 or -2
int zshift_tridiag_apply(ZShift& S, hipStream_t s, const double* b, double* y);
// z = x + 0i (x real, z interleaved complex); y = Re z (imag = 0) or Im z
void zpack_real(hipStream_t s, int64_t n, const double* x, double* z);
void zextract(hipStream_t s, int64_t n, const double* z, int imag, double* y);
// algorithmic HBM bytes of one BiCGStab iteration (two CSR products at 20 B a
// stored entry + rowptr + x/y vectors, and the fused vector passes)
double zshift_iter_bytes(const ZShift& S);

}  // namespace ahip::zdev
