// Device shift-invert operator of the symmetric engine: y = (A - sigma I)^{-1} x
// by conjugate gradients (positive-definite A - sigma I) or MINRES (any
// symmetric A - sigma I: sigma inside the spectrum, interior eigenvalues) on the
// real CSR operator, every step on the GPU.
//
// The caller-side solve of dsaupd's mode 3 (SRC/dsaupd.f:30-48, OP = inv[A -
// sigma M] M with M = I), which the reference's drivers do with a banded LU on
// the host (EXAMPLES/SYM/dsdrv2.f: dgttrf / dgttrs).  For a symmetric operator
// with sigma below its spectrum (the usual "smallest eigenvalues" use, e.g.
// dsdrv2's sigma = 0 on a Laplacian) A - sigma I is positive definite and CG is
// the Krylov solve of choice: one SpMV a step (the engine's own, full or
// symmetric storage) and three fused vector kernels whose scalars never leave
// the device -- each reducing kernel's blocks sum the previous kernel's
// partials themselves in one fixed order (as the complex BiCGStab,
// zsolve.hip).  An indefinite A - sigma I can break CG down: the solve then
// reports failure (a non-positive curvature p'(A - sigma I)p, or no
// convergence within maxit) and the Lanczos run stops with info = -9999;
// MINRES (method kDShiftMinres) serves indefinite shifts, one more vector pass
// an iteration.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device.hpp"

namespace ahip::dev {

// MINRES recurrence scalars at the start of an iteration (Paige & Saunders)
struct MrRec {
    double beta, oldb, cs, sn, dbar, epsln, phibar;
};

// device-resident solver state (CG, or MINRES: rec double-buffered by
// iteration parity, so a kernel's blocks read one copy while block 0 writes the other)
struct CgState {
    int done;       // converged, broke down or hit maxit: later kernels return at once
    int breakdown;  // CG: p'(A - sigma I)p <= 0 (not positive definite); MINRES: gamma = 0
    int iters;      // iterations taken when done
    int failed;     // done without reaching rtol
    double rho[2];  // CG: r'r of iteration k at [k & 1]
    double alpha;   // CG: alpha; MINRES: alfa = v'(A - sigma I)v of the iteration
    double bnorm2;  // ||b||^2
    double rnorm2;  // ||r||^2 of the last iteration (MINRES: phibar^2, its estimate)
    double beta1;   // MINRES: ||b||
    MrRec rec[2];
    double omega;   // BiCGStab
};

// CG: A - sigma I symmetric positive definite; MINRES: symmetric; BiCGStab:
// general (dnaupd's real shift-invert)
// Tridiag: a direct solve (dgttrf on the host once, the triangular solves as
// device scans, dtri.hip) for a tridiagonal A - sigma I -- the operators a
// Krylov solve cannot serve (dndrv2's non-normal convection-diffusion)
enum DShiftMethod { kDShiftCg = 0, kDShiftMinres = 1, kDShiftBicgstab = 2, kDShiftTridiag = 3 };

struct DShift {
    const Csr* A = nullptr;
    double sigma = 0.0;
    double rtol = 1e-12;
    int maxit = 1000;
    int method = kDShiftCg;
    int64_t n = 0;
    int nblk = 0;
    double* vec[7] = {};  // n each -- CG: r, p, w; MINRES: v, r1, r2, y, w, w2;
                          // BiCGStab: r, rh, p, v, s, t, w
    double* part = nullptr;                           // 2 regions x 2 slots x nblk
    CgState* st = nullptr;                            // device
    CgState* st_host = nullptr;                       // pinned mirror
    int chunk = 8;  // iterations enqueued before the first state read
    long long n_solves = 0, n_iters = 0, n_fail = 0;
    double max_relres = 0.0;
    double ms_total = 0.0;  // device time of the solves (hipEvents)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // kDShiftTridiag: the LU factors (dgttrf layout, 0-based pivots) and the
    // scans' block composites / carries
    double *tri_dl = nullptr, *tri_d = nullptr, *tri_du = nullptr, *tri_du2 = nullptr;
    int* tri_ipiv = nullptr;
    void* tri_bc = nullptr;
    double* tri_cin = nullptr;
};

// 0, or a hipError_t on allocation failure (nothing leaks)
int dshift_create(DShift& S, const Csr* A, double sigma, double rtol, int maxit);
void dshift_destroy(DShift& S);
// y = (A - sigma I)^{-1} b on `stream` (device pointers; y must not alias b).
// Returns the iterations (>= 0) and *relres = ||r|| / ||b|| of the recursively
// updated residual; -1 if CG broke down or did not reach rtol within maxit (y
// then holds the last iterate), -2 on a HIP error.
int dshift_apply(DShift& S, hipStream_t stream, const double* b, double* y, double* relres);
// algorithmic HBM bytes of one iteration (the CSR product in its storage and
// the fused vector passes of the method; Tridiag: one direct solve)
double dshift_iter_bytes(const DShift& S);
// kDShiftTridiag (dtri.hip): factor A - sigma I (0; -1 not tridiagonal or
// singular; -2 HIP failure), free the factors, one solve (0 or -2)
int dshift_tridiag_factor(DShift& S);
void dshift_tridiag_free(DShift& S);
int dshift_tridiag_apply(DShift& S, hipStream_t s, const double* b, double* y);

}  // namespace ahip::dev
