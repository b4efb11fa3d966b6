// Device operator pair of dsaupd's generalized modes (bmat = 'G', modes 2-5):
// B*x and OP*x served on the GPU, the inverse by the device Krylov solve of
// dshift.hip on C = A - sigma M (dgen.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dshift.hpp"

struct arpack_hip_csr;
struct arpack_hip_zcsr;

namespace ahip::zdev {
struct ZShift;
}

namespace ahip::dev {

struct DGen {
    const Csr* A = nullptr;   // A (mode 4: K)
    const Csr* B = nullptr;   // M (mode 4: KG)
    arpack_hip_csr* C = nullptr;  // owned: A - sigma M (modes 3-5)
    int mode = 0;
    double sigma = 0.0;
    int64_t n = 0;
    DShift S;                 // the solve on C (mode 2: on M)
    double* t = nullptr;      // 2n device scratch: the right-hand side and M x
    // dnaupd's complex shifts (SRC/dnaupd.f:28-33, EXAMPLES/NONSYM/dndrv5-6.f):
    // OP = Re (mode 3) or Im (mode 4) of inv[A - sigma M] M with a complex
    // sigma, the solve complex -- C = A - sigma M as a complex CSR, BiCGStab or
    // the direct tridiagonal solve of zsolve.hip / ztri.hip
    bool cshift = false;
    int part = 0;                  // 0: real part, 1: imaginary part
    arpack_hip_zcsr* ZC = nullptr; // owned
    zdev::ZShift* ZS = nullptr;    // owned (dgen.cpp)
    double* zb = nullptr;          // 2 x 2n device scratch: complex rhs and solution
};

// 0; -1 bad arguments (sizes differ, mode not 2..5); -2 HIP / allocation failure
int dgen_create(DGen& G, const arpack_hip_csr* A, const arpack_hip_csr* B, int mode, double sigma,
                double rtol, int maxit, int method);
// complex-shift pair (dnaupd modes 3 / 4): 0; -1 bad arguments (sizes, mode
// not 3 or 4, sigmai == 0, method not 0 BiCGStab / 1 tridiagonal, C not
// tridiagonal for method 1); -2 HIP / allocation failure
int dgen_create_cshift(DGen& G, const arpack_hip_csr* A, const arpack_hip_csr* B, int mode,
                       double sigmar, double sigmai, double rtol, int maxit, int method);
void dgen_destroy(DGen& G);
// one request: 0 done; -1 the solve missed its tolerance or broke down; -2 HIP error
int dgen_apply(DGen& G, hipStream_t s, int ido, const double* x, double* y, const double* bx,
               double* xw);

}  // namespace ahip::dev
