// Device operator pair of znaupd's generalized modes (bmat = 'G', modes 2-3):
// B*x and OP*x served on the GPU, the inverse by the device BiCGStab of
// zsolve.hip on C = A - sigma M (M itself in mode 2), formed once (zgen.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <complex>
#include <cstdint>

#include "zsolve.hpp"

struct arpack_hip_zcsr;

namespace ahip::zdev {

struct ZGen {
    const ZCsr* A = nullptr;
    const ZCsr* M = nullptr;
    arpack_hip_zcsr* C = nullptr;  // owned: A - sigma M (mode 3)
    int mode = 0;
    std::complex<double> sigma;
    int64_t n = 0;
    ZShift S;               // BiCGStab on C (mode 2: on M)
    double* t = nullptr;    // n complex device scratch: the right-hand side
};

// 0; -1 bad arguments (sizes differ, mode not 2..3); -2 HIP / allocation failure
int zgen_create(ZGen& G, const arpack_hip_zcsr* A, const arpack_hip_zcsr* M, int mode,
                std::complex<double> sigma, double rtol, int maxit);
void zgen_destroy(ZGen& G);
// One request (ido = -1, 1 or 2) on interleaved-complex device vectors x, y;
// bx: B x the engine already formed (ido = 1 in mode 3), else nullptr.
// 0 done; -1 the solve missed its tolerance or broke down; -2 HIP error.
int zgen_apply(ZGen& G, hipStream_t s, int ido, const double* x, double* y, const double* bx);

}  // namespace ahip::zdev

// the engine view of a C-ABI complex operator (zsolver.cpp)
const ahip::zdev::ZCsr* ahip_zcsr_view(const arpack_hip_zcsr* A);
