// Device conjugate gradients for the shift-invert operator y = (A - sigma I)^{-1} b
// of the symmetric engine (mode 3, SRC/dsaupd.f:30-48; see dshift.hpp).
//
// One iteration k (x0 = 0, r0 = p0 = b, rho_0 = b'b):
//
//   w = A p                                   csr_spmv (full or symmetric storage)
//   q = w - sigma p;  P0 <- partials of p'q   k_cg_pq
//   alpha = rho_k / p'q;  y += alpha p;       k_cg_xr   (reduces P0; p'q <= 0: breakdown)
//   r -= alpha q;     P1 <- partials of r'r
//   rho_{k+1} = r'r;  stop if ||r|| <= rtol ||b||, else
//   p = r + (rho_{k+1} / rho_k) p             k_cg_p    (reduces P1)
//
// Every block of a reducing kernel sums the previous kernel's per-block
// partials itself in one fixed order (all blocks hold the same scalars; results
// reproducible run to run); block 0 records them in the device state.  A kernel
// never writes the partial buffer it reads.  The SpMVs are not gated: after
// the stop the remaining products of the enqueued chunk run on a frozen p and
// feed nothing (the host sizes its chunks from the previous solve's count, or
// from the residual's decrease so far, so few are spent).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "dshift.hpp"
#include "passes.hpp"

namespace ahip::dev {

namespace {
constexpr int kT = 256;       // threads a block
constexpr int kMaxBlk = 512;  // blocks of the vector kernels (partials per slot)

template <int NS>
__device__ __forceinline__ void cg_put(const double (&acc)[NS], double* __restrict__ part, int nblk) {
    __shared__ double red[kT / 64][NS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const double v = wave_sum(acc[q]);
        if (lane == 0) red[wave][q] = v;
    }
    __syncthreads();
    if (threadIdx.x < NS) {
        const int q = threadIdx.x;
        part[(int64_t)q * nblk + blockIdx.x] = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
    }
}

__device__ __forceinline__ double cg_total(const double* __restrict__ part, int nblk) {
    __shared__ double red[kT / 64];
    double a = 0.0;
    for (int b = threadIdx.x; b < nblk; b += kT) a += part[b];
    a = wave_sum(a);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(kT) void k_cg_init(int64_t n, const double* __restrict__ b,
                                                double* __restrict__ r, double* __restrict__ p,
                                                double* __restrict__ y, double* __restrict__ part,
                                                int nblk) {
    double acc[1] = {0.0};
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        const double bi = b[i];
        r[i] = bi;
        p[i] = bi;
        y[i] = 0.0;
        acc[0] += bi * bi;
    }
    cg_put<1>(acc, part, nblk);
}

__global__ __launch_bounds__(kT) void k_cg_init_fin(const double* __restrict__ part, int nblk,
                                                    CgState* __restrict__ st) {
    const double t = cg_total(part, nblk);
    if (threadIdx.x == 0) {
        st->done = t == 0.0 ? 1 : 0;  // b = 0: y = 0 is exact
        st->breakdown = 0;
        st->iters = 0;
        st->failed = 0;
        st->rho[0] = t;
        st->bnorm2 = t;
        st->rnorm2 = t;
    }
}

// partials of p'(w - sigma p)
__global__ __launch_bounds__(kT) void k_cg_pq(int64_t n, const double* __restrict__ w,
                                              const double* __restrict__ p, double sigma,
                                              const CgState* __restrict__ st,
                                              double* __restrict__ part, int nblk) {
    if (st->done) return;
    double acc[1] = {0.0};
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        const double pi = p[i];
        acc[0] += pi * (w[i] - sigma * pi);
    }
    cg_put<1>(acc, part, nblk);
}

// alpha = rho_k / p'q; y += alpha p; r -= alpha q; partials of r'r
__global__ __launch_bounds__(kT) void k_cg_xr(int64_t n, const double* __restrict__ w,
                                              const double* __restrict__ p, double sigma,
                                              double* __restrict__ y, double* __restrict__ r,
                                              CgState* __restrict__ st, int k,
                                              const double* __restrict__ part_in,
                                              double* __restrict__ part_out, int nblk) {
    if (st->done) return;
    const double pq = cg_total(part_in, nblk);
    if (!(pq > 0.0)) {  // not positive definite along p (or NaN): CG cannot continue
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->breakdown = 1;
            st->failed = 1;
            st->iters = k;
            st->done = 1;
        }
        return;
    }
    const double alpha = st->rho[k & 1] / pq;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->alpha = alpha;
    double acc[1] = {0.0};
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        const double pi = p[i];
        y[i] += alpha * pi;
        const double ri = r[i] - alpha * (w[i] - sigma * pi);
        r[i] = ri;
        acc[0] += ri * ri;
    }
    cg_put<1>(acc, part_out, nblk);
}

// rho_{k+1} = r'r, convergence test; p = r + beta p
__global__ __launch_bounds__(kT) void k_cg_p(int64_t n, const double* __restrict__ r,
                                             double* __restrict__ p, CgState* __restrict__ st,
                                             int k, double rtol2, const double* __restrict__ part,
                                             int nblk) {
    if (st->done) return;
    const double rho1 = cg_total(part, nblk);
    const double rho0 = st->rho[k & 1];
    const bool conv = rho1 <= rtol2 * st->bnorm2;
    const bool stop = conv || rho1 == 0.0 || !(rho1 == rho1);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->rho[(k + 1) & 1] = rho1;
        st->rnorm2 = rho1;
        if (stop) {
            st->iters = k + 1;
            st->failed = conv ? 0 : 1;
            st->done = 1;
        }
    }
    if (stop) return;
    const double beta = rho1 / rho0;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT)
        p[i] = r[i] + beta * p[i];
}

}  // namespace

int dshift_create(DShift& S, const Csr* A, double sigma, double rtol, int maxit) {
    S = DShift{};
    S.A = A;
    S.sigma = sigma;
    S.rtol = rtol;
    S.maxit = maxit;
    S.n = A->n;
    int64_t g = (S.n + kT - 1) / kT;
    S.nblk = (int)(g < 1 ? 1 : (g > kMaxBlk ? kMaxBlk : g));
    const size_t vb = sizeof(double) * (size_t)(S.n > 0 ? S.n : 1);
    hipError_t e = hipSuccess;
    double** vecs[] = {&S.r, &S.p, &S.w};
    for (double** q : vecs)
        if (e == hipSuccess) e = hipMalloc(q, vb);
    if (e == hipSuccess) e = hipMalloc(&S.part, sizeof(double) * 2 * (size_t)S.nblk);
    if (e == hipSuccess) e = hipMalloc(&S.st, sizeof(CgState));
    if (e == hipSuccess) e = hipHostMalloc(&S.st_host, sizeof(CgState));
    if (e == hipSuccess) e = hipEventCreate(&S.ev0);
    if (e == hipSuccess) e = hipEventCreate(&S.ev1);
    if (e != hipSuccess) {
        dshift_destroy(S);
        return (int)e;
    }
    std::memset(S.st_host, 0, sizeof(CgState));
    return 0;
}

void dshift_destroy(DShift& S) {
    double* vecs[] = {S.r, S.p, S.w, S.part};
    for (double* q : vecs)
        if (q) (void)hipFree(q);
    if (S.st) (void)hipFree(S.st);
    if (S.st_host) (void)hipHostFree(S.st_host);
    if (S.ev0) (void)hipEventDestroy(S.ev0);
    if (S.ev1) (void)hipEventDestroy(S.ev1);
    S = DShift{};
}

double dshift_iter_bytes(const DShift& S) {
    // the product as its storage streams it (csr_bytes: matrix + x/y), and the
    // 11 n-vector passes of k_cg_pq (w, p), k_cg_xr (w, p, y, r; y, r) and k_cg_p (r, p; p)
    return csr_bytes(*S.A) + 88.0 * (double)S.n;
}

int dshift_apply(DShift& S, hipStream_t strm, const double* b, double* y, double* relres) {
    const int64_t n = S.n;
    const int nb = S.nblk;
    double* P0 = S.part;
    double* P1 = S.part + nb;
    if (hipEventRecord(S.ev0, strm) != hipSuccess) return -2;
    hipLaunchKernelGGL(k_cg_init, dim3(nb), dim3(kT), 0, strm, n, b, S.r, S.p, y, P0, nb);
    hipLaunchKernelGGL(k_cg_init_fin, dim3(1), dim3(kT), 0, strm, P0, nb, S.st);
    const double rtol2 = S.rtol * S.rtol;
    int k = 0, chunk = S.chunk > 0 ? S.chunk : 8;
    bool done = false;
    while (k < S.maxit) {
        const int m = chunk < S.maxit - k ? chunk : S.maxit - k;
        for (int q = 0; q < m; ++q, ++k) {
            csr_spmv(strm, *S.A, S.p, S.w);
            hipLaunchKernelGGL(k_cg_pq, dim3(nb), dim3(kT), 0, strm, n, S.w, S.p, S.sigma, S.st, P0, nb);
            hipLaunchKernelGGL(k_cg_xr, dim3(nb), dim3(kT), 0, strm, n, S.w, S.p, S.sigma, y, S.r, S.st,
                               k, P0, P1, nb);
            hipLaunchKernelGGL(k_cg_p, dim3(nb), dim3(kT), 0, strm, n, S.r, S.p, S.st, k, rtol2, P1, nb);
        }
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(S.st_host, S.st, sizeof(CgState), hipMemcpyDeviceToHost, strm) !=
                hipSuccess ||
            hipStreamSynchronize(strm) != hipSuccess)
            return -2;
        if (S.st_host->done) {
            done = true;
            break;
        }
        // the next chunk from the residual's geometric decrease so far (CG on
        // a fixed operator: log(r'r / b'b) falls about linearly in k), bounded
        // so that a stall costs few idle products
        const CgState& h = *S.st_host;
        int next = 2 * chunk;
        if (h.rnorm2 > 0.0 && h.rnorm2 < h.bnorm2 && k > 0) {
            const double rate = std::log(h.rnorm2 / h.bnorm2) / k;  // < 0
            const double need = std::log(rtol2) / rate - k;
            next = need < 2.0 ? 2 : (int)std::ceil(0.9 * need);
        }
        chunk = next < 2 ? 2 : (next > 256 ? 256 : next);
    }
    if (hipEventRecord(S.ev1, strm) != hipSuccess || hipEventSynchronize(S.ev1) != hipSuccess)
        return -2;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, S.ev0, S.ev1) == hipSuccess) S.ms_total += ms;
    const CgState& h = *S.st_host;
    const int iters = done ? h.iters : S.maxit;
    const double rr = h.bnorm2 > 0.0 ? std::sqrt(h.rnorm2 / h.bnorm2) : 0.0;
    if (relres) *relres = rr;
    S.n_solves += 1;
    S.n_iters += iters;
    if (rr > S.max_relres) S.max_relres = rr;
    // the next solve enqueues this one's count first (the shift-invert solves of
    // one Lanczos run take similar counts)
    S.chunk = iters > 0 ? iters : 1;
    if (!done || h.failed || (h.bnorm2 > 0.0 && !(h.rnorm2 <= S.rtol * S.rtol * h.bnorm2))) {
        S.n_fail += 1;
        return -1;
    }
    return iters;
}

}  // namespace ahip::dev
