// Direct tridiagonal solve for the device shift-invert operator (DShift method
// kDShiftTridiag): y = C^{-1} b with C = A - sigma I (or the generalized
// modes' C = A - sigma M) tridiagonal -- what the reference's drivers do on the
// host with LAPACK's dgttrf / dgttrs (EXAMPLES/NONSYM/dndrv2.f:197-258,
// dndrv4.f; EXAMPLES/SYM/dsdrv2.f), for the operators a Krylov solve cannot
// serve: dndrv2's strongly non-normal convection-diffusion takes BiCGStab
// ~3,500 iterations to stagnate near 2e-11, and no restarted GMRES converges
// on it.
//
// The factorization is dgttrf restated (LU with partial pivoting: row
// interchanges between neighbours, a second superdiagonal du2), once, on the
// host.  The two triangular solves are linear recurrences,
//   forward   c_{i+1} = alpha_i c_i + beta_i        (one state value)
//   backward  (x_i, x_{i+1}) = M_i (x_{i+1}, x_{i+2}) + v_i   (two)
// which the device evaluates as a parallel scan of affine maps instead of
// dgttrs's sequential loops: each thread composes the maps of a contiguous
// segment, the block scans the segment composites in LDS, one thread carries
// the block composites across the grid, and every thread then re-applies its
// segment from its incoming state.  The association differs from the
// sequential loop's, so the result equals dgttrs's to rounding (for the
// stable recurrences a pivoted LU gives: |multipliers| <= 1), not bitwise;
// `arpack_hip_kit_dgttrf` / `_dgttrs` keep the sequential restatement for the
// CPU tests against LAPACK.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/arpack_hip.h"
#include "dshift.hpp"

namespace ahip::dev {

namespace {

constexpr int kTT = 256;  // threads a block

// z -> M z + v on a 2-vector state
struct AMap {
    double m00, m01, m10, m11, v0, v1;
};
__device__ __forceinline__ AMap amap_id() { return AMap{1.0, 0.0, 0.0, 1.0, 0.0, 0.0}; }
// (b after a): z -> b(a(z))
__device__ __forceinline__ AMap amap_then(const AMap& a, const AMap& b) {
    return AMap{b.m00 * a.m00 + b.m01 * a.m10, b.m00 * a.m01 + b.m01 * a.m11,
                b.m10 * a.m00 + b.m11 * a.m10, b.m10 * a.m01 + b.m11 * a.m11,
                b.m00 * a.v0 + b.m01 * a.v1 + b.v0, b.m10 * a.v0 + b.m11 * a.v1 + b.v1};
}
__device__ __forceinline__ void amap_apply(const AMap& a, double& z0, double& z1) {
    const double t0 = a.m00 * z0 + a.m01 * z1 + a.v0;
    const double t1 = a.m10 * z0 + a.m11 * z1 + a.v1;
    z0 = t0;
    z1 = t1;
}

// The forward solve's map k (k = 0..n-2) takes c_k to c_{k+1}; the state's
// second component stays 0.  Output: y_k = c_k, or (a row interchange at k)
// the original b_{k+1}; y_{n-1} = c_{n-1}.
struct Fwd {
    const double* dl;
    const int* ipiv;
    const double* b;
    double* y;
    int64_t n;
    __device__ AMap map(int64_t k) const {
        const double bn = b[k + 1];
        if (ipiv[k] == k) return AMap{-dl[k], 0.0, 0.0, 0.0, bn, 0.0};
        return AMap{1.0, 0.0, 0.0, 0.0, -dl[k] * bn, 0.0};
    }
    __device__ void out(int64_t k, double before0, double after0) const {
        y[k] = ipiv[k] == k ? before0 : b[k + 1];
        if (k == n - 2) y[n - 1] = after0;
    }
};

// The backward solve's map k (k = 0..n-1) is row i = n-1-k:
// (x_i, x_{i+1}) = [[-du_i/d_i, -du2_i/d_i], [1, 0]] (x_{i+1}, x_{i+2}) + (y_i/d_i, 0)
// with du_{n-1} = du2_{n-2} = du2_{n-1} = 0 (x_n = x_{n+1} = 0).  Output x_i.
struct Bwd {
    const double* d;
    const double* du;
    const double* du2;
    const double* y;
    double* x;
    int64_t n;
    __device__ AMap map(int64_t k) const {
        const int64_t i = n - 1 - k;
        const double u1 = i + 1 < n ? du[i] : 0.0;
        const double u2 = i + 2 < n ? du2[i] : 0.0;
        const double r = 1.0 / d[i];
        return AMap{-u1 * r, -u2 * r, 1.0, 0.0, y[i] * r, 0.0};
    }
    __device__ void out(int64_t k, double, double after0) const { x[n - 1 - k] = after0; }
};

// segment of thread t of block b over m maps: [lo, hi)
__device__ __forceinline__ void seg_range(int64_t m, int64_t per, int64_t& lo, int64_t& hi) {
    lo = ((int64_t)blockIdx.x * kTT + threadIdx.x) * per;
    hi = lo + per < m ? lo + per : m;
    if (lo > m) lo = m;
}

// inclusive scan of the block's segment composites in LDS; returns this
// thread's EXCLUSIVE prefix and writes the block total to *total (thread 0)
__device__ AMap block_scan(AMap mine, AMap* total) {
    __shared__ AMap s[kTT];
    const int t = threadIdx.x;
    s[t] = mine;
    __syncthreads();
    for (int o = 1; o < kTT; o <<= 1) {
        AMap v = s[t];
        if (t >= o) v = amap_then(s[t - o], v);
        __syncthreads();
        s[t] = v;
        __syncthreads();
    }
    if (t == kTT - 1 && total) *total = s[t];
    const AMap ex = t > 0 ? s[t - 1] : amap_id();
    __syncthreads();
    return ex;
}

template <class F>
__global__ __launch_bounds__(kTT) void k_tri_local(F f, int64_t m, int64_t per, AMap* __restrict__ bc) {
    int64_t lo, hi;
    seg_range(m, per, lo, hi);
    AMap c = amap_id();
    for (int64_t k = lo; k < hi; ++k) c = amap_then(c, f.map(k));
    AMap tot;
    (void)block_scan(c, &tot);
    if (threadIdx.x == kTT - 1) bc[blockIdx.x] = tot;
}

// the state entering every block, from the initial state (*z0p or 0, 0)
__global__ void k_tri_carry(const AMap* __restrict__ bc, int nb, const double* __restrict__ z0p,
                            double* __restrict__ cin) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double z0 = z0p ? z0p[0] : 0.0, z1 = 0.0;
    for (int b = 0; b < nb; ++b) {
        cin[2 * b] = z0;
        cin[2 * b + 1] = z1;
        amap_apply(bc[b], z0, z1);
    }
}

template <class F>
__global__ __launch_bounds__(kTT) void k_tri_apply(F f, int64_t m, int64_t per,
                                                   const double* __restrict__ cin) {
    int64_t lo, hi;
    seg_range(m, per, lo, hi);
    AMap c = amap_id();
    for (int64_t k = lo; k < hi; ++k) c = amap_then(c, f.map(k));
    const AMap ex = block_scan(c, nullptr);
    double z0 = cin[2 * blockIdx.x], z1 = cin[2 * blockIdx.x + 1];
    amap_apply(ex, z0, z1);
    for (int64_t k = lo; k < hi; ++k) {
        const double b0 = z0;
        amap_apply(f.map(k), z0, z1);
        f.out(k, b0, z0);
    }
}

__global__ void k_scale1(const double* __restrict__ d, const double* __restrict__ a, double* __restrict__ b) {
    b[0] = a[0] / d[0];
}

// grid of a scan over m maps: per-thread segments of >= 16 maps, <= 1024 blocks
void scan_geom(int64_t m, int& nb, int64_t& per) {
    const int64_t threads = (m + 15) / 16;
    int64_t b = (threads + kTT - 1) / kTT;
    if (b > 1024) b = 1024;
    if (b < 1) b = 1;
    nb = (int)b;
    per = (m + b * kTT - 1) / (b * kTT);
    if (per < 1) per = 1;
}

template <class F>
void run_scan(hipStream_t s, const F& f, int64_t m, const double* z0p, DShift& S) {
    int nb;
    int64_t per;
    scan_geom(m, nb, per);
    hipLaunchKernelGGL(k_tri_local<F>, dim3(nb), dim3(kTT), 0, s, f, m, per,
                       reinterpret_cast<AMap*>(S.tri_bc));
    hipLaunchKernelGGL(k_tri_carry, dim3(1), dim3(64), 0, s, reinterpret_cast<const AMap*>(S.tri_bc), nb,
                       z0p, S.tri_cin);
    hipLaunchKernelGGL(k_tri_apply<F>, dim3(nb), dim3(kTT), 0, s, f, m, per, S.tri_cin);
}

}  // namespace

// dgttrf (LAPACK 3.x, SRC/dgttrf.f) restated: LU of the tridiagonal (dl, d, du)
// with partial pivoting; du2 the second superdiagonal of U, ipiv 0-based.
// 0, or i + 1 when U(i, i) is exactly zero.
int tri_factor(int64_t n, double* dl, double* d, double* du, double* du2, int* ipiv) {
    for (int64_t i = 0; i < n; ++i) ipiv[i] = (int)i;
    for (int64_t i = 0; i + 2 < n; ++i) du2[i] = 0.0;
    for (int64_t i = 0; i + 2 < n; ++i) {
        if (std::fabs(d[i]) >= std::fabs(dl[i])) {  // no row interchange
            if (d[i] != 0.0) {
                const double fact = dl[i] / d[i];
                dl[i] = fact;
                d[i + 1] = d[i + 1] - fact * du[i];
            }
        } else {  // interchange rows i and i + 1
            const double fact = d[i] / dl[i];
            d[i] = dl[i];
            dl[i] = fact;
            const double temp = du[i];
            du[i] = d[i + 1];
            d[i + 1] = temp - fact * d[i + 1];
            du2[i] = du[i + 1];
            du[i + 1] = -fact * du[i + 1];
            ipiv[i] = (int)(i + 1);
        }
    }
    if (n > 1) {
        const int64_t i = n - 2;
        if (std::fabs(d[i]) >= std::fabs(dl[i])) {
            if (d[i] != 0.0) {
                const double fact = dl[i] / d[i];
                dl[i] = fact;
                d[i + 1] = d[i + 1] - fact * du[i];
            }
        } else {
            const double fact = d[i] / dl[i];
            d[i] = dl[i];
            dl[i] = fact;
            const double temp = du[i];
            du[i] = d[i + 1];
            d[i + 1] = temp - fact * d[i + 1];
            ipiv[i] = (int)(i + 1);
        }
    }
    for (int64_t i = 0; i < n; ++i)
        if (d[i] == 0.0) return (int)(i + 1);
    return 0;
}

// dgttrs (trans = 'N', one right-hand side; SRC/dgtts2.f) restated, sequential
void tri_solve_host(int64_t n, const double* dl, const double* d, const double* du, const double* du2,
                    const int* ipiv, double* b) {
    for (int64_t i = 0; i + 1 < n; ++i) {
        const int64_t ip = ipiv[i];
        const double temp = b[i + 1 - ip + i] - dl[i] * b[ip];
        b[i] = b[ip];
        b[i + 1] = temp;
    }
    b[n - 1] = b[n - 1] / d[n - 1];
    if (n > 1) b[n - 2] = (b[n - 2] - du[n - 2] * b[n - 1]) / d[n - 2];
    for (int64_t i = n - 3; i >= 0; --i) b[i] = (b[i] - du[i] * b[i + 1] - du2[i] * b[i + 2]) / d[i];
}

// Factor C = A - sigma I of S.A (which must be tridiagonal) for the direct
// solve: 0; -1 not tridiagonal (an entry outside |i - j| <= 1) or singular;
// -2 HIP failure.
int dshift_tridiag_factor(DShift& S) {
    const Csr& A = *S.A;
    const int64_t n = A.n;
    if (n < 1) return -1;
    std::vector<int64_t> rp((size_t)n + 1);
    std::vector<int32_t> col((size_t)(A.nnz > 0 ? A.nnz : 1));
    std::vector<double> val((size_t)(A.nnz > 0 ? A.nnz : 1));
    if (hipMemcpy(rp.data(), A.rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost) != hipSuccess ||
        (A.nnz > 0 &&
         (hipMemcpy(col.data(), A.col, sizeof(int32_t) * A.nnz, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(val.data(), A.val, sizeof(double) * A.nnz, hipMemcpyDeviceToHost) != hipSuccess)))
        return -2;
    std::vector<double> dl((size_t)n, 0.0), d((size_t)n, 0.0), du((size_t)n, 0.0), du2((size_t)n, 0.0);
    std::vector<int> ipiv((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            const int64_t j = col[k];
            if (j == i) d[i] += val[k];
            else if (j == i - 1) dl[i - 1] += val[k];
            else if (j == i + 1) du[i] += val[k];
            else return -1;
        }
        d[i] -= S.sigma;
    }
    if (tri_factor(n, dl.data(), d.data(), du.data(), du2.data(), ipiv.data()) != 0) return -1;
    const int nbmax = 1024;
    hipError_t e = hipSuccess;
    auto alloc = [&](auto*& p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(&p, bytes);
    };
    alloc(S.tri_dl, sizeof(double) * n);
    alloc(S.tri_d, sizeof(double) * n);
    alloc(S.tri_du, sizeof(double) * n);
    alloc(S.tri_du2, sizeof(double) * n);
    alloc(S.tri_ipiv, sizeof(int) * n);
    alloc(S.tri_bc, sizeof(AMap) * nbmax);
    alloc(S.tri_cin, sizeof(double) * 2 * nbmax);
    if (e == hipSuccess) e = hipMemcpy(S.tri_dl, dl.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(S.tri_d, d.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(S.tri_du, du.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(S.tri_du2, du2.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(S.tri_ipiv, ipiv.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        dshift_tridiag_free(S);
        return -2;
    }
    return 0;
}

void dshift_tridiag_free(DShift& S) {
    for (void* p : {(void*)S.tri_dl, (void*)S.tri_d, (void*)S.tri_du, (void*)S.tri_du2, (void*)S.tri_ipiv,
                    (void*)S.tri_bc, (void*)S.tri_cin})
        if (p) (void)hipFree(p);
    S.tri_dl = S.tri_d = S.tri_du = S.tri_du2 = S.tri_cin = nullptr;
    S.tri_ipiv = nullptr;
    S.tri_bc = nullptr;
}

// y = C^{-1} b on `s` (b, y device, not aliased; the forward result goes to the
// solver's first work vector)
int dshift_tridiag_apply(DShift& S, hipStream_t s, const double* b, double* y) {
    const int64_t n = S.n;
    double* w = S.vec[0];
    if (n == 1) {
        hipLaunchKernelGGL(k_scale1, dim3(1), dim3(1), 0, s, S.tri_d, b, y);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    // forward: c_0 = b_0, maps 0..n-2
    run_scan(s, Fwd{S.tri_dl, S.tri_ipiv, b, w, n}, n - 1, b, S);
    // backward: z_n = (0, 0), maps 0..n-1 (rows n-1..0)
    run_scan(s, Bwd{S.tri_d, S.tri_du, S.tri_du2, w, y, n}, n, nullptr, S);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace ahip::dev

extern "C" {

// CPU-testable restatements (tests/test_kit_tri.py against LAPACK's own)
int arpack_hip_kit_dgttrf(int64_t n, double* dl, double* d, double* du, double* du2, int* ipiv) {
    return ahip::dev::tri_factor(n, dl, d, du, du2, ipiv);
}
void arpack_hip_kit_dgttrs(int64_t n, const double* dl, const double* d, const double* du,
                           const double* du2, const int* ipiv, double* b) {
    ahip::dev::tri_solve_host(n, dl, d, du, du2, ipiv, b);
}

}  // extern "C"
