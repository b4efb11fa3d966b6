// Direct complex tridiagonal solve for the device shift-invert operator of the
// complex engine (ZShift method 1): y = (A - sigma I)^{-1} b with A tridiagonal
// -- what the reference's complex driver does on the host with LAPACK's zgttrf
// / zgttrs (EXAMPLES/COMPLEX/zndrv2.f:179, 250), the complex twin of dtri.hip.
//
// The factorization is zgttrf restated (LU with partial pivoting by CABS1 =
// |re| + |im|, as LAPACK's zgttrf compares; a second superdiagonal du2), once,
// on the host.  The two triangular solves are linear recurrences evaluated on
// the device as a parallel scan of complex affine maps (dtri.hip's scheme:
// per-thread segment composites, an LDS block scan, a one-thread carry across
// blocks, a re-apply pass), so the result equals zgttrs's to rounding, not
// bitwise; `arpack_hip_kit_zgttrf` / `_zgttrs` keep the sequential restatement
// for the CPU tests against LAPACK.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstring>
#include <vector>

#include "../../include/arpack_hip.h"
#include "zcommon.hpp"
#include "zsolve.hpp"

namespace ahip::zdev {

namespace {
using zc::cmul;
using cd = std::complex<double>;

constexpr int kTT = 256;  // threads a block

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 cneg(double2 a) { return make_double2(-a.x, -a.y); }
// a / b (Smith's algorithm, as zsolve.hip's)
__device__ __forceinline__ double2 cdivd(double2 a, double2 b) {
    if (fabs(b.x) < fabs(b.y)) {
        const double ratio = b.x / b.y, denom = b.x * ratio + b.y;
        return make_double2((a.x * ratio + a.y) / denom, (a.y * ratio - a.x) / denom);
    }
    const double ratio = b.y / b.x, denom = b.y * ratio + b.x;
    return make_double2((a.y * ratio + a.x) / denom, (a.y - a.x * ratio) / denom);
}

// z -> M z + v on a 2-vector complex state
struct ZMap {
    double2 m00, m01, m10, m11, v0, v1;
};
__device__ __forceinline__ ZMap zmap_id() {
    const double2 o = make_double2(1.0, 0.0), z = make_double2(0.0, 0.0);
    return ZMap{o, z, z, o, z, z};
}
// (b after a): z -> b(a(z))
__device__ __forceinline__ ZMap zmap_then(const ZMap& a, const ZMap& b) {
    return ZMap{cadd(cmul(b.m00, a.m00), cmul(b.m01, a.m10)), cadd(cmul(b.m00, a.m01), cmul(b.m01, a.m11)),
                cadd(cmul(b.m10, a.m00), cmul(b.m11, a.m10)), cadd(cmul(b.m10, a.m01), cmul(b.m11, a.m11)),
                cadd(cadd(cmul(b.m00, a.v0), cmul(b.m01, a.v1)), b.v0),
                cadd(cadd(cmul(b.m10, a.v0), cmul(b.m11, a.v1)), b.v1)};
}
__device__ __forceinline__ void zmap_apply(const ZMap& a, double2& z0, double2& z1) {
    const double2 t0 = cadd(cadd(cmul(a.m00, z0), cmul(a.m01, z1)), a.v0);
    const double2 t1 = cadd(cadd(cmul(a.m10, z0), cmul(a.m11, z1)), a.v1);
    z0 = t0;
    z1 = t1;
}

// forward solve (L with the row interchanges): map k (k = 0..n-2) takes c_k to
// c_{k+1}; output y_k = c_k, or (an interchange at k) the original b_{k+1}
struct ZFwd {
    const double2* dl;
    const int* ipiv;
    const double2* b;
    double2* y;
    int64_t n;
    __device__ ZMap map(int64_t k) const {
        const double2 z = make_double2(0.0, 0.0), bn = b[k + 1];
        if (ipiv[k] == k) return ZMap{cneg(dl[k]), z, z, z, bn, z};
        return ZMap{make_double2(1.0, 0.0), z, z, z, cneg(cmul(dl[k], bn)), z};
    }
    __device__ void out(int64_t k, double2 before0, double2 after0) const {
        y[k] = ipiv[k] == k ? before0 : b[k + 1];
        if (k == n - 2) y[n - 1] = after0;
    }
};

// backward solve (U): map k is row i = n-1-k,
// (x_i, x_{i+1}) = [[-du_i/d_i, -du2_i/d_i], [1, 0]] (x_{i+1}, x_{i+2}) + (y_i/d_i, 0)
struct ZBwd {
    const double2* d;
    const double2* du;
    const double2* du2;
    const double2* y;
    double2* x;
    int64_t n;
    __device__ ZMap map(int64_t k) const {
        const int64_t i = n - 1 - k;
        const double2 z = make_double2(0.0, 0.0), one = make_double2(1.0, 0.0);
        const double2 u1 = i + 1 < n ? du[i] : z;
        const double2 u2 = i + 2 < n ? du2[i] : z;
        return ZMap{cneg(cdivd(u1, d[i])), cneg(cdivd(u2, d[i])), one, z, cdivd(y[i], d[i]), z};
    }
    __device__ void out(int64_t k, double2, double2 after0) const { x[n - 1 - k] = after0; }
};

__device__ __forceinline__ void seg_range(int64_t m, int64_t per, int64_t& lo, int64_t& hi) {
    lo = ((int64_t)blockIdx.x * kTT + threadIdx.x) * per;
    hi = lo + per < m ? lo + per : m;
    if (lo > m) lo = m;
}

// inclusive scan of the block's segment composites in LDS; this thread's
// EXCLUSIVE prefix, the block total to *total (the last thread)
__device__ ZMap zblock_scan(ZMap mine, ZMap* total) {
    __shared__ ZMap s[kTT];
    const int t = threadIdx.x;
    s[t] = mine;
    __syncthreads();
    for (int o = 1; o < kTT; o <<= 1) {
        ZMap v = s[t];
        if (t >= o) v = zmap_then(s[t - o], v);
        __syncthreads();
        s[t] = v;
        __syncthreads();
    }
    if (t == kTT - 1 && total) *total = s[t];
    const ZMap ex = t > 0 ? s[t - 1] : zmap_id();
    __syncthreads();
    return ex;
}

template <class F>
__global__ __launch_bounds__(kTT) void k_ztri_local(F f, int64_t m, int64_t per, ZMap* __restrict__ bc) {
    int64_t lo, hi;
    seg_range(m, per, lo, hi);
    ZMap c = zmap_id();
    for (int64_t k = lo; k < hi; ++k) c = zmap_then(c, f.map(k));
    ZMap tot;
    (void)zblock_scan(c, &tot);
    if (threadIdx.x == kTT - 1) bc[blockIdx.x] = tot;
}

// the state entering every block, from the initial state (*z0p or 0, 0)
__global__ void k_ztri_carry(const ZMap* __restrict__ bc, int nb, const double2* __restrict__ z0p,
                             double2* __restrict__ cin) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double2 z0 = z0p ? z0p[0] : make_double2(0.0, 0.0), z1 = make_double2(0.0, 0.0);
    for (int b = 0; b < nb; ++b) {
        cin[2 * b] = z0;
        cin[2 * b + 1] = z1;
        zmap_apply(bc[b], z0, z1);
    }
}

template <class F>
__global__ __launch_bounds__(kTT) void k_ztri_apply(F f, int64_t m, int64_t per,
                                                    const double2* __restrict__ cin) {
    int64_t lo, hi;
    seg_range(m, per, lo, hi);
    ZMap c = zmap_id();
    for (int64_t k = lo; k < hi; ++k) c = zmap_then(c, f.map(k));
    const ZMap ex = zblock_scan(c, nullptr);
    double2 z0 = cin[2 * blockIdx.x], z1 = cin[2 * blockIdx.x + 1];
    zmap_apply(ex, z0, z1);
    for (int64_t k = lo; k < hi; ++k) {
        const double2 b0 = z0;
        zmap_apply(f.map(k), z0, z1);
        f.out(k, b0, z0);
    }
}

__global__ void k_zscale1(const double2* __restrict__ d, const double2* __restrict__ a, double2* __restrict__ b) {
    b[0] = cdivd(a[0], d[0]);
}

// grid of a scan over m maps: per-thread segments of >= 16 maps, <= 1024 blocks
void zscan_geom(int64_t m, int& nb, int64_t& per) {
    const int64_t threads = (m + 15) / 16;
    int64_t b = (threads + kTT - 1) / kTT;
    if (b > 1024) b = 1024;
    if (b < 1) b = 1;
    nb = (int)b;
    per = (m + b * kTT - 1) / (b * kTT);
    if (per < 1) per = 1;
}

template <class F>
void zrun_scan(hipStream_t s, const F& f, int64_t m, const double2* z0p, ZShift& S) {
    int nb;
    int64_t per;
    zscan_geom(m, nb, per);
    hipLaunchKernelGGL(k_ztri_local<F>, dim3(nb), dim3(kTT), 0, s, f, m, per,
                       reinterpret_cast<ZMap*>(S.tri_bc));
    hipLaunchKernelGGL(k_ztri_carry, dim3(1), dim3(64), 0, s, reinterpret_cast<const ZMap*>(S.tri_bc), nb,
                       z0p, reinterpret_cast<double2*>(S.tri_cin));
    hipLaunchKernelGGL(k_ztri_apply<F>, dim3(nb), dim3(kTT), 0, s, f, m, per,
                       reinterpret_cast<const double2*>(S.tri_cin));
}

inline double cabs1(const cd& z) { return std::fabs(z.real()) + std::fabs(z.imag()); }

}  // namespace

// zgttrf (LAPACK 3.x, SRC/zgttrf.f) restated: LU of the tridiagonal (dl, d, du)
// with partial pivoting by CABS1; du2 the second superdiagonal of U, ipiv
// 0-based.  0, or i + 1 when U(i, i) is exactly zero.
int ztri_factor(int64_t n, cd* dl, cd* d, cd* du, cd* du2, int* ipiv) {
    for (int64_t i = 0; i < n; ++i) ipiv[i] = (int)i;
    for (int64_t i = 0; i + 2 < n; ++i) du2[i] = 0.0;
    auto step = [&](int64_t i, bool inner) {
        if (cabs1(d[i]) >= cabs1(dl[i])) {  // no row interchange
            if (cabs1(d[i]) != 0.0) {
                const cd fact = dl[i] / d[i];
                dl[i] = fact;
                d[i + 1] = d[i + 1] - fact * du[i];
            }
        } else {  // interchange rows i and i + 1
            const cd fact = d[i] / dl[i];
            d[i] = dl[i];
            dl[i] = fact;
            const cd temp = du[i];
            du[i] = d[i + 1];
            d[i + 1] = temp - fact * d[i + 1];
            if (inner) {
                du2[i] = du[i + 1];
                du[i + 1] = -fact * du[i + 1];
            }
            ipiv[i] = (int)(i + 1);
        }
    };
    for (int64_t i = 0; i + 2 < n; ++i) step(i, true);
    if (n > 1) step(n - 2, false);
    for (int64_t i = 0; i < n; ++i)
        if (cabs1(d[i]) == 0.0) return (int)(i + 1);
    return 0;
}

// zgttrs (trans = 'N', one right-hand side; SRC/zgtts2.f) restated, sequential
void ztri_solve_host(int64_t n, const cd* dl, const cd* d, const cd* du, const cd* du2, const int* ipiv,
                     cd* b) {
    for (int64_t i = 0; i + 1 < n; ++i) {
        if (ipiv[i] == i) {
            b[i + 1] = b[i + 1] - dl[i] * b[i];
        } else {
            const cd temp = b[i];
            b[i] = b[i + 1];
            b[i + 1] = temp - dl[i] * b[i];
        }
    }
    b[n - 1] = b[n - 1] / d[n - 1];
    if (n > 1) b[n - 2] = (b[n - 2] - du[n - 2] * b[n - 1]) / d[n - 2];
    for (int64_t i = n - 3; i >= 0; --i) b[i] = (b[i] - du[i] * b[i + 1] - du2[i] * b[i + 2]) / d[i];
}

int zshift_tridiag_factor(ZShift& S) {
    const ZCsr& A = *S.A;
    const int64_t n = A.n;
    if (n < 1) return -1;
    std::vector<int64_t> rp((size_t)n + 1);
    std::vector<int32_t> col((size_t)(A.nnz > 0 ? A.nnz : 1));
    std::vector<cd> val((size_t)(A.nnz > 0 ? A.nnz : 1));
    if (hipMemcpy(rp.data(), A.rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost) != hipSuccess ||
        (A.nnz > 0 &&
         (hipMemcpy(col.data(), A.col, sizeof(int32_t) * A.nnz, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(val.data(), A.val, sizeof(cd) * A.nnz, hipMemcpyDeviceToHost) != hipSuccess)))
        return -2;
    std::vector<cd> dl((size_t)n, 0.0), d((size_t)n, 0.0), du((size_t)n, 0.0), du2((size_t)n, 0.0);
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
    if (ztri_factor(n, dl.data(), d.data(), du.data(), du2.data(), ipiv.data()) != 0) return -1;
    zshift_tridiag_free(S);
    const int nbmax = 1024;
    hipError_t e = hipSuccess;
    auto alloc = [&](auto*& p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(&p, bytes);
    };
    alloc(S.tri_dl, sizeof(cd) * n);
    alloc(S.tri_d, sizeof(cd) * n);
    alloc(S.tri_du, sizeof(cd) * n);
    alloc(S.tri_du2, sizeof(cd) * n);
    alloc(S.tri_ipiv, sizeof(int) * n);
    alloc(S.tri_bc, sizeof(ZMap) * nbmax);
    alloc(S.tri_cin, sizeof(cd) * 2 * nbmax);
    auto up = [&](double* dst, const std::vector<cd>& v) {
        if (e == hipSuccess) e = hipMemcpy(dst, v.data(), sizeof(cd) * n, hipMemcpyHostToDevice);
    };
    up(S.tri_dl, dl);
    up(S.tri_d, d);
    up(S.tri_du, du);
    up(S.tri_du2, du2);
    if (e == hipSuccess) e = hipMemcpy(S.tri_ipiv, ipiv.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        zshift_tridiag_free(S);
        return -2;
    }
    S.method = 1;
    return 0;
}

void zshift_tridiag_free(ZShift& S) {
    for (void* p : {(void*)S.tri_dl, (void*)S.tri_d, (void*)S.tri_du, (void*)S.tri_du2, (void*)S.tri_ipiv,
                    S.tri_bc, (void*)S.tri_cin})
        if (p) (void)hipFree(p);
    S.tri_dl = S.tri_d = S.tri_du = S.tri_du2 = S.tri_cin = nullptr;
    S.tri_ipiv = nullptr;
    S.tri_bc = nullptr;
    S.method = 0;
}

// y = (A - sigma I)^{-1} b on `s` (b, y device, not aliased; the forward
// result goes to the solver's work vector w)
int zshift_tridiag_apply(ZShift& S, hipStream_t s, const double* b, double* y) {
    const int64_t n = S.n;
    const auto* b2 = reinterpret_cast<const double2*>(b);
    auto* y2 = reinterpret_cast<double2*>(y);
    auto* w = reinterpret_cast<double2*>(S.w);
    const auto* dl = reinterpret_cast<const double2*>(S.tri_dl);
    const auto* d = reinterpret_cast<const double2*>(S.tri_d);
    const auto* du = reinterpret_cast<const double2*>(S.tri_du);
    const auto* du2 = reinterpret_cast<const double2*>(S.tri_du2);
    if (n == 1) {
        hipLaunchKernelGGL(k_zscale1, dim3(1), dim3(1), 0, s, d, b2, y2);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    zrun_scan(s, ZFwd{dl, S.tri_ipiv, b2, w, n}, n - 1, b2, S);
    zrun_scan(s, ZBwd{d, du, du2, w, y2, n}, n, nullptr, S);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace ahip::zdev

extern "C" {

// CPU-testable restatements (tests/test_kit_tri.py against LAPACK's own);
// complex arrays interleaved (re, im)
int arpack_hip_kit_zgttrf(int64_t n, double* dl, double* d, double* du, double* du2, int* ipiv) {
    using cd = std::complex<double>;
    return ahip::zdev::ztri_factor(n, reinterpret_cast<cd*>(dl), reinterpret_cast<cd*>(d),
                                   reinterpret_cast<cd*>(du), reinterpret_cast<cd*>(du2), ipiv);
}
void arpack_hip_kit_zgttrs(int64_t n, const double* dl, const double* d, const double* du,
                           const double* du2, const int* ipiv, double* b) {
    using cd = std::complex<double>;
    ahip::zdev::ztri_solve_host(n, reinterpret_cast<const cd*>(dl), reinterpret_cast<const cd*>(d),
                                reinterpret_cast<const cd*>(du), reinterpret_cast<const cd*>(du2), ipiv,
                                reinterpret_cast<cd*>(b));
}

}  // extern "C"
