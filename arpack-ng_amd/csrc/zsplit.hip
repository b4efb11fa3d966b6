// XCD column split of the complex CSR operator (config 5: n = 5e5, ~100
// random columns a row).  x (8 MB) does not fit one XCD's 4 MB L2, so the
// wave-per-row kernel's random gathers miss to the Infinity Cache (0.63 ms,
// 1.6 TB/s of algorithmic bytes).  Here the columns are cut into 8 slices of
// x; workgroup b works on slice b % 8 -- the hardware deals workgroups
// round-robin over the 8 XCDs, so every slice's gathers stay in ONE XCD's L2 --
// with 8 lanes a row on the slice's own CSR (slice-relative 16-bit columns,
// non-temporal matrix loads), and writes a partial y per slice; a second
// kernel sums the 8 partials in a fixed order.  tools/zspmv_split.hip: 0.41 ms
// against 0.63 (and 0.72 for the same split WITHOUT the XCD alignment: the
// alignment, not the split, is the gain); results within 5e-16 of the
// wave-per-row kernel (a different, fixed summation order).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdlib>

#include "zcommon.hpp"
#include "zengine.hpp"

namespace ahip::zdev {

namespace {
using namespace zc;
constexpr int kSlices = 8;  // = XCDs
constexpr int kLanes = 8;   // lanes per row (tools/zspmv_split.hip: 8 of 4/8/16)

__global__ void k_zsplit_count(int64_t n, int64_t sw, const int64_t* __restrict__ rp,
                               const int32_t* __restrict__ col, int32_t* __restrict__ cnt) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        int32_t c[kSlices] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) c[col[k] / sw]++;
#pragma unroll
        for (int s = 0; s < kSlices; ++s) cnt[(int64_t)s * (n + 1) + r] = c[s];
    }
}

template <class CT>
__global__ void k_zsplit_fill(int64_t n, int64_t sw, const int64_t* __restrict__ rp,
                              const int32_t* __restrict__ col, const double2* __restrict__ val,
                              const int32_t* __restrict__ srp, const int64_t* __restrict__ base,
                              CT* __restrict__ scol, double2* __restrict__ sval) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        int64_t pos[kSlices];
#pragma unroll
        for (int s = 0; s < kSlices; ++s) pos[s] = base[s] + srp[(int64_t)s * (n + 1) + r];
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {  // row order kept inside each slice
            const int s = (int)(col[k] / sw);
            scol[pos[s]] = (CT)(col[k] - s * sw);
            sval[pos[s]] = val[k];
            pos[s]++;
        }
    }
}

template <class CT>
__global__ __launch_bounds__(256) void k_zsplit_spmv(int64_t n, int64_t sw,
                                                     const int32_t* __restrict__ srp,
                                                     const int64_t* __restrict__ base,
                                                     const CT* __restrict__ scol,
                                                     const double2* __restrict__ sval,
                                                     const double2* __restrict__ x,
                                                     double2* __restrict__ yp,
                                                     const int* __restrict__ gate) {
    if (gate && *gate) return;  // a finished Krylov solve (zsolve.hip) skips its queued products
    typedef double dv2 __attribute__((ext_vector_type(2)));
    const int s = (int)(blockIdx.x % kSlices);  // the XCD this workgroup runs on
    const int64_t q = blockIdx.x / kSlices, nq = gridDim.x / kSlices;
    const int lane = threadIdx.x & (kLanes - 1);
    constexpr int64_t kRows = 256 / kLanes;
    const int32_t* rp = srp + (int64_t)s * (n + 1);
    const int64_t b0 = base[s];
    const double2* xs = x + (int64_t)s * sw;
    double2* y = yp + (int64_t)s * n;
    for (int64_t r = q * kRows + threadIdx.x / kLanes; r < n; r += nq * kRows) {
        double re = 0.0, im = 0.0;
        const int64_t k1 = b0 + rp[r + 1];
        for (int64_t k = b0 + rp[r] + lane; k < k1; k += kLanes) {
            const dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(sval) + k);
            const double2 xv = xs[__builtin_nontemporal_load(&scol[k])];
            re += v.x * xv.x - v.y * xv.y;
            im += v.x * xv.y + v.y * xv.x;
        }
#pragma unroll
        for (int o = kLanes / 2; o > 0; o >>= 1) {
            re += __shfl_xor(re, o, kLanes);
            im += __shfl_xor(im, o, kLanes);
        }
        if (lane == 0) y[r] = make_double2(re, im);
    }
}

__global__ void k_zsplit_combine(int64_t n, const double2* __restrict__ yp, double2* __restrict__ y,
                                 const int* __restrict__ gate) {
    if (gate && *gate) return;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        double2 a[kSlices];
#pragma unroll
        for (int s = 0; s < kSlices; ++s) a[s] = yp[(int64_t)s * n + r];
        y[r] = make_double2(((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x)),
                            ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y)));
    }
}

inline int grid1(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}
}  // namespace

void zcsr_free_split(ZCsr& A) {
    if (A.s_rp) (void)hipFree(A.s_rp);
    if (A.s_base) (void)hipFree(A.s_base);
    if (A.s_col) (void)hipFree(A.s_col);
    if (A.s_val) (void)hipFree(A.s_val);
    if (A.s_y) (void)hipFree(A.s_y);
    A.s_rp = nullptr;
    A.s_base = nullptr;
    A.s_col = nullptr;
    A.s_val = nullptr;
    A.s_y = nullptr;
    A.split = false;
}

int zcsr_build_split(ZCsr& A) {
    static const bool off = [] {
        const char* e = getenv("AHIP_ZSPLIT");
        return e && e[0] == '0';
    }();
    const int64_t n = A.n;
    if (off || n < (int64_t(1) << 18) || A.nnz < 32 * n) return 1;
    const int64_t sw = (n + kSlices - 1) / kSlices;
    A.s_w = sw;
    A.s_col16 = sw <= 65536;
    const size_t cb = A.s_col16 ? 2 : 4;
    int32_t* cnt = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto fail = [&](int rc) {
        if (cnt) (void)hipFree(cnt);
        if (tmp) (void)hipFree(tmp);
        zcsr_free_split(A);
        return rc;
    };
    if (hipMalloc(&cnt, sizeof(int32_t) * kSlices * (n + 1)) ||
        hipMalloc(&A.s_rp, sizeof(int32_t) * kSlices * (n + 1)) ||
        hipMalloc(&A.s_base, sizeof(int64_t) * (kSlices + 1)))
        return fail(-2);
    hipLaunchKernelGGL(k_zsplit_count, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr, A.col, cnt);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, cnt, A.s_rp, (int)(n + 1));
    if (hipMalloc(&tmp, tmpb ? tmpb : 1)) return fail(-2);
    int64_t hb[kSlices + 1];
    hb[0] = 0;
    for (int s = 0; s < kSlices; ++s) {
        int32_t* c = cnt + (size_t)s * (n + 1);
        (void)hipMemsetAsync(c + n, 0, sizeof(int32_t), nullptr);
        // per-slice row offsets; int32: a slice holds < 2^31 entries (checked below)
        (void)hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, c, A.s_rp + (size_t)s * (n + 1), (int)(n + 1));
        int32_t tot = 0;
        if (hipMemcpy(&tot, A.s_rp + (size_t)s * (n + 1) + n, sizeof(int32_t), hipMemcpyDeviceToHost))
            return fail(-1);
        if (tot < 0) return fail(1);  // int32 overflow: keep the wave-per-row kernel
        hb[s + 1] = hb[s] + tot;
    }
    if (hb[kSlices] != A.nnz) return fail(-1);
    (void)hipMemcpy(A.s_base, hb, sizeof(hb), hipMemcpyHostToDevice);
    (void)hipFree(cnt);
    cnt = nullptr;
    (void)hipFree(tmp);
    tmp = nullptr;
    if (hipMalloc(&A.s_col, cb * (A.nnz ? A.nnz : 1)) || hipMalloc(&A.s_val, 16 * (A.nnz ? A.nnz : 1)) ||
        hipMalloc(&A.s_y, 16 * (size_t)kSlices * n))
        return fail(-2);
    const auto* v2 = reinterpret_cast<const double2*>(A.val);
    if (A.s_col16)
        hipLaunchKernelGGL(k_zsplit_fill<uint16_t>, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr,
                           A.col, v2, A.s_rp, A.s_base, (uint16_t*)A.s_col, (double2*)A.s_val);
    else
        hipLaunchKernelGGL(k_zsplit_fill<int32_t>, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr,
                           A.col, v2, A.s_rp, A.s_base, (int32_t*)A.s_col, (double2*)A.s_val);
    if (hipDeviceSynchronize() != hipSuccess) return fail(-1);
    A.split = true;
    return 0;
}

void zcsr_split_spmv(hipStream_t s, const ZCsr& A, const double* x, double* y, const int* gate) {
    const auto* x2 = reinterpret_cast<const double2*>(x);
    auto* yp = reinterpret_cast<double2*>(A.s_y);
    const int g = 1024;  // 128 workgroups a slice (tools/zspmv_split.hip)
    if (A.s_col16)
        hipLaunchKernelGGL(k_zsplit_spmv<uint16_t>, dim3(g), dim3(256), 0, s, A.n, A.s_w, A.s_rp, A.s_base,
                           (const uint16_t*)A.s_col, (const double2*)A.s_val, x2, yp, gate);
    else
        hipLaunchKernelGGL(k_zsplit_spmv<int32_t>, dim3(g), dim3(256), 0, s, A.n, A.s_w, A.s_rp, A.s_base,
                           (const int32_t*)A.s_col, (const double2*)A.s_val, x2, yp, gate);
    hipLaunchKernelGGL(k_zsplit_combine, dim3(2048), dim3(256), 0, s, A.n, yp, reinterpret_cast<double2*>(y),
                       gate);
}

}  // namespace ahip::zdev
