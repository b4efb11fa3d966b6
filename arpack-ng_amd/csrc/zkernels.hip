// Complex (complex128) n-length kernels of the znaupd engine and the complex
// CSR operator.  Vectors are interleaved (re, im) doubles, i.e. the layout of
// Fortran COMPLEX*16 / C double _Complex.  All HBM-bound:
//   zdots   partial sums of V(:,c0:c0+8)^H u, 8 columns per pass over u
//   zupdate r = w - V h
//   zgemm   Z = V(:,0:k) M (row-local, alias-safe): znapps V*Q, zneupd
//   zcsr    y = A x, one wavefront per row (measured against 4..32 lanes per row
//           on the config-5 operator: 0.64 ms vs 0.67-0.73 -- the random x
//           gathers, not idle lanes, bound it)
// Reductions are two-stage and fixed-order (bitwise reproducible).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "../../include/arpack_hip.h"
#include "dist.hpp"
#include "zcommon.hpp"
#include "zengine.hpp"

namespace ahip::zdev {

namespace {
using namespace zc;
// part layout: part[slot * nblk + block]; slot 2c = Re, 2c+1 = Im of column c0+c
template <class R, int C>
__global__ __launch_bounds__(kB) void k_zdots(int64_t n, int c0, int cnt,
                                              const typename C2<R>::T* __restrict__ V, int64_t ld,
                                              const typename C2<R>::T* __restrict__ u,
                                              double* __restrict__ part, int nblk) {
    double2 acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = make_double2(0.0, 0.0);
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        const double2 ui = d2(u[i]);
#pragma unroll
        for (int c = 0; c < C; ++c)
            if (c < cnt) {
                const double2 p = cmulc(d2(V[i + (int64_t)(c0 + c) * ld]), ui);
                acc[c].x += p.x;
                acc[c].y += p.y;
            }
    }
    __shared__ double red[4][2 * C];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        if (c < cnt) {
            const double re = wsum(acc[c].x), im = wsum(acc[c].y);
            if (lane == 0) {
                red[wave][2 * c] = re;
                red[wave][2 * c + 1] = im;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < 2 * cnt) {
        const int s = threadIdx.x;
        const double v = (red[0][s] + red[1][s]) + (red[2][s] + red[3][s]);
        part[(int64_t)(2 * c0 + s) * nblk + blockIdx.x] = v;
    }
}

__global__ __launch_bounds__(kB) void k_sum_slots(const double* __restrict__ part, int nblk,
                                                  double* __restrict__ sums) {
    __shared__ double red[4];
    const double* p = part + (int64_t)blockIdx.x * nblk;
    double s = 0.0;
    for (int b = threadIdx.x; b < nblk; b += kB) s += p[b];
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

template <class R>
__global__ __launch_bounds__(kB) void k_zupdate(int64_t n, int j,
                                                const typename C2<R>::T* __restrict__ V, int64_t ld,
                                                const double2* __restrict__ h,
                                                const typename C2<R>::T* rin,
                                                typename C2<R>::T* rout) {
    // the first kSh coefficients are staged in LDS; beyond that (ncv > kSh) they
    // are read from global memory (uniform across the block: cache hits)
    constexpr int kSh = 256;
    __shared__ double2 sh[kSh];
    for (int c = threadIdx.x; c < j && c < kSh; c += kB) sh[c] = h[c];
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        double2 r = d2(rin[i]);
        for (int c = 0; c < j; ++c) {
            const double2 p = cmul(d2(V[i + (int64_t)c * ld]), c < kSh ? sh[c] : h[c]);
            r.x -= p.x;
            r.y -= p.y;
        }
        rout[i] = st2<R>(r);
    }
}

template <class R, int MAXK>
__global__ __launch_bounds__(kB) void k_zgemm(int64_t n, const typename C2<R>::T* V, int64_t ld,
                                              int k, int nz, const double2* __restrict__ M,
                                              typename C2<R>::T* Z, int64_t ldz) {
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        double2 v[MAXK];
#pragma unroll
        for (int t = 0; t < MAXK; ++t) v[t] = (t < k) ? d2(V[i + (int64_t)t * ld]) : make_double2(0.0, 0.0);
        for (int l = 0; l < nz; ++l) {
            double2 o = make_double2(0.0, 0.0);
#pragma unroll
            for (int t = 0; t < MAXK; ++t)
                if (t < k) {
                    const double2 p = cmul(v[t], M[t + (int64_t)l * k]);
                    o.x += p.x;
                    o.y += p.y;
                }
            Z[i + (int64_t)l * ldz] = st2<R>(o);
        }
    }
}

// Z = V(:,0:k) * M for k > 64, alias-safe through per-thread scratch columns
// (tmp[l * S + tid], S = grid threads); same summation order as k_zgemm
template <class R>
__global__ __launch_bounds__(kB) void k_zgemm_generic(int64_t n, const typename C2<R>::T* V,
                                                      int64_t ld, int k, int nz,
                                                      const double2* __restrict__ M,
                                                      typename C2<R>::T* Z, int64_t ldz,
                                                      double2* __restrict__ tmp) {
    const int64_t stride = (int64_t)gridDim.x * kB;
    const int64_t tid = (int64_t)blockIdx.x * kB + threadIdx.x;
    for (int64_t i = tid; i < n; i += stride) {
        for (int l = 0; l < nz; ++l) tmp[l * stride + tid] = make_double2(0.0, 0.0);
        for (int t = 0; t < k; ++t) {
            const double2 vt = d2(V[i + (int64_t)t * ld]);
            for (int l = 0; l < nz; ++l) {
                const double2 p = cmul(vt, M[t + (int64_t)l * k]);
                double2 o = tmp[l * stride + tid];
                o.x += p.x;
                o.y += p.y;
                tmp[l * stride + tid] = o;
            }
        }
        for (int l = 0; l < nz; ++l) Z[i + (int64_t)l * ldz] = st2<R>(tmp[l * stride + tid]);
    }
}

template <class R>
__global__ void k_zaxpby(int64_t n, double2 a, typename C2<R>::T* y, double2 b,
                         const typename C2<R>::T* x) {
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        double2 r = cmul(a, d2(y[i]));
        if (x) {
            const double2 p = cmul(b, d2(x[i]));
            r.x += p.x;
            r.y += p.y;
        }
        y[i] = st2<R>(r);
    }
}

template <class R>
__global__ void k_zger(int64_t n, int k, const typename C2<R>::T* __restrict__ x,
                       const double2* __restrict__ w, typename C2<R>::T* Z, int64_t ldz) {
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        const double2 xi = d2(x[i]);
        for (int c = 0; c < k; ++c) {
            const double2 p = cmul(xi, w[c]);
            double2 z = d2(Z[i + (int64_t)c * ldz]);
            z.x += p.x;
            z.y += p.y;
            Z[i + (int64_t)c * ldz] = st2<R>(z);
        }
    }
}

// y = A x, one 64-lane wavefront per row, fixed-order lane reduction
__global__ __launch_bounds__(kB) void k_zcsr(int64_t n, const int64_t* __restrict__ rp,
                                             const int32_t* __restrict__ col,
                                             const double2* __restrict__ val,
                                             const double2* __restrict__ x, double2* __restrict__ y,
                                             const int* __restrict__ gate) {
    if (gate && *gate) return;  // a finished Krylov solve (zsolve.hip) skips its queued products
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * kB + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * kB) >> 6;
    for (int64_t r = wid; r < n; r += nw) {
        double re = 0.0, im = 0.0;
        for (int64_t k = rp[r] + lane; k < rp[r + 1]; k += 64) {
            const double2 p = cmul(val[k], x[col[k]]);
            re += p.x;
            im += p.y;
        }
        re = wsum(re);
        im = wsum(im);
        if (lane == 0) y[r] = make_double2(re, im);
    }
}

// ---- complex random operator (BASELINE config 5) ----------
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
constexpr int kMaxPerRow = 128;

__device__ void zrow(int64_t i, int64_t n, uint32_t sm, int per_row, uint32_t* cols, double* re,
                     double* im) {
    for (int k = 0; k < per_row; ++k) {
        const uint32_t h = mix32(mix32((uint32_t)i ^ sm) + (uint32_t)k * 0x9E3779B9u);
        cols[k] = (uint32_t)((uint64_t)h % (uint64_t)n);
        re[k] = (double)(mix32(h ^ 0x68e31da4u) >> 21) * 0x1p-10 - 1.0;
        im[k] = (double)(mix32(h ^ 0x1b873593u) >> 21) * 0x1p-10 - 1.0;
    }
    for (int a = 1; a < per_row; ++a) {  // insertion sort by column (stable)
        const uint32_t c = cols[a];
        const double xr = re[a], xi = im[a];
        int b = a - 1;
        while (b >= 0 && cols[b] > c) {
            cols[b + 1] = cols[b];
            re[b + 1] = re[b];
            im[b + 1] = im[b];
            --b;
        }
        cols[b + 1] = c;
        re[b + 1] = xr;
        im[b + 1] = xi;
    }
}

__global__ void k_zgen_count(int64_t n, uint32_t sm, int per_row, int64_t* cnt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t cols[kMaxPerRow];
        double re[kMaxPerRow], im[kMaxPerRow];
        zrow(i, n, sm, per_row, cols, re, im);
        int64_t c = 0;
        bool diag = false;
        for (int k = 0; k < per_row; ++k) {
            if (k == 0 || cols[k] != cols[k - 1]) ++c;
            if (cols[k] == (uint32_t)i) diag = true;
        }
        cnt[i] = c + (diag ? 0 : 1);
    }
}

__global__ void k_zgen_fill(int64_t n, uint32_t sm, int per_row, double dshift, const int64_t* rp,
                            int32_t* col, double2* val) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t cols[kMaxPerRow];
        double re[kMaxPerRow], im[kMaxPerRow];
        zrow(i, n, sm, per_row, cols, re, im);
        int64_t o = rp[i];
        bool dput = false;
        for (int k = 0; k < per_row;) {
            const uint32_t c = cols[k];
            if (!dput && c > (uint32_t)i) {  // diagonal not hit by the hash: insert it
                col[o] = (int32_t)i;
                val[o++] = make_double2(dshift, 0.0);
                dput = true;
            }
            double sr = 0.0, si = 0.0;
            while (k < per_row && cols[k] == c) {  // duplicates summed (exact: 2^-10 grid)
                sr += re[k];
                si += im[k];
                ++k;
            }
            if (c == (uint32_t)i) {
                sr += dshift;
                dput = true;
            }
            col[o] = (int32_t)c;
            val[o++] = make_double2(sr, si);
        }
        if (!dput) {
            col[o] = (int32_t)i;
            val[o++] = make_double2(dshift, 0.0);
        }
    }
}

inline int grid(int64_t n, int cap = 8192) {
    int64_t g = (n + kB - 1) / kB;
    if (g > cap) g = cap;
    return (int)(g < 1 ? 1 : g);
}
}  // namespace

template <class R>
void dots(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, const R* u, const R* w,
          std::complex<double>* out) {
    using T = typename C2<R>::T;
    const T* V2 = reinterpret_cast<const T*>(V);
    const T* u2 = reinterpret_cast<const T*>(u);
    for (int c0 = 0; c0 < j; c0 += 8) {
        const int cnt = j - c0 < 8 ? j - c0 : 8;
        hipLaunchKernelGGL((k_zdots<R, 8>), dim3(ws.nblk), dim3(kB), 0, ws.stream, n, c0, cnt, V2, ld,
                           u2, ws.part, ws.nblk);
    }
    // slot j: w^H u (a "column" at w with ld irrelevant)
    if (w) {
        hipLaunchKernelGGL((k_zdots<R, 1>), dim3(ws.nblk), dim3(kB), 0, ws.stream, n, 0, 1,
                           reinterpret_cast<const T*>(w), 0, u2, ws.part + (int64_t)2 * j * ws.nblk,
                           ws.nblk);
    }
    const int m = 2 * (j + (w ? 1 : 0));
    hipLaunchKernelGGL(k_sum_slots, dim3(m), dim3(kB), 0, ws.stream, ws.part, ws.nblk, ws.sums);
    if (ws.comm) comm_allreduce_sum(ws.comm, ws.sums, m, ws.stream);  // the ranks' local sums
    ws.ck(hipMemcpyAsync(ws.host, ws.sums, sizeof(double) * m, hipMemcpyDeviceToHost, ws.stream));
    ws.ck(hipStreamSynchronize(ws.stream));
    for (int c = 0; c < m / 2; ++c) out[c] = std::complex<double>(ws.host[2 * c], ws.host[2 * c + 1]);
}

template <class R>
void update(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, const std::complex<double>* h,
            const R* rin, R* rout) {
    using T = typename C2<R>::T;
    if (j > 0) ws.ck(hipMemcpyAsync(ws.coef, h, sizeof(double) * 2 * j, hipMemcpyHostToDevice, ws.stream));
    hipLaunchKernelGGL(k_zupdate<R>, dim3(grid(n)), dim3(kB), 0, ws.stream, n, j,
                       reinterpret_cast<const T*>(V), ld, reinterpret_cast<const double2*>(ws.coef),
                       reinterpret_cast<const T*>(rin), reinterpret_cast<T*>(rout));
    ws.ck(hipStreamSynchronize(ws.stream));  // h is host memory
}

template <class R>
void gemm(const Ws& ws, int64_t n, const R* V, int64_t ld, int k, int nz,
          const std::complex<double>* M, R* Z, int64_t ldz) {
    using T = typename C2<R>::T;
    ws.ck(hipMemcpyAsync(ws.q, M, sizeof(double) * 2 * (size_t)k * nz, hipMemcpyHostToDevice, ws.stream));
    auto V2 = reinterpret_cast<const T*>(V);
    auto M2 = reinterpret_cast<const double2*>(ws.q);
    auto Z2 = reinterpret_cast<T*>(Z);
    if (k <= 16)
        hipLaunchKernelGGL((k_zgemm<R, 16>), dim3(grid(n)), dim3(kB), 0, ws.stream, n, V2, ld, k, nz, M2,
                           Z2, ldz);
    else if (k <= 32)
        hipLaunchKernelGGL((k_zgemm<R, 32>), dim3(grid(n)), dim3(kB), 0, ws.stream, n, V2, ld, k, nz, M2,
                           Z2, ldz);
    else if (k <= 40)  // ncv = 40 (config 5): 40 row values in registers, not 64
        hipLaunchKernelGGL((k_zgemm<R, 40>), dim3(grid(n)), dim3(kB), 0, ws.stream, n, V2, ld, k, nz, M2,
                           Z2, ldz);
    else if (k <= 64)
        hipLaunchKernelGGL((k_zgemm<R, 64>), dim3(grid(n)), dim3(kB), 0, ws.stream, n, V2, ld, k, nz, M2,
                           Z2, ldz);
    else  // grid = nblk: ws.scratch holds nblk * kB rows of ncv outputs
        hipLaunchKernelGGL((k_zgemm_generic<R>), dim3(ws.nblk), dim3(kB), 0, ws.stream, n, V2, ld, k,
                           nz, M2, Z2, ldz, reinterpret_cast<double2*>(ws.scratch));
    ws.ck(hipStreamSynchronize(ws.stream));
}

template <class R>
void axpby(const Ws& ws, int64_t n, std::complex<double> a, R* y, std::complex<double> b,
           const R* x) {
    using T = typename C2<R>::T;
    hipLaunchKernelGGL(k_zaxpby<R>, dim3(grid(n)), dim3(kB), 0, ws.stream, n,
                       make_double2(a.real(), a.imag()), reinterpret_cast<T*>(y),
                       make_double2(b.real(), b.imag()), reinterpret_cast<const T*>(x));
}

template <class R>
void ger(const Ws& ws, int64_t n, int k, const R* x, const std::complex<double>* w, R* Z,
         int64_t ldz) {
    using T = typename C2<R>::T;
    ws.ck(hipMemcpyAsync(ws.coef, w, sizeof(double) * 2 * k, hipMemcpyHostToDevice, ws.stream));
    hipLaunchKernelGGL(k_zger<R>, dim3(grid(n)), dim3(kB), 0, ws.stream, n, k,
                       reinterpret_cast<const T*>(x), reinterpret_cast<const double2*>(ws.coef),
                       reinterpret_cast<T*>(Z), ldz);
    ws.ck(hipStreamSynchronize(ws.stream));
}

#define AHIP_ZINST(R)                                                                              \
    template void dots<R>(const Ws&, int64_t, int, const R*, int64_t, const R*, const R*,          \
                          std::complex<double>*);                                                  \
    template void update<R>(const Ws&, int64_t, int, const R*, int64_t,                            \
                            const std::complex<double>*, const R*, R*);                            \
    template void gemm<R>(const Ws&, int64_t, const R*, int64_t, int, int,                         \
                          const std::complex<double>*, R*, int64_t);                               \
    template void axpby<R>(const Ws&, int64_t, std::complex<double>, R*, std::complex<double>,     \
                           const R*);                                                              \
    template void ger<R>(const Ws&, int64_t, int, const R*, const std::complex<double>*, R*,       \
                         int64_t);
AHIP_ZINST(double)
AHIP_ZINST(float)
#undef AHIP_ZINST

static hipError_t ws_alloc(Ws& ws, int64_t n, int ncv, hipStream_t s);

// on failure everything allocated so far is released (ws left empty)
hipError_t ws_create(Ws& ws, int64_t n, int ncv, hipStream_t s) {
    const hipError_t e = ws_alloc(ws, n, ncv, s);
    if (e != hipSuccess) ws_destroy(ws);
    return e;
}

static hipError_t ws_alloc(Ws& ws, int64_t n, int ncv, hipStream_t s) {
    ws.stream = s;
    int64_t g = (n + kB - 1) / kB;
    ws.nblk = (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
    const int slots = 2 * (ncv + 2);
    hipError_t e;
    if ((e = hipMalloc(&ws.part, sizeof(double) * (size_t)ws.nblk * slots))) return e;
    if ((e = hipMalloc(&ws.sums, sizeof(double) * slots))) return e;
    ws.cstride = ncv + 2;
    // coefficient slots: CGS h, DGKS-1, DGKS-2, and the fold's t = H s
    if ((e = hipMalloc(&ws.coef, sizeof(double) * 2 * 4 * (size_t)ws.cstride))) return e;
    ws.hld = ncv;
    if ((e = hipMalloc(&ws.hcol, sizeof(double) * 2 * (size_t)ncv * ncv))) return e;
    if ((e = hipMalloc(&ws.rec, sizeof(double) * (size_t)(ncv + 1)))) return e;
    if ((e = hipMalloc(&ws.st, sizeof(dev::LzState)))) return e;
    if ((e = hipHostMalloc(&ws.st_host, sizeof(dev::LzState)))) return e;
    memset(ws.st_host, 0, sizeof(dev::LzState));
    {   // test hook, as the real engine's (AHIP_FORCE_DGKS2=1)
        const char* f = getenv("AHIP_FORCE_DGKS2");
        ws.st_host->force_dgks2 = (f && f[0] == '1') ? 1 : 0;
    }
    if ((e = hipMemcpyAsync(ws.st, ws.st_host, sizeof(dev::LzState), hipMemcpyHostToDevice, s))) return e;
    if ((e = hipMalloc(&ws.q, sizeof(double) * 2 * (size_t)ncv * ncv))) return e;
    if ((e = hipHostMalloc(&ws.host, sizeof(double) * slots))) return e;
    if (ncv > 64 &&  // per-thread output columns of k_zgemm_generic
        (e = hipMalloc(&ws.scratch, sizeof(double) * 2 * (size_t)ws.nblk * kB * ncv)))
        return e;
    return hipSuccess;
}

void ws_destroy(Ws& ws) {
    if (ws.part) (void)hipFree(ws.part);
    if (ws.sums) (void)hipFree(ws.sums);
    if (ws.coef) (void)hipFree(ws.coef);
    if (ws.q) (void)hipFree(ws.q);
    if (ws.host) (void)hipHostFree(ws.host);
    if (ws.scratch) (void)hipFree(ws.scratch);
    if (ws.hcol) (void)hipFree(ws.hcol);
    if (ws.rec) (void)hipFree(ws.rec);
    if (ws.st) (void)hipFree(ws.st);
    if (ws.st_host) (void)hipHostFree(ws.st_host);
    ws = Ws{};
}

void zcsr_spmv(hipStream_t s, const ZCsr& A, const double* x, double* y, const int* gate) {
    if (A.split) return zcsr_split_spmv(s, A, x, y, gate);  // zsplit.hip
    hipLaunchKernelGGL(k_zcsr, dim3(grid(A.n * 64, 65536)), dim3(kB), 0, s, A.n, A.rowptr, A.col,
                       reinterpret_cast<const double2*>(A.val), reinterpret_cast<const double2*>(x),
                       reinterpret_cast<double2*>(y), gate);
}

int gen_zrandom(ZCsr& A, int64_t n, int per_row, uint32_t seed, double dshift) {
    if (per_row < 1 || per_row > kMaxPerRow) return -1;
    int64_t *cnt = nullptr, *rp = nullptr;
    int32_t* col = nullptr;
    double* val = nullptr;
    auto fail = [&]() {  // every HIP error ends here: nothing leaks, A stays empty
        for (void* q : {(void*)cnt, (void*)rp, (void*)col, (void*)val})
            if (q) (void)hipFree(q);
        return -1;
    };
    if (hipMalloc(&cnt, sizeof(int64_t) * (n + 1)) || hipMalloc(&rp, sizeof(int64_t) * (n + 1)))
        return fail();
    const uint32_t sm = mix32(seed);
    hipLaunchKernelGGL(k_zgen_count, dim3(grid(n, 65536)), dim3(kB), 0, nullptr, n, sm, per_row, cnt);
    std::vector<int64_t> h(n + 1);
    if (hipMemcpy(h.data(), cnt, sizeof(int64_t) * n, hipMemcpyDeviceToHost)) return fail();
    int64_t acc = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c = h[i];
        h[i] = acc;
        acc += c;
    }
    h[n] = acc;
    if (hipMemcpy(rp, h.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice)) return fail();
    (void)hipFree(cnt);
    cnt = nullptr;
    if (hipMalloc(&col, sizeof(int32_t) * (acc ? acc : 1)) ||
        hipMalloc(&val, sizeof(double) * 2 * (acc ? acc : 1)))
        return fail();
    hipLaunchKernelGGL(k_zgen_fill, dim3(grid(n, 65536)), dim3(kB), 0, nullptr, n, sm, per_row, dshift, rp,
                       col, reinterpret_cast<double2*>(val));
    if (hipDeviceSynchronize() != hipSuccess) return fail();
    A.n = n;
    A.nnz = acc;
    A.rowptr = rp;
    A.col = col;
    A.val = val;
    A.owned = true;
    return 0;
}

}  // namespace ahip::zdev
