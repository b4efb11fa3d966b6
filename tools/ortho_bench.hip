// Micro-benchmark of the Gram-Schmidt pass shapes (V' u and r = w - V c) at
// the north-star size, to pick the kernel form: one row per thread with 8-B
// loads (current), two rows per thread with 16-B loads, and grid sizes.
//   hipcc -O3 --offload-arch=gfx950 tools/ortho_bench.hip -o /tmp/ob && /tmp/ob
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);            \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int J>
__global__ __launch_bounds__(256) void dots1(long n, const double* __restrict__ V, long ld,
                                             const double* __restrict__ u, double* __restrict__ part) {
    double acc[J];
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const double ui = u[i];
#pragma unroll
        for (int k = 0; k < J; ++k) acc[k] += V[i + (long)k * ld] * ui;
    }
    double s = 0;
    for (int k = 0; k < J; ++k) s += acc[k];
    if (s == 12345.678) part[blockIdx.x] = s;
}

template <int J>
__global__ __launch_bounds__(256) void dots2(long n, const double* __restrict__ V, long ld,
                                             const double* __restrict__ u, double* __restrict__ part) {
    double acc[J];
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    const long n2 = n / 2;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
        const double2 ui = reinterpret_cast<const double2*>(u)[i];
#pragma unroll
        for (int k = 0; k < J; ++k) {
            const double2 v = reinterpret_cast<const double2*>(V + (long)k * ld)[i];
            acc[k] += v.x * ui.x + v.y * ui.y;
        }
    }
    double s = 0;
    for (int k = 0; k < J; ++k) s += acc[k];
    if (s == 12345.678) part[blockIdx.x] = s;
}

template <int J>
__global__ __launch_bounds__(256) void upd1(long n, const double* __restrict__ V, long ld,
                                            const double* __restrict__ w, double* __restrict__ r,
                                            double* __restrict__ part) {
    double acc[J];
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        double v[J], s = 0;
#pragma unroll
        for (int k = 0; k < J; ++k) v[k] = V[i + (long)k * ld];
#pragma unroll
        for (int k = 0; k < J; ++k) s += v[k] * (0.001 * k);
        const double ri = w[i] - s;
        r[i] = ri;
#pragma unroll
        for (int k = 0; k < J; ++k) acc[k] += v[k] * ri;
    }
    double s = 0;
    for (int k = 0; k < J; ++k) s += acc[k];
    if (s == 12345.678) part[blockIdx.x] = s;
}

template <int J>
__global__ __launch_bounds__(256) void upd2(long n, const double* __restrict__ V, long ld,
                                            const double* __restrict__ w, double* __restrict__ r,
                                            double* __restrict__ part) {
    double acc[J];
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n / 2; i += stride) {
        double2 v[J];
        double sx = 0, sy = 0;
#pragma unroll
        for (int k = 0; k < J; ++k) v[k] = reinterpret_cast<const double2*>(V + (long)k * ld)[i];
#pragma unroll
        for (int k = 0; k < J; ++k) {
            sx += v[k].x * (0.001 * k);
            sy += v[k].y * (0.001 * k);
        }
        const double2 wi = reinterpret_cast<const double2*>(w)[i];
        const double2 ri = make_double2(wi.x - sx, wi.y - sy);
        reinterpret_cast<double2*>(r)[i] = ri;
#pragma unroll
        for (int k = 0; k < J; ++k) acc[k] += v[k].x * ri.x + v[k].y * ri.y;
    }
    double s = 0;
    for (int k = 0; k < J; ++k) s += acc[k];
    if (s == 12345.678) part[blockIdx.x] = s;
}

__global__ void fill(long n, double* x, double v) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) x[i] = v * (i % 7);
}

int main() {
    const long n = 10000000;
    const int J = 20;
    double *V, *u, *r, *part;
    for (long pad : {0L, 64L, 512L}) {
        const long ld = n + pad;
        CK(hipMalloc(&V, sizeof(double) * ld * 32));
        CK(hipMalloc(&u, sizeof(double) * n));
        CK(hipMalloc(&r, sizeof(double) * n));
        CK(hipMalloc(&part, sizeof(double) * 65536));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, ld * 32, V, 1.0);
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, n, u, 2.0);
        CK(hipDeviceSynchronize());
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int grid : {1024, 2048, 4096, 8192}) {
            for (int kind = 0; kind < 4; ++kind) {
                for (int rep = 0; rep < 2; ++rep) {
                    hipEventRecord(a, 0);
                    const int R = 10;
                    for (int it = 0; it < R; ++it) {
                        if (kind == 0) hipLaunchKernelGGL(dots1<J>, dim3(grid), dim3(256), 0, 0, n, V, ld, u, part);
                        if (kind == 1) hipLaunchKernelGGL(dots2<J>, dim3(grid), dim3(256), 0, 0, n, V, ld, u, part);
                        if (kind == 2) hipLaunchKernelGGL(upd1<J>, dim3(grid), dim3(256), 0, 0, n, V, ld, u, r, part);
                        if (kind == 3) hipLaunchKernelGGL(upd2<J>, dim3(grid), dim3(256), 0, 0, n, V, ld, u, r, part);
                    }
                    hipEventRecord(b, 0);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    ms /= R;
                    const double bytes = 8.0 * n * (J + 1 + (kind >= 2 ? 1 : 0));
                    if (rep == 1)
                        printf("{\"pad\": %ld, \"grid\": %d, \"kind\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", pad,
                               grid, kind == 0 ? "dots1" : kind == 1 ? "dots2" : kind == 2 ? "upd1" : "upd2", ms,
                               bytes / ms / 1e6);
                }
            }
        }
        hipFree(V);
        hipFree(u);
        hipFree(r);
        hipFree(part);
    }
    return 0;
}
