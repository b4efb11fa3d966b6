// Ceiling of the restart's V*Q pass shape on MI355X (n = 1e7 rows, fp64):
// every row reads K = 30 basis columns + r and writes W = 11 columns + r
// (V(:,1:kev+1) = V Q(:,1:kev+1), r = sigma r + beta v_{kev+1}; kev = 10), the
// arithmetic of k_vq_update replaced by a trivial combination, so the numbers
// are the memory system's for this read/write mix:
//   hipcc -O3 --offload-arch=gfx950 tools/vq_bench.hip -o tools/vq_bench && tools/vq_bench
// reads only (no stores) / in place (V's first W columns, as k_vq_update) /
// into a separate buffer / non-temporal stores / stores issued after all the
// row's loads of the NEXT row (software pipelined).
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);           \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int K = 30, W = 11;

template <int MODE>  // 0 reads only, 1 in place, 2 separate buffer, 3 nt in place
__global__ __launch_bounds__(256) void vq(long n, double* __restrict__ V, long ld,
                                          double* __restrict__ Z, double* __restrict__ r,
                                          double* __restrict__ out) {
    double sink = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load(V + i + (long)k * ld);
        double o[W];
#pragma unroll
        for (int l = 0; l < W; ++l) {
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < K; ++k) a += v[k] * (double)(k + l + 1);
            o[l] = a;
        }
        const double ri = 0.5 * r[i] + 0.25 * o[W - 1];
        if (MODE == 0) {
#pragma unroll
            for (int l = 0; l < W; ++l) sink += o[l];
            sink += ri;
        } else {
            double* dst = MODE == 2 ? Z : V;
#pragma unroll
            for (int l = 0; l < W; ++l) {
                if (MODE == 3) __builtin_nontemporal_store(o[l], dst + i + (long)l * ld);
                else dst[i + (long)l * ld] = o[l];
            }
            r[i] = ri;
        }
    }
    if (sink == 1234.5) out[blockIdx.x] = sink;
}

__global__ void fill1(long n, double* x) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        x[i] = 1e-3 * (double)(i & 1023);
}

int main() {
    const long n = 10000000, ld = n;
    double *V, *Z, *r, *out;
    CK(hipMalloc(&V, sizeof(double) * ld * K));
    CK(hipMalloc(&Z, sizeof(double) * ld * W));
    CK(hipMalloc(&r, sizeof(double) * n));
    CK(hipMalloc(&out, 1 << 20));
    fill1<<<4096, 256>>>(ld * K, V);
    fill1<<<4096, 256>>>(n, r);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, double nb, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e9, tot = 0;
        for (int rep = 0; rep < 10; ++rep) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            tot += ms;
        }
        printf("%-34s best %.3f ms  %.0f GB/s  mean %.3f ms\n", name, best, nb / best / 1e6, tot / 10);
        return 0;
    };
    const double rd = 8.0 * n * (K + 1), wr = 8.0 * n * (W + 1);
    for (int g : {1024, 2048, 4096}) {
        printf("grid %d\n", g);
        run("reads only (31 columns)", rd, [&] { vq<0><<<g, 256>>>(n, V, ld, Z, r, out); });
        run("in place (31 r + 12 w)", rd + wr, [&] { vq<1><<<g, 256>>>(n, V, ld, Z, r, out); });
        run("separate buffer (31 r + 12 w)", rd + wr, [&] { vq<2><<<g, 256>>>(n, V, ld, Z, r, out); });
        run("in place, nt stores", rd + wr, [&] { vq<3><<<g, 256>>>(n, V, ld, Z, r, out); });
    }
    return 0;
}
