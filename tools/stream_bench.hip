// Read-stream ceiling on MI355X for the shapes of the Lanczos passes (n = 1e7
// rows, J basis columns, fp64): what rate can a pass over V reach at all?
//   hipcc -O3 --offload-arch=gfx950 tools/stream_bench.hip -o /tmp/sb && /tmp/sb
// K1 col8    : one row per thread, one 8-B load per column (the fold/update shape)
// K2 col8nt  : K1 with non-temporal loads
// K3 col16nt : two rows per thread, one 16-B load per column, non-temporal
// K4 flat16  : the J columns as one flat array, 16-B loads, 4 in flight per thread
// K5 flat16nt: K4 non-temporal
// K6 glds    : the flat array by LDS-DMA (global_load_lds_dwordx4, nt), a 2-deep
//              per-wave ring of 4 KiB, consumed by ds_read_b128
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double dv2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);            \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int J, bool NT>
__global__ __launch_bounds__(256) void col8(long n, const double* __restrict__ V, long ld,
                                            double* __restrict__ out) {
    double acc[J];
#pragma unroll
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int k = 0; k < J; ++k) {
            const double* p = V + i + (long)k * ld;
            acc[k] += NT ? __builtin_nontemporal_load(p) : *p;
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < J; ++k) s += acc[k];
    if (s == 12345.678) out[blockIdx.x] = s;
}

template <int J>
__global__ __launch_bounds__(256) void col16nt(long n, const double* __restrict__ V, long ld,
                                               double* __restrict__ out) {
    double acc[J];
#pragma unroll
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; 2 * i < n; i += stride) {
#pragma unroll
        for (int k = 0; k < J; ++k) {
            const dv2 v = __builtin_nontemporal_load(
                reinterpret_cast<const dv2*>(V + (long)k * ld) + i);
            acc[k] += v.x + v.y;
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < J; ++k) s += acc[k];
    if (s == 12345.678) out[blockIdx.x] = s;
}

template <bool NT>
__global__ __launch_bounds__(256) void flat16(long n2, const dv2* __restrict__ V,
                                              double* __restrict__ out) {
    double s = 0.0;
    const long stride = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n2; i += 4 * stride) {
        dv2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = NT ? __builtin_nontemporal_load(V + i + u * stride) : V[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u].x + v[u].y;
    }
    for (; i < n2; i += stride) s += V[i].x + V[i].y;
    if (s == 12345.678) out[blockIdx.x] = s;
}

// each wave streams contiguous 4-KiB pieces (64 lanes x 16 B x 4) of the flat
// array into its own 2-slot LDS ring by LDS-DMA, then sums the previous piece
__global__ __launch_bounds__(256) void glds(long npiece, const double2* __restrict__ V,
                                            double* __restrict__ out) {
    __shared__ double2 ring[4][2][4][64];  // [wave][slot][instr][lane]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long gw = (long)blockIdx.x * 4 + w, nw = (long)gridDim.x * 4;
    double s = 0.0;
    int slot = 0;
    long p = gw;
    auto issue = [&](long piece, int sl) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_amdgcn_global_load_lds(
                (const void*)(V + piece * 256 + u * 64 + lane), (void*)&ring[w][sl][u][0], 16, 0, 2);
    };
    if (p < npiece) issue(p, 0);
    for (; p < npiece; p += nw) {
        const long q = p + nw;
        if (q < npiece) {
            issue(q, slot ^ 1);
            __builtin_amdgcn_s_waitcnt((4 & 0xF) | (0x7 << 4) | (0xF << 8));  // vmcnt(4)
        } else {
            __builtin_amdgcn_s_waitcnt((0) | (0x7 << 4) | (0xF << 8));  // vmcnt(0)
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double2 v = ring[w][slot][u][lane];
            s += v.x + v.y;
        }
        slot ^= 1;
    }
    if (s == 12345.678) out[blockIdx.x] = s;
}

// Pass-shaped variants of col8 nt: EX extra n-vectors read (plain), WR
// n-vectors written (WNT: non-temporal stores), MATH: the fold pass's
// arithmetic (r' = r - V s, w = y - V t - c r', J+2 accumulators).
template <int J, int EX, int WR, bool WNT, bool MATH>
__global__ __launch_bounds__(256) void pass(long n, double* __restrict__ V, long ld,
                                            const double* __restrict__ a,
                                            const double* __restrict__ b,
                                            const double* __restrict__ s,
                                            const double* __restrict__ t,
                                            double* __restrict__ o1, double* __restrict__ o2,
                                            double* __restrict__ out) {
    double acc[J + 2];
#pragma unroll
    for (int k = 0; k < J + 2; ++k) acc[k] = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        double v[J];
#pragma unroll
        for (int k = 0; k < J; ++k) v[k] = __builtin_nontemporal_load(V + i + (long)k * ld);
        double x = EX >= 1 ? a[i] : 0.0, y = EX >= 2 ? b[i] : 0.0;
        double w = y;
        if (MATH) {
            double sv = 0.0;
#pragma unroll
            for (int k = 0; k < J; ++k) sv += v[k] * s[k];
            x = x - sv;
            double q = 0.0;
#pragma unroll
            for (int k = 0; k < J; ++k) q = fma(v[k], t[k], q);
            q = fma(s[J - 1], x, q);
            w = y - q;
#pragma unroll
            for (int k = 0; k < J; ++k) acc[k] += v[k] * w;
            acc[J] += x * w;
            acc[J + 1] += w * w;
        } else {
#pragma unroll
            for (int k = 0; k < J; ++k) acc[k] += v[k];
            acc[J] += x + y;
        }
        if (WR >= 1) {
            if (WNT) __builtin_nontemporal_store(x, o1 + i); else o1[i] = x;
        }
        if (WR >= 2) {
            if (WNT) __builtin_nontemporal_store(w, o2 + i); else o2[i] = w;
        }
    }
    double r = 0;
#pragma unroll
    for (int k = 0; k < J + 2; ++k) r += acc[k];
    if (r == 12345.678) out[blockIdx.x] = r;
}

__global__ void fill1(long n, double* x) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        x[i] = 1.0 + 1e-3 * (double)(i & 1023);
}

int main() {
    const long n = 10000000, J = 20, ld = n;
    const size_t bytes = sizeof(double) * (size_t)ld * J;
    double *V, *out, *vec, *coef;
    CK(hipMalloc(&V, bytes));
    CK(hipMalloc(&vec, sizeof(double) * 4 * n));
    CK(hipMalloc(&coef, sizeof(double) * 128));
    CK(hipMalloc(&out, 1 << 20));
    fill1<<<4096, 256>>>((long)ld * J, V);
    fill1<<<4096, 256>>>(4 * n, vec);
    fill1<<<1, 256>>>(128, coef);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    size_t nb = bytes;
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e9, tot = 0;
        const int reps = 10;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            tot += ms;
        }
        printf("%-28s best %.3f ms  %.0f GB/s   mean %.0f GB/s\n", name, best, nb / best / 1e6,
               nb / (tot / reps) / 1e6);
        return 0;
    };
    double *a = vec, *b = vec + n, *o1 = vec + 2 * n, *o2 = vec + 3 * n, *cs = coef, *ct = coef + 64;
    for (int grid : {1024, 2048}) {
        printf("grid %d (non-zero data)\n", grid);
        nb = bytes;
        run("col8 nt J20", [&] { col8<20, true><<<grid, 256>>>(n, V, ld, out); });
        nb = bytes + 16 * n;
        run("pass +2 reads", [&] { pass<20, 2, 0, false, false><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
        nb = bytes + 24 * n;
        run("pass +2r +1w", [&] { pass<20, 2, 1, false, false><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
        run("pass +2r +1w nt", [&] { pass<20, 2, 1, true, false><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
        run("pass fold math +1w", [&] { pass<20, 2, 1, false, true><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
        run("pass fold math +1w nt", [&] { pass<20, 2, 1, true, true><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
        nb = bytes + 32 * n;
        run("pass +2r +2w", [&] { pass<20, 2, 2, false, false><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
        run("pass +2r +2w nt", [&] { pass<20, 2, 2, true, false><<<grid, 256>>>(n, V, ld, a, b, cs, ct, o1, o2, out); });
    }
    nb = bytes;
    for (int grid : {1024}) {
        printf("grid %d\n", grid);
        run("col8 plain", [&] { col8<20, false><<<grid, 256>>>(n, V, ld, out); });
        run("col8 nt", [&] { col8<20, true><<<grid, 256>>>(n, V, ld, out); });
        run("col16 nt", [&] { col16nt<20><<<grid, 256>>>(n, V, ld, out); });
        run("flat16 plain", [&] { flat16<false><<<grid, 256>>>((long)bytes / 16, (dv2*)V, out); });
        run("flat16 nt", [&] { flat16<true><<<grid, 256>>>((long)bytes / 16, (dv2*)V, out); });
        run("glds nt", [&] { glds<<<grid, 256>>>((long)bytes / 4096, (double2*)V, out); });
    }
    return 0;
}
