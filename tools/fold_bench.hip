// Standalone timing of the folded-step passes (fold.hip) at the north-star
// size, against the read-stream ceiling of tools/stream_bench.hip: is a pass
// slower in the solve than alone (cache state left by the SpMV), or alone?
// Findings (r02): back to back, k_fold_dots<20> runs at 6.8-6.9 TB/s (255 us)
// against 285 us inside the solve (after the SpMV, inputs no longer in the
// Infinity Cache); a software-pipelined form (next row's loads first) is 1.5%
// faster back to back but 0.8% slower in the solve (same-box A/B through
// ARPACK_HIP_LIB, 3 runs each), so the library keeps the plain loop.
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -Iarpack-ng_amd/csrc tools/fold_bench.hip \
//         -o tools/fold_bench && tools/fold_bench
#include "../arpack-ng_amd/csrc/fold.hip"

#include <cstdio>

namespace ahip::dev {  // the profiler is not linked: spans are no-ops here
void prof_arm(ProfClass) {}
void prof_disarm(ProfClass, double) {}
bool prof_kernel_events(hipEvent_t*, hipEvent_t*) { return false; }
}  // namespace ahip::dev


// Variant: the next row's loads issued before the current row's arithmetic
// (software pipelining, as k_dots), same arithmetic order per row.
template <class R, int J, int POL = ahip::dev::kPolNt>
__global__ __launch_bounds__(256) void k_fold_dots_pipe(int64_t n, R* __restrict__ V, int64_t ld,
                                                        const R* __restrict__ r,
                                                        const R* __restrict__ y,
                                                        const double* __restrict__ s,
                                                        const double* __restrict__ t,
                                                        double* __restrict__ part, int pstride,
                                                        const ahip::dev::LzState* __restrict__ st) {
    using namespace ahip::dev;
    if (st->abort) return;
    const bool fold = st->fold != 0;
    const double c = fold ? s[J - 1] : 0.0;
    double acc[J + 2];
#pragma unroll
    for (int k = 0; k < J + 2; ++k) acc[k] = 0.0;
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    double cur[J], cr = 0.0, cy = 0.0;
    auto load = [&](int64_t i, double (&dst)[J], double& dr, double& dy) {
#pragma unroll
        for (int k = 0; k < J; ++k) dst[k] = vld<POL>(V + i + (int64_t)k * ld);
        dr = (double)r[i];
        dy = (double)y[i];
    };
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) load(i, cur, cr, cy);
    for (; i < n; i += stride) {
        double nxt[J], nr = 0.0, ny = 0.0;
        if (i + stride < n) load(i + stride, nxt, nr, ny);
        double rp = cr, w = cy;
        if (fold) {
            rp = (double)(R)fold_r<J>(rp, cur, s);
            w = fold_w<J>(w, cur, t, c, rp);
        }
#pragma unroll
        for (int k = 0; k < J; ++k) acc[k] += cur[k] * w;
        acc[J] += rp * w;
        acc[J + 1] += w * w;
        rr += rp * rp;
#pragma unroll
        for (int k = 0; k < J; ++k) cur[k] = nxt[k];
        cr = nr;
        cy = ny;
    }
    block_partials<J + 2>(acc, J + 2, rr, true, part, 0, pstride);
}

// The previous (unpipelined) form of k_fold_dots, for the A/B.
template <class R, int J, int POL = ahip::dev::kPolNt>
__global__ __launch_bounds__(256) void k_fold_dots_plain(int64_t n, R* __restrict__ V, int64_t ld,
                                                         const R* __restrict__ r,
                                                         const R* __restrict__ y,
                                                         const double* __restrict__ s,
                                                         const double* __restrict__ t,
                                                         double* __restrict__ part, int pstride,
                                                         const ahip::dev::LzState* __restrict__ st) {
    using namespace ahip::dev;
    if (st->abort) return;
    const bool fold = st->fold != 0;
    const double c = fold ? s[J - 1] : 0.0;
    double acc[J + 2];
#pragma unroll
    for (int k = 0; k < J + 2; ++k) acc[k] = 0.0;
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        double vrow[J];
#pragma unroll
        for (int k = 0; k < J; ++k) vrow[k] = vld<POL>(V + i + (int64_t)k * ld);
        double rp = (double)r[i], w = (double)y[i];
        if (fold) {
            rp = (double)(R)fold_r<J>(rp, vrow, s);
            w = fold_w<J>(w, vrow, t, c, rp);
        }
#pragma unroll
        for (int k = 0; k < J; ++k) acc[k] += vrow[k] * w;
        acc[J] += rp * w;
        acc[J + 1] += w * w;
        rr += rp * rp;
    }
    block_partials<J + 2>(acc, J + 2, rr, true, part, 0, pstride);
}

__global__ void fill(long n, double* x, double a) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        x[i] = a * (1.0 + 1e-3 * (double)(i & 1023));
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);           \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main() {
    using namespace ahip::dev;
    const long n = 10000000;
    const int ncv = 30;
    double *V, *r, *y, *x2, *junk;
    CK(hipMalloc(&V, sizeof(double) * n * ncv));
    CK(hipMalloc(&r, sizeof(double) * n));
    CK(hipMalloc(&y, sizeof(double) * n));
    CK(hipMalloc(&x2, sizeof(double) * n));
    const size_t junkn = 400000000;  // 3.2 GB: evicts the Infinity Cache between reps
    CK(hipMalloc(&junk, sizeof(double) * junkn));
    fill<<<4096, 256>>>(n * ncv, V, 0.01);
    fill<<<4096, 256>>>(n, r, 1.0);
    fill<<<4096, 256>>>(n, y, 2.0);
    Workspace ws;
    ws.stream = nullptr;
    ws.nblk = 1024;
    ws.stride = ncv + 2;
    CK(hipMalloc(&ws.part, sizeof(double) * 2 * ws.nblk * ws.stride));
    CK(hipMalloc(&ws.coef, sizeof(double) * 4 * ws.stride));
    fill<<<1, 256>>>(4 * ws.stride, ws.coef, 1e-3);
    CK(hipMalloc(&ws.st, sizeof(LzState)));
    LzState h{};
    h.rnorm = 1.0;
    h.vscale = 1.0;
    h.fold = 1;
    CK(hipMemcpy(ws.st, &h, sizeof h, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // each kernel timed back to back (10 launches), the same cache state for all
    auto timeit = [&](auto launch) {
        launch();
        (void)hipDeviceSynchronize();
        float ms = 0;
        (void)hipEventRecord(e0);
        for (int rep = 0; rep < 10; ++rep) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 10;
    };
    for (int j : {11, 21, 30}) {
        const double bd = 8.0 * n * (j + 1), bu = 8.0 * n * (j + 3);
        const float td = timeit([&] { fold_dots<double>(ws, n, j, V, n, r, y); });
        const float tu = timeit([&] { fold_update<double>(ws, n, j, V, n, y, r, nullptr); });
        printf("j=%2d  fold_dots %.1f us %.0f GB/s   fold_update %.1f us %.0f GB/s\n", j, td * 1e3,
               bd / td / 1e6, tu * 1e3, bu / tu / 1e6);
        if (j == 21) {
            const float tp = timeit([&] {
                k_fold_dots_pipe<double, 20><<<1024, 256>>>(n, V, n, r, y, ws.coef + ws.stride,
                                                          ws.coef + 3 * ws.stride, ws.part,
                                                          ws.stride, ws.st);
            });
            printf("j=21  fold_dots variant (tools copy) %.1f us %.0f GB/s\n", tp * 1e3, bd / tp / 1e6);
            const float tq = timeit([&] {
                k_fold_dots_plain<double, 20><<<1024, 256>>>(n, V, n, r, y, ws.coef + ws.stride,
                                                           ws.coef + 3 * ws.stride, ws.part,
                                                           ws.stride, ws.st);
            });
            printf("j=21  fold_dots unpipelined (previous form) %.1f us %.0f GB/s\n", tq * 1e3, bd / tq / 1e6);
        }
    }
    return 0;
}
