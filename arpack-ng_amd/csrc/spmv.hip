// CSR SpMV y = A x — the user OP of the `ido = +-1` requests, served on device.
//
// HBM-bound (0.17 flop/byte): the job is to stream val (8 B/nnz) and col
// (4 B/nnz) once at full bandwidth while x is re-read from L2 (for banded
// operators every x window is shared by ~50 neighbouring rows).
//
//  k_csr_stream  (default) CSR-stream: one 256-thread workgroup owns a row
//                block whose nonzeros (<= TILE) it streams with fully
//                coalesced loads, every lane issuing all TILE/256 val/col loads
//                before the first x gather (deep memory-level parallelism);
//                products go to LDS and each row is reduced by a power-of-two
//                lane group with wave shuffles.  NT=true marks val/col as
//                non-temporal so they do not evict x from L2.
//  k_csr_vector  G lanes per row (fallback for rows longer than TILE).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <vector>

#include "device.hpp"
#include "finalize.hpp"

namespace ahip::dev {

namespace {

// a plan-table HIP call succeeded (the fault-injection hook sees every one)
inline bool hok(hipError_t e) { return fault_filter(e) == hipSuccess; }

template <int G>
__global__ __launch_bounds__(kBlock) void k_csr_vector(int64_t n, const int64_t* __restrict__ rp,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val,
                                                       const double* __restrict__ x,
                                                       double* __restrict__ y) {
    const int lane = threadIdx.x % G;
    const int64_t rows_per_block = kBlock / G;
    const int64_t stride = (int64_t)gridDim.x * rows_per_block;
    for (int64_t row = (int64_t)blockIdx.x * rows_per_block + threadIdx.x / G; row < n;
         row += stride) {
        const int64_t b = rp[row], e = rp[row + 1];
        double s = 0.0;
        for (int64_t k = b + lane; k < e; k += G) s += val[k] * x[col[k]];
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, G);
        if (lane == 0) y[row] = s;
    }
}

template <class T, bool NT>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int TILE, bool NT>
__global__ __launch_bounds__(kBlock) void k_csr_stream(const int64_t* __restrict__ rblk,
                                                       const int64_t* __restrict__ rp,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val,
                                                       const double* __restrict__ x,
                                                       double* __restrict__ y) {
    constexpr int PER = TILE / kBlock;
    __shared__ double prod[TILE];
    const int t = threadIdx.x;
    const int64_t r0 = rblk[blockIdx.x], r1 = rblk[blockIdx.x + 1];
    const int64_t k0 = rp[r0];
    const int cnt = (int)(rp[r1] - k0);
    const int last = cnt > 0 ? cnt - 1 : 0;
    // 1) issue every val/col load of this lane first (clamped, branch-free)
    double v[PER];
    int c[PER];
    if (cnt > 0) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = min(t + u * kBlock, last);
            v[u] = ld<double, NT>(val + k0 + k);
            c[u] = ld<int32_t, NT>(col + k0 + k);
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) { v[u] = 0.0; c[u] = 0; }
    }
    // 2) gather x and park the products in LDS
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int k = t + u * kBlock;
        const double p = v[u] * x[c[u]];
        if (k < cnt) prod[k] = p;
    }
    __syncthreads();
    // 3) per-row reduction: L lanes per row (power of two, same wave)
    const int nrows = (int)(r1 - r0);
    if (nrows <= kBlock) {
        int L = 1;
        while (L * 2 * nrows <= kBlock && L < 64) L *= 2;
        const int row = t / L, sub = t % L;
        double s = 0.0;
        int b = 0, e = 0;
        if (row < nrows) {
            b = (int)(rp[r0 + row] - k0);
            e = (int)(rp[r0 + row + 1] - k0);
            for (int k = b + sub; k < e; k += L) s += prod[k];
        }
        for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        if (row < nrows && sub == 0) y[r0 + row] = s;
    } else {
        for (int row = t; row < nrows; row += kBlock) {
            const int b = (int)(rp[r0 + row] - k0), e = (int)(rp[r0 + row + 1] - k0);
            double s = 0.0;
            for (int k = b; k < e; ++k) s += prod[k];
            y[r0 + row] = s;
        }
    }
}

// Window kernel: one 1024-thread workgroup owns a SUPERBLOCK of rows whose
// column span fits the LDS x-window.  It loads x[c0, c0+span) into LDS once
// (coalesced), then streams the superblock's nonzeros tile by tile: val/col of
// tile t+1 are issued before the rows of tile t are reduced, x is gathered from
// LDS (no L2 gather traffic: for banded operators the per-nonzero gathers, not
// the val/col stream, otherwise saturate the L2).
constexpr int kWinThreads = 1024;
constexpr int kWinTile = 8192;   // nonzeros per tile (8 per lane)
constexpr int kWinX = 10240;     // doubles of x per window (80 KB)

template <bool NT>
__global__ __launch_bounds__(kWinThreads) void k_csr_window(
    const int64_t* __restrict__ sb_tile0, const int64_t* __restrict__ tiles,
    const int64_t* __restrict__ sb_c0, const int32_t* __restrict__ sb_span,
    const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ x, double* __restrict__ y) {
    constexpr int PER = kWinTile / kWinThreads;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xw = lds;             // kWinX
    double* prod = lds + kWinX;   // kWinTile
    const int t = threadIdx.x;
    const int64_t c0 = sb_c0[blockIdx.x];
    const int span = sb_span[blockIdx.x];
    const int64_t tb = sb_tile0[blockIdx.x], te = sb_tile0[blockIdx.x + 1];

    // One tile in registers: its val/col slice and this lane's reduction row.
    struct Buf {
        double v[PER];
        int c[PER];
        int cnt, nrows, L, rb, re;
        int64_t r0, k0;
    };
    auto issue = [&](int64_t tile, Buf& B) {
        B.r0 = tiles[tile];
        const int64_t r1 = tiles[tile + 1];
        B.k0 = rp[B.r0];
        B.cnt = (int)(rp[r1] - B.k0);
        B.nrows = (int)(r1 - B.r0);
        if (B.cnt == 0) {
#pragma unroll
            for (int u = 0; u < PER; ++u) { B.v[u] = 0.0; B.c[u] = (int)c0; }
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int k = min(t + u * kWinThreads, B.cnt - 1);
                B.v[u] = ld<double, NT>(val + B.k0 + k);
                B.c[u] = ld<int32_t, NT>(col + B.k0 + k);
            }
        }
        int L = 1;
        while (L * 2 * B.nrows <= kWinThreads && L < 64) L *= 2;
        B.L = L;
        const int row = t / L;
        B.rb = B.re = 0;
        if (B.nrows <= kWinThreads && row < B.nrows) {  // prefetch the row bounds
            B.rb = (int)(rp[B.r0 + row] - B.k0);
            B.re = (int)(rp[B.r0 + row + 1] - B.k0);
        }
    };
    auto step = [&](int64_t tile, Buf& B) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = t + u * kWinThreads;
            const double p = B.v[u] * xw[B.c[u] - c0];
            if (k < B.cnt) prod[k] = p;
        }
        const int nrows = B.nrows, L = B.L, rb = B.rb, re = B.re;
        const int64_t r0 = B.r0, k0 = B.k0;
        if (tile + 2 < te) issue(tile + 2, B);  // two tiles stay in flight
        __syncthreads();
        if (nrows <= kWinThreads) {
            const int row = t / L, sub = t % L;
            double s = 0.0;
            for (int k = rb + sub; k < re; k += L) s += prod[k];
            for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
            if (row < nrows && sub == 0) y[r0 + row] = s;
        } else {
            for (int row = t; row < nrows; row += kWinThreads) {
                const int b = (int)(rp[r0 + row] - k0), e = (int)(rp[r0 + row + 1] - k0);
                double s = 0.0;
                for (int k = b; k < e; ++k) s += prod[k];
                y[r0 + row] = s;
            }
        }
        __syncthreads();  // prod is reused by the next tile
    };
    Buf A, B;
    issue(tb, A);
    if (tb + 1 < te) issue(tb + 1, B);
    for (int i = t; i < span; i += kWinThreads) xw[i] = x[c0 + i];
    __syncthreads();  // x window ready
    for (int64_t tile = tb; tile < te; tile += 2) {
        step(tile, A);
        if (tile + 1 < te) step(tile + 1, B);
    }
}

// Window-vector kernel: same LDS x-window superblocks, but rows are reduced
// straight from registers — L lanes per row, each lane holding U of the row's
// nonzeros — so there is no product buffer and no barrier after the window
// load (LDS = the window only: two workgroups per CU).  Rows of the next pass
// are loaded before the current pass is reduced (two passes in flight).
// CW: read the 16-bit window-relative column indices (colw = col - c0 of the
// superblock, built by the analysis) instead of int32 col: 10 instead of 12
// bytes per nonzero.
// XCD-aware superblock order (xcd_block, device.hpp): consecutive superblocks
// (whose x windows overlap by ~80%) would otherwise land on different XCDs and
// fetch their windows from HBM eight times over.

template <int L, int U, bool NT, bool CW, bool XCD = false>
__global__ __launch_bounds__(kWinThreads) void k_csr_wvec(
    const int64_t* __restrict__ sb_tile0, const int64_t* __restrict__ tiles,
    const int64_t* __restrict__ sb_c0, const int32_t* __restrict__ sb_span,
    const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
    const uint16_t* __restrict__ colw, const double* __restrict__ val,
    const double* __restrict__ x, double* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xw = lds;
    constexpr int RPP = kWinThreads / L;  // rows per pass
    const int t = threadIdx.x, sub = t % L;
    const int64_t sb = XCD ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t c0 = sb_c0[sb];
    const int span = sb_span[sb];
    const int64_t R0 = tiles[sb_tile0[sb]], R1 = tiles[sb_tile0[sb + 1]];
    const int64_t npass = (R1 - R0 + RPP - 1) / RPP;
    // Pipeline: row bounds are loaded two passes ahead of the val/col loads,
    // which run two passes ahead of the reduction.
    struct Bounds {
        int64_t b, e;
    };
    struct Buf {
        double v[U];
        int c[U];
        int64_t row, b, e;
    };
    auto bounds = [&](int64_t pass) {
        Bounds r{0, 0};
        const int64_t row = R0 + pass * RPP + t / L;
        if (pass < npass && row < R1) {
            r.b = rp[row];
            r.e = rp[row + 1];
        }
        return r;
    };
    auto issue = [&](int64_t pass, const Bounds& bd, Buf& B) {
        B.row = R0 + pass * RPP + t / L;
        B.b = bd.b;
        B.e = bd.e;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = B.b + sub + u * L;
            const bool in = k < B.e;
            B.v[u] = in ? ld<double, NT>(val + k) : 0.0;
            if constexpr (CW) B.c[u] = in ? (int)ld<uint16_t, NT>(colw + k) : 0;
            else B.c[u] = in ? ld<int32_t, NT>(col + k) - (int)c0 : 0;
        }
    };
    auto finish = [&](Buf& B) {
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) s += B.v[u] * xw[B.c[u]];
        for (int64_t k = B.b + sub + U * L; k < B.e; k += L) s += val[k] * xw[col[k] - c0];
#pragma unroll
        for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        if (B.row < R1 && sub == 0) y[B.row] = s;
    };
    Buf A, B;
    issue(0, bounds(0), A);
    issue(1, bounds(1), B);
    Bounds nA = bounds(2), nB = bounds(3);
    for (int i = t; i < span; i += kWinThreads) xw[i] = x[c0 + i];
    __syncthreads();
    for (int64_t p = 0; p < npass; p += 2) {
        finish(A);
        if (p + 2 < npass) {
            issue(p + 2, nA, A);
            nA = bounds(p + 4);
        }
        if (p + 1 < npass) {
            finish(B);
            if (p + 3 < npass) {
                issue(p + 3, nB, B);
                nB = bounds(p + 5);
            }
        }
    }
}

// Same kernel with P row passes in flight (P = 2 is k_csr_wvec's schedule):
// more outstanding loads per wave to cover HBM latency.
template <int L, int U, int P, bool XCD>
__global__ __launch_bounds__(kWinThreads) void k_csr_wvecp(
    const int64_t* __restrict__ sb_tile0, const int64_t* __restrict__ tiles,
    const int64_t* __restrict__ sb_c0, const int32_t* __restrict__ sb_span,
    const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
    const uint16_t* __restrict__ colw, const double* __restrict__ val,
    const double* __restrict__ x, double* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xw = lds;
    constexpr int RPP = kWinThreads / L;
    const int t = threadIdx.x, sub = t % L;
    const int64_t sb = XCD ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t c0 = sb_c0[sb];
    const int span = sb_span[sb];
    const int64_t R0 = tiles[sb_tile0[sb]], R1 = tiles[sb_tile0[sb + 1]];
    const int64_t npass = (R1 - R0 + RPP - 1) / RPP;
    struct Buf {
        double v[U];
        int c[U];
        int64_t row, b, e;
    };
    auto issue = [&](int64_t pass, Buf& B) {
        B.row = R0 + pass * RPP + t / L;
        B.b = 0;
        B.e = 0;
        if (pass < npass && B.row < R1) {
            B.b = rp[B.row];
            B.e = rp[B.row + 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = B.b + sub + u * L;
            const bool in = k < B.e;
            B.v[u] = in ? val[k] : 0.0;
            B.c[u] = in ? (int)colw[k] : 0;
        }
    };
    auto finish = [&](Buf& B) {
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) s += B.v[u] * xw[B.c[u]];
        for (int64_t k = B.b + sub + U * L; k < B.e; k += L) s += val[k] * xw[col[k] - c0];
#pragma unroll
        for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        if (B.row < R1 && sub == 0) y[B.row] = s;
    };
    Buf buf[P];
#pragma unroll
    for (int q = 0; q < P; ++q) issue(q, buf[q]);
    for (int i = t; i < span; i += kWinThreads) xw[i] = x[c0 + i];
    __syncthreads();
    for (int64_t p = 0; p < npass; p += P) {
#pragma unroll
        for (int q = 0; q < P; ++q) {
            if (p + q < npass) {
                finish(buf[q]);
                if (p + q + P < npass) issue(p + q + P, buf[q]);
            }
        }
    }
}

// SELL-64 over the LDS x window: one workgroup per superblock, each wave takes
// whole slices (lane = row); a column step is one coalesced 512-B val load and
// one 128-B colw load per wave.  Each row is summed sequentially in its CSR
// (column) order.  FIN (1, or 2 with the Arnoldi H staging): the step's
// deferred finalize (kernels.hip finalize(..., defer)) runs in workgroup 0
// after its rows, over the spent x window -- it reads the partial sums of the
// pass before the SpMV and writes the state the pass after it reads, so the
// launch it saves costs no ordering.  (k_csr_sell_fin below: its own kernel,
// held to 64 VGPRs so two workgroups still share a CU.)
template <int U, bool XCD, bool NTL, bool MR, int FIN>
__device__ __forceinline__ void csr_sell_body(
    const int64_t* __restrict__ sb_slice0, const int64_t* __restrict__ sptr,
    const int32_t* __restrict__ srow, const int64_t* __restrict__ sb_c0,
    const int32_t* __restrict__ sb_span, const uint16_t* __restrict__ scolw,
    const double* __restrict__ sval, const double* __restrict__ x, double* __restrict__ y,
    const int64_t* __restrict__ rng, const FinArgs& fa) {
    // unfused multiply-add: each row is summed exactly as a sequential CSR loop
    // (y_i = ((0 + a_i1 x_1) + a_i2 x_2) + ...) -- SciPy's csr_matvec, the OP
    // the reference's RCI callers use -- so y is bitwise the CPU result
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xw = lds;
    constexpr int NW = kWinThreads / 64;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t sb = XCD ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t c0 = sb_c0[sb];
    const int span = sb_span[sb];
    const int64_t s0 = sb_slice0[sb], s1 = sb_slice0[sb + 1];
    // double-buffered column steps: chunk k+U (or the next slice's first chunk)
    // is in flight while chunk k is consumed; the first chunk is issued before
    // the x window is staged so the HBM stream starts with the x loads
    struct Chunk {
        double v[U];
        int c[U];
    };
    auto load = [&](Chunk& ch, int64_t base, int w, int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k0 + u < w;
            ch.v[u] = in ? ld<double, NTL>(sval + base + (int64_t)(k0 + u) * 64 + lane) : 0.0;
            ch.c[u] = in ? (int)ld<uint16_t, NTL>(scolw + base + (int64_t)(k0 + u) * 64 + lane) : 0;
        }
    };
    int64_t s = s0 + wave;
    int64_t base = 0;
    int w = 0;
    Chunk cur, nxt;
    if (s < s1) {
        base = sptr[s];
        w = (int)((sptr[s + 1] - base) >> 6);
        load(cur, base, w, 0);
    }
    if constexpr (MR) {  // the superblock's column bands, back to back in LDS
#pragma unroll
        for (int r = 0; r < kMaxRanges; ++r) {
            const int64_t a = rng[8 * sb + r], ol = rng[8 * sb + 4 + r];
            const int off = (int)(ol >> 32), len = (int)(ol & 0xffffffff);
            for (int i = t; i < len; i += kWinThreads) xw[off + i] = x[a + i];
        }
    } else {
        for (int i = t; i < span; i += kWinThreads) xw[i] = x[c0 + i];
    }
    __syncthreads();
    for (; s < s1; s += NW) {
        const int row = srow[s * 64 + lane];
        const int64_t sn = s + NW;
        int64_t nbase = 0;
        int nw = 0;
        if (sn < s1) {
            nbase = sptr[sn];
            nw = (int)((sptr[sn + 1] - nbase) >> 6);
        }
        double acc = 0.0;
        int k = 0;
        do {
            if (k + U < w) load(nxt, base, w, k + U);
            else if (sn < s1) load(nxt, nbase, nw, 0);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += cur.v[u] * xw[cur.c[u]];
            cur = nxt;
            k += U;
        } while (k < w);
        if (row >= 0) y[row] = acc;
        base = nbase;
        w = nw;
    }
    if constexpr (FIN > 0) {
        if (blockIdx.x == 0) {
            __syncthreads();  // every wave is done with the x window
            finalize_block<FIN == 2>(fa, reinterpret_cast<FinLds*>(lds), lds + kWinX - kFoldHMax * kFoldHMax);
        }
    }
}

template <int U, bool XCD, bool NTL = false, bool MR = false>
__global__ __launch_bounds__(kWinThreads) void k_csr_sell(
    const int64_t* __restrict__ sb_slice0, const int64_t* __restrict__ sptr,
    const int32_t* __restrict__ srow, const int64_t* __restrict__ sb_c0,
    const int32_t* __restrict__ sb_span, const uint16_t* __restrict__ scolw,
    const double* __restrict__ sval, const double* __restrict__ x, double* __restrict__ y,
    const int64_t* __restrict__ rng) {
    csr_sell_body<U, XCD, NTL, MR, 0>(sb_slice0, sptr, srow, sb_c0, sb_span, scolw, sval, x, y, rng,
                                      FinArgs{});
}

// The default form (U = 4, XCD order, non-temporal val/col) carrying a deferred
// finalize.  waves_per_eu(8): the finalize's code must not raise the kernel's
// VGPRs past 64, or one workgroup a CU would fit instead of two.
template <bool MR, int FIN>
__global__ __launch_bounds__(kWinThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_csr_sell_fin(
    const int64_t* __restrict__ sb_slice0, const int64_t* __restrict__ sptr,
    const int32_t* __restrict__ srow, const int64_t* __restrict__ sb_c0,
    const int32_t* __restrict__ sb_span, const uint16_t* __restrict__ scolw,
    const double* __restrict__ sval, const double* __restrict__ x, double* __restrict__ y,
    const int64_t* __restrict__ rng, FinArgs fa) {
    csr_sell_body<4, true, true, MR, FIN>(sb_slice0, sptr, srow, sb_c0, sb_span, scolw, sval, x, y,
                                          rng, fa);
}

// Two slices per wave at once (s and s + NW): twice the independent column
// streams per wave, each double-buffered.
template <int U, bool XCD>
__global__ __launch_bounds__(kWinThreads) void k_csr_sell2(
    const int64_t* __restrict__ sb_slice0, const int64_t* __restrict__ sptr,
    const int32_t* __restrict__ srow, const int64_t* __restrict__ sb_c0,
    const int32_t* __restrict__ sb_span, const uint16_t* __restrict__ scolw,
    const double* __restrict__ sval, const double* __restrict__ x, double* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xw = lds;
    constexpr int NW = kWinThreads / 64;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t sb = XCD ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t c0 = sb_c0[sb];
    const int span = sb_span[sb];
    const int64_t s0 = sb_slice0[sb], s1 = sb_slice0[sb + 1];
    struct Chunk {
        double v[U];
        int c[U];
    };
    auto load = [&](Chunk& ch, int64_t base, int w, int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k0 + u < w;
            ch.v[u] = in ? sval[base + (int64_t)(k0 + u) * 64 + lane] : 0.0;
            ch.c[u] = in ? (int)scolw[base + (int64_t)(k0 + u) * 64 + lane] : 0;
        }
    };
    auto geom = [&](int64_t sl, int64_t& base, int& w) {
        base = 0;
        w = 0;
        if (sl < s1) {
            base = sptr[sl];
            w = (int)((sptr[sl + 1] - base) >> 6);
        }
    };
    int64_t s = s0 + wave;
    int64_t ba, bb;
    int wa, wb;
    geom(s, ba, wa);
    geom(s + NW, bb, wb);
    Chunk ca, cb, na, nb;
    load(ca, ba, wa, 0);
    load(cb, bb, wb, 0);
    for (int i = t; i < span; i += kWinThreads) xw[i] = x[c0 + i];
    __syncthreads();
    for (; s < s1; s += 2 * NW) {
        const int ra = srow[s * 64 + lane];
        const int rb = s + NW < s1 ? srow[(s + NW) * 64 + lane] : -1;
        int64_t nba, nbb;
        int nwa, nwb;
        geom(s + 2 * NW, nba, nwa);
        geom(s + 3 * NW, nbb, nwb);
        double acc_a = 0.0, acc_b = 0.0;
        const int w = wa > wb ? wa : wb;
        int k = 0;
        do {
            const bool last = k + U >= w;
            if (k + U < wa) load(na, ba, wa, k + U);
            else if (last) load(na, nba, nwa, 0);
            if (k + U < wb) load(nb, bb, wb, k + U);
            else if (last) load(nb, nbb, nwb, 0);
            if (k < wa) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc_a += ca.v[u] * xw[ca.c[u]];
            }
            if (k < wb) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc_b += cb.v[u] * xw[cb.c[u]];
            }
            if (k + U < wa) ca = na;
            if (k + U < wb) cb = nb;
            k += U;
        } while (k < w);
        // the chunks left in na / nb are the next pair's first chunks
        ca = na;
        cb = nb;
        if (ra >= 0) y[ra] = acc_a;
        if (rb >= 0) y[rb] = acc_b;
        ba = nba;
        wa = nwa;
        bb = nbb;
        wb = nwb;
    }
}

// fill the SELL arrays: one 64-thread block per slice, lane = row of the slice
__global__ void k_sell_fill(const int64_t* __restrict__ sptr, const int32_t* __restrict__ srow,
                            const int64_t* __restrict__ rp, const uint16_t* __restrict__ colw,
                            const double* __restrict__ val, uint16_t* __restrict__ scolw,
                            double* __restrict__ sval) {
    const int64_t s = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t base = sptr[s];
    const int w = (int)((sptr[s + 1] - base) >> 6);
    const int row = srow[s * 64 + lane];
    const int64_t b = row >= 0 ? rp[row] : 0, len = row >= 0 ? rp[row + 1] - rp[row] : 0;
    for (int k = 0; k < w; ++k) {
        const bool in = k < len;
        sval[base + (int64_t)k * 64 + lane] = in ? val[b + k] : 0.0;
        scolw[base + (int64_t)k * 64 + lane] = in ? colw[b + k] : (uint16_t)0;
    }
}

__global__ void k_colw(const int64_t* __restrict__ sb_tile0, const int64_t* __restrict__ tiles,
                       const int64_t* __restrict__ sb_c0, const int64_t* __restrict__ rp,
                       const int32_t* __restrict__ col, uint16_t* __restrict__ colw) {
    const int64_t c0 = sb_c0[blockIdx.x];
    const int64_t k0 = rp[tiles[sb_tile0[blockIdx.x]]], k1 = rp[tiles[sb_tile0[blockIdx.x + 1]]];
    for (int64_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) colw[k] = (uint16_t)(col[k] - c0);
}

// per-row [min col, max col] (rows may be unsorted); empty rows -> [INT_MAX, -1]
__global__ void k_row_span(int64_t n, const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                           int32_t* __restrict__ mn, int32_t* __restrict__ mx) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int32_t a = 0x7fffffff, b = -1;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            a = min(a, col[k]);
            b = max(b, col[k]);
        }
        mn[i] = a;
        mx[i] = b;
    }
}

// Superblock height cap: at least two workgroups per CU (the SELL kernel's
// 80 KB x window lets two share a CU's LDS).  Without it a wide-band operator
// of ~10^6 rows (a 2-D stencil with m = 1000: 8,240 rows per 10,240-column
// window) gives ~120 superblocks -- half the CUs idle.  Capped superblocks
// stage more x (R + band per R rows) but fill the chip.
static int cu_count() {
    static const int ncu = [] {
        int v = 0;
        return hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0) == hipSuccess && v > 0
                   ? v
                   : 256;
    }();
    return ncu;
}

int64_t sb_row_cap(int64_t n) {
    const int ncu = cu_count();
    const int64_t cap = (n + 2 * (int64_t)ncu - 1) / (2 * (int64_t)ncu);
    return cap < 1024 ? 1024 : cap;
}

// Row caps of the superblocks when the cap binds: superblock 0 -- workgroup 0,
// which carries the step's deferred finalize after its rows (k_csr_sell_fin)
// -- gets half the cap, and the others share the remaining rows in the same
// number of superblocks, so the finalize runs while the other workgroups
// still stream instead of as a serial tail on an idle chip (one round of
// workgroups: 2 a CU); cap0 / cap_rest.
static void sb_row_caps(int64_t n, int64_t& cap0, int64_t& rest) {
    const int64_t rcap = sb_row_cap(n);
    const int64_t slots = 2 * (int64_t)cu_count();
    if (!light_first_sb()) {  // AHIP_LIGHT_SB=0: every superblock at the cap
        cap0 = rest = rcap;
        return;
    }
    // an eighth of the cap (AHIP_LIGHT_SB=1: half, 4: a quarter; A/B): the
    // finalize -- the Arnoldi one with its H staging most -- then ends inside
    // the other workgroups' stream.  Configs 2 / 3, same box
    // (profiles/r06ak_light_sb8_ab.txt): SpMV 14.8 -> 14.2-14.5 / 18.0-18.3 ->
    // 17.2-18.2 µs, cycles/s +0.8%; the rows' results do not depend on it.
    static const int div = [] {
        const char* e = getenv("AHIP_LIGHT_SB");
        return e && e[0] == '4' ? 4 : e && e[0] == '1' ? 2 : 8;
    }();
    cap0 = rcap / div > 128 ? rcap / div : rcap;
    rest = (n - cap0 + slots - 2) / (slots - 1);
    if (rest < rcap) rest = rcap;  // small n: the 1,024-row floor (fewer superblocks than slots)
    if (rest < cap0) rest = cap0;
}

// per row up to kMaxRanges column bands: sorted columns split where two
// consecutive ones are more than kBandGap apart; cnt = -1 if the row's columns
// are unsorted or form more bands
constexpr int kBandGap = 1024;
__global__ void k_row_bands(int64_t n, const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                            int32_t* __restrict__ lo, int32_t* __restrict__ hi, int8_t* __restrict__ cnt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int c = 0;
        int32_t prev = 0;
        bool ok = true;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            const int32_t j = col[k];
            if (c == 0 || j > prev + kBandGap) {
                if (c == kMaxRanges || (c > 0 && j < prev)) {
                    ok = false;
                    break;
                }
                lo[i * kMaxRanges + c] = j;
                ++c;
            } else if (j < prev) {
                ok = false;
                break;
            }
            hi[i * kMaxRanges + c - 1] = j;
            prev = j;
        }
        cnt[i] = ok ? (int8_t)c : (int8_t)-1;
    }
}

// 16-bit LDS slot of every nonzero of superblock blockIdx.x (range lookup)
__global__ void k_colw_ranges(const int64_t* __restrict__ sb_tile0, const int64_t* __restrict__ tiles,
                              const int64_t* __restrict__ rng, const int64_t* __restrict__ rp,
                              const int32_t* __restrict__ col, uint16_t* __restrict__ colw) {
    const int64_t sb = blockIdx.x;
    const int64_t k0 = rp[tiles[sb_tile0[sb]]], k1 = rp[tiles[sb_tile0[sb + 1]]];
    int64_t a[kMaxRanges];
    int off[kMaxRanges], len[kMaxRanges];
#pragma unroll
    for (int r = 0; r < kMaxRanges; ++r) {
        a[r] = rng[8 * sb + r];
        off[r] = (int)(rng[8 * sb + 4 + r] >> 32);
        len[r] = (int)(rng[8 * sb + 4 + r] & 0xffffffff);
    }
    for (int64_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) {
        const int64_t c = col[k];
        int slot = 0;
#pragma unroll
        for (int r = 0; r < kMaxRanges; ++r)
            if (c >= a[r] && c < a[r] + len[r]) slot = off[r] + (int)(c - a[r]);
        colw[k] = (uint16_t)slot;
    }
}

}  // namespace

// AHIP_LIGHT_SB=0: no lighter first superblock (A/B of the finalize-carrying
// workgroup's load; read once)
bool light_first_sb() {
    static const bool on = [] {
        const char* e = getenv("AHIP_LIGHT_SB");
        return !(e && e[0] == '0');
    }();
    return on;
}
bool light_sb_chain() {
    static const bool on = [] {
        const char* e = getenv("AHIP_LIGHT_SB");
        return e && e[0] == '2';
    }();
    return on;
}

int csr_analyse_ranges(Csr& A, int64_t ncols, void** owned) {
    const int64_t n = A.n;
    if (n <= 0 || A.nnz <= 0) return -1;
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> lo((size_t)n * kMaxRanges), hi((size_t)n * kMaxRanges);
    std::vector<int8_t> cnt(n);
    int32_t *dlo = nullptr, *dhi = nullptr;
    int8_t* dcnt = nullptr;
    auto cleanup = [&]() {
        for (void* q : {(void*)dlo, (void*)dhi, (void*)dcnt})
            if (q) (void)hipFree(q);
    };
    const size_t bb = sizeof(int32_t) * (size_t)n * kMaxRanges;
    if (!hok(hipMalloc(&dlo, bb)) || !hok(hipMalloc(&dhi, bb)) || !hok(hipMalloc(&dcnt, (size_t)n))) {
        cleanup();
        return -2;
    }
    int64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    AHIP_LAUNCH(k_row_bands, dim3((unsigned)g), dim3(256), 0, nullptr, n, A.rowptr, A.col, dlo, dhi, dcnt);
    const bool ok = hok(hipMemcpy(lo.data(), dlo, bb, hipMemcpyDeviceToHost)) &&
                    hok(hipMemcpy(hi.data(), dhi, bb, hipMemcpyDeviceToHost)) &&
                    hok(hipMemcpy(cnt.data(), dcnt, (size_t)n, hipMemcpyDeviceToHost)) &&
                    hok(hipMemcpy(rp.data(), A.rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost));
    cleanup();
    if (!ok) return -2;
    // greedy superblocks: the union of their rows' bands, merged when they
    // overlap or touch (gap <= kBandGap), must stay within kMaxRanges bands of
    // kWinX columns in total; tiles (<= kWinTile nonzeros) as in csr_analyse_window
    struct Band {
        int64_t a, b;  // [a, b]
    };
    std::vector<Band> cur, nxt;
    auto merge_into = [](std::vector<Band>& S, const Band& x) {
        S.push_back(x);
        std::sort(S.begin(), S.end(), [](const Band& p, const Band& q) { return p.a < q.a; });
        std::vector<Band> m;
        for (const Band& q : S) {
            if (!m.empty() && q.a <= m.back().b + kBandGap) m.back().b = std::max(m.back().b, q.b);
            else m.push_back(q);
        }
        S.swap(m);
    };
    auto fits = [](const std::vector<Band>& S) {
        int64_t len = 0;
        for (const Band& q : S) len += q.b - q.a + 1;
        return (int)S.size() <= kMaxRanges && len <= kWinX;
    };
    std::vector<int64_t> tiles{0}, sb_tile0{0}, sb_c0, rng;
    std::vector<int32_t> sb_span;
    auto close_sb = [&]() {
        int64_t off = 0, a0 = cur.empty() ? 0 : cur[0].a;
        for (int r = 0; r < kMaxRanges; ++r) rng.push_back(r < (int)cur.size() ? cur[r].a : 0);
        for (int r = 0; r < kMaxRanges; ++r) {
            const int64_t len = r < (int)cur.size() ? cur[r].b - cur[r].a + 1 : 0;
            rng.push_back((off << 32) | len);
            off += len;
        }
        sb_c0.push_back(a0);
        sb_span.push_back((int32_t)off);
        sb_tile0.push_back((int64_t)tiles.size() - 1);
    };
    int64_t sb_start = 0, tile_start = 0;
    int64_t cap0 = 0, cap_rest = 0;
    sb_row_caps(n, cap0, cap_rest);
    for (int64_t i = 0; i < n; ++i) {
        if (cnt[i] < 0 || rp[i + 1] - rp[i] > kWinTile) return -1;
        nxt = cur;
        for (int c = 0; c < cnt[i]; ++c)
            merge_into(nxt, Band{lo[(size_t)i * kMaxRanges + c], hi[(size_t)i * kMaxRanges + c]});
        const int64_t rcap = sb_c0.empty() ? cap0 : cap_rest;
        if (!fits(nxt) || i - sb_start >= rcap) {
            if (i == sb_start) return -1;  // the row alone does not fit
            tiles.push_back(i);
            close_sb();
            sb_start = tile_start = i;
            cur.clear();
            for (int c = 0; c < cnt[i]; ++c)
                merge_into(cur, Band{lo[(size_t)i * kMaxRanges + c], hi[(size_t)i * kMaxRanges + c]});
            if (!fits(cur)) return -1;
            continue;
        }
        cur.swap(nxt);
        if (i > tile_start && rp[i + 1] - rp[tile_start] > kWinTile) {
            tiles.push_back(i);
            tile_start = i;
        }
    }
    tiles.push_back(n);
    close_sb();
    const int64_t nsb = (int64_t)sb_c0.size();
    const size_t b_tiles = sizeof(int64_t) * tiles.size(), b_t0 = sizeof(int64_t) * sb_tile0.size(),
                 b_c0 = sizeof(int64_t) * nsb, b_sp = sizeof(int32_t) * nsb,
                 b_rng = sizeof(int64_t) * rng.size();
    char* d = nullptr;
    if (!hok(hipMalloc(&d, b_tiles + b_t0 + b_c0 + b_rng + b_sp))) return -2;
    bool cp = hok(hipMemcpy(d, tiles.data(), b_tiles, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles, sb_tile0.data(), b_t0, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles + b_t0, sb_c0.data(), b_c0, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles + b_t0 + b_c0, rng.data(), b_rng, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles + b_t0 + b_c0 + b_rng, sb_span.data(), b_sp, hipMemcpyHostToDevice));
    uint16_t* cw = nullptr;
    if (cp && hok(hipMalloc(&cw, sizeof(uint16_t) * A.nnz))) {
        AHIP_LAUNCH(k_colw_ranges, dim3((unsigned)nsb), dim3(256), 0, nullptr,
                    (const int64_t*)(d + b_tiles), (const int64_t*)d,
                    (const int64_t*)(d + b_tiles + b_t0 + b_c0), A.rowptr, A.col, cw);
        cp = hok(hipDeviceSynchronize());
    } else {
        cp = false;
    }
    if (!cp) {
        if (cw) (void)hipFree(cw);
        (void)hipFree(d);
        return -2;
    }
    A.w_tiles = (const int64_t*)d;
    A.w_sb_tile0 = (const int64_t*)(d + b_tiles);
    A.w_sb_c0 = (const int64_t*)(d + b_tiles + b_t0);
    A.w_rng = (const int64_t*)(d + b_tiles + b_t0 + b_c0);
    A.w_sb_span = (const int32_t*)(d + b_tiles + b_t0 + b_c0 + b_rng);
    A.w_nsb = nsb;
    A.w_colw = cw;
    *owned = d;
    (void)ncols;
    return 0;
}

int csr_analyse_window(Csr& A, int64_t ncols, void** owned) {
    const int64_t n = A.n;
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> mn(n), mx(n);
    int32_t *dmn = nullptr, *dmx = nullptr;
    if (!hok(hipMalloc(&dmn, sizeof(int32_t) * n)) || !hok(hipMalloc(&dmx, sizeof(int32_t) * n))) {
        (void)hipFree(dmn);
        return -2;
    }
    int64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    AHIP_LAUNCH(k_row_span, dim3((unsigned)g), dim3(256), 0, nullptr, n, A.rowptr, A.col, dmn, dmx);
    const bool got = hok(hipMemcpy(mn.data(), dmn, sizeof(int32_t) * n, hipMemcpyDeviceToHost)) &&
                     hok(hipMemcpy(mx.data(), dmx, sizeof(int32_t) * n, hipMemcpyDeviceToHost)) &&
                     hok(hipMemcpy(rp.data(), A.rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost));
    (void)hipFree(dmn);
    (void)hipFree(dmx);
    if (!got) return -2;
    // greedy superblocks (column span <= kWinX) split into tiles (<= kWinTile nnz)
    std::vector<int64_t> tiles{0}, sb_tile0{0}, sb_c0;
    std::vector<int32_t> sb_span;
    int64_t sb_start = 0, tile_start = 0;
    int64_t lo = INT64_MAX, hi = -1;
    int64_t cap0 = 0, cap_rest = 0;
    sb_row_caps(n, cap0, cap_rest);
    auto close_sb = [&](int64_t end_row) {
        if (lo > hi) { lo = 0; hi = 0; }
        sb_c0.push_back(lo);
        sb_span.push_back((int32_t)(hi - lo + 1));
        sb_tile0.push_back((int64_t)tiles.size() - 1);
        (void)end_row;
    };
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = rp[i + 1] - rp[i];
        if (len > kWinTile) return -1;
        int64_t nlo = lo, nhi = hi;
        if (mx[i] >= 0) {
            nlo = std::min<int64_t>(lo, mn[i]);
            nhi = std::max<int64_t>(hi, mx[i]);
            if (mx[i] - mn[i] + 1 > kWinX) return -1;
        }
        const int64_t rcap = sb_c0.empty() ? cap0 : cap_rest;
        if (i > sb_start && ((nhi >= nlo && nhi - nlo + 1 > kWinX) || i - sb_start >= rcap)) {
            // close tile and superblock before row i
            tiles.push_back(i);
            close_sb(i);
            sb_start = tile_start = i;
            lo = INT64_MAX;
            hi = -1;
            if (mx[i] >= 0) { lo = mn[i]; hi = mx[i]; }
            continue;
        }
        lo = nlo;
        hi = nhi;
        if (i > tile_start && rp[i + 1] - rp[tile_start] > kWinTile) {
            tiles.push_back(i);
            tile_start = i;
        }
    }
    tiles.push_back(n);
    close_sb(n);
    const int64_t nsb = (int64_t)sb_c0.size();
    // one device allocation holding all four arrays
    const size_t b_tiles = sizeof(int64_t) * tiles.size(), b_t0 = sizeof(int64_t) * sb_tile0.size(),
                 b_c0 = sizeof(int64_t) * nsb, b_sp = sizeof(int32_t) * nsb;
    char* d = nullptr;
    if (!hok(hipMalloc(&d, b_tiles + b_t0 + b_c0 + b_sp))) return -2;
    bool cp = hok(hipMemcpy(d, tiles.data(), b_tiles, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles, sb_tile0.data(), b_t0, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles + b_t0, sb_c0.data(), b_c0, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d + b_tiles + b_t0 + b_c0, sb_span.data(), b_sp, hipMemcpyHostToDevice));
    // 16-bit window-relative column indices (one per nonzero)
    uint16_t* cw = nullptr;
    if (cp && A.nnz > 0) {
        cp = hok(hipMalloc(&cw, sizeof(uint16_t) * A.nnz));
        if (cp) {
            AHIP_LAUNCH(k_colw, dim3((unsigned)nsb), dim3(256), 0, nullptr,
                        (const int64_t*)(d + b_tiles), (const int64_t*)d,
                        (const int64_t*)(d + b_tiles + b_t0), A.rowptr, A.col, cw);
            cp = hok(hipDeviceSynchronize());
        }
    }
    if (!cp) {
        if (cw) (void)hipFree(cw);
        (void)hipFree(d);
        return -2;
    }
    A.w_tiles = (const int64_t*)d;
    A.w_sb_tile0 = (const int64_t*)(d + b_tiles);
    A.w_sb_c0 = (const int64_t*)(d + b_tiles + b_t0);
    A.w_sb_span = (const int32_t*)(d + b_tiles + b_t0 + b_c0);
    A.w_nsb = nsb;
    A.w_colw = cw;
    *owned = d;
    (void)ncols;
    return 0;
}

int csr_build_sell(Csr& A, void** owned) {
    if (!A.w_colw || A.w_nsb <= 0 || A.n >= (int64_t)INT32_MAX) return -1;
    const int64_t n = A.n, nsb = A.w_nsb;
    std::vector<int64_t> rp(n + 1), sb_tile0(nsb + 1);
    if (!hok(hipMemcpy(rp.data(), A.rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost)) ||
        !hok(hipMemcpy(sb_tile0.data(), A.w_sb_tile0, sizeof(int64_t) * (nsb + 1), hipMemcpyDeviceToHost)))
        return -2;
    std::vector<int64_t> tiles((size_t)sb_tile0[nsb] + 1);
    if (!hok(hipMemcpy(tiles.data(), A.w_tiles, sizeof(int64_t) * tiles.size(), hipMemcpyDeviceToHost)))
        return -2;
    std::vector<int64_t> sb_slice0{0}, sptr{0};
    std::vector<int32_t> srow;
    std::vector<int32_t> order;
    for (int64_t b = 0; b < nsb; ++b) {
        const int64_t R0 = tiles[sb_tile0[b]], R1 = tiles[sb_tile0[b + 1]];
        order.resize((size_t)(R1 - R0));
        for (int64_t r = R0; r < R1; ++r) order[r - R0] = (int32_t)r;
        // longest rows first (stable): a slice's width is its first row's length
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t c) {
            return rp[a + 1] - rp[a] > rp[c + 1] - rp[c];
        });
        for (size_t q = 0; q < order.size(); q += 64) {
            const int64_t w = rp[order[q] + 1] - rp[order[q]];
            for (size_t l = 0; l < 64; ++l) srow.push_back(q + l < order.size() ? order[q + l] : -1);
            sptr.push_back(sptr.back() + 64 * w);
        }
        sb_slice0.push_back((int64_t)sptr.size() - 1);
    }
    const int64_t ns = (int64_t)sptr.size() - 1, padded = sptr.back();
    const size_t b0 = sizeof(int64_t) * sb_slice0.size(), b1 = sizeof(int64_t) * sptr.size(),
                 b2 = sizeof(int32_t) * srow.size(), bv = sizeof(double) * (size_t)(padded ? padded : 1),
                 bc = sizeof(uint16_t) * (size_t)(padded ? padded : 1);
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* d = nullptr;
    if (!hok(hipMalloc(&d, up(b0) + up(b1) + up(b2) + up(bv) + up(bc)))) return -2;
    char* p = d;
    auto take = [&](size_t bytes) {
        char* r = p;
        p += up(bytes);
        return r;
    };
    auto* d0 = (int64_t*)take(b0);
    auto* d1 = (int64_t*)take(b1);
    auto* d2 = (int32_t*)take(b2);
    auto* dv = (double*)take(bv);
    auto* dc = (uint16_t*)take(bc);
    bool cp = hok(hipMemcpy(d0, sb_slice0.data(), b0, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d1, sptr.data(), b1, hipMemcpyHostToDevice)) &&
              hok(hipMemcpy(d2, srow.data(), b2, hipMemcpyHostToDevice));
    if (cp && ns > 0)
        AHIP_LAUNCH(k_sell_fill, dim3((unsigned)ns), dim3(64), 0, nullptr, d1, d2, A.rowptr,
                           A.w_colw, A.val, dc, dv);
    if (!cp || !hok(hipDeviceSynchronize())) {
        (void)hipFree(d);
        return -2;
    }
    A.s_sb_slice0 = d0;
    A.s_ptr = d1;
    A.s_row = d2;
    A.s_val = dv;
    A.s_colw = dc;
    A.s_nslices = ns;
    A.s_padded = padded;
    *owned = d;
    return 0;
}

int csr_analyse(Csr& A, int tile, int64_t** rblk_dev) {
    std::vector<int64_t> rp(A.n + 1);
    if (!hok(hipMemcpy(rp.data(), A.rowptr, sizeof(int64_t) * (A.n + 1), hipMemcpyDeviceToHost)))
        return -2;
    std::vector<int64_t> blk;
    blk.reserve(A.nnz / (tile / 2) + 16);
    blk.push_back(0);
    int64_t start = 0;
    for (int64_t i = 0; i < A.n; ++i) {
        const int64_t len = rp[i + 1] - rp[i];
        if (len > tile) return -1;
        // close the block before row i if adding it would exceed the tile
        if (rp[i + 1] - rp[start] > tile) {
            blk.push_back(i);
            start = i;
        }
    }
    blk.push_back(A.n);
    int64_t* d = nullptr;
    if (!hok(hipMalloc(&d, sizeof(int64_t) * blk.size()))) return -2;
    if (!hok(hipMemcpy(d, blk.data(), sizeof(int64_t) * blk.size(), hipMemcpyHostToDevice))) {
        (void)hipFree(d);
        return -2;
    }
    *rblk_dev = d;
    A.rblk = d;
    A.nrblk = (int64_t)blk.size() - 1;
    A.tile = tile;
    return 0;
}

double csr_bytes(const Csr& A) {
    // bytes the selected kernel must move: val + column index (+ rowptr, x, y);
    // SELL: 10 B per stored nonzero + the 4-B row map (padding not counted)
    if (csr_sym_det_fallback(A)) {  // the full-storage kernel csr_spmv runs instead
        Csr F = A;
        F.kernel = A.s_val ? kCsrSell : (A.rblk ? kCsrStream : kCsrVector);
        return csr_bytes(F);
    }
    if (A.kernel == kCsrSell && A.s_val)
        return 10.0 * (double)A.nnz + 4.0 * (double)A.n + 16.0 * (double)A.n;
    // symmetric storage: 10 B per stored upper-triangle entry + row map + x + y
    if (A.kernel == kCsrSymSell && A.ss_val)
        return 10.0 * (double)A.ss_nnz + 4.0 * (double)A.n + 16.0 * (double)A.n;
    const bool cw = A.w_colw != nullptr && (A.kernel == kCsrWVec || A.kernel == kCsrWVec8 ||
                                          A.kernel == kCsrWVecX || A.kernel == kCsrWVecP3 ||
                                          A.kernel == kCsrWVecP4);
    return (cw ? 10.0 : 12.0) * (double)A.nnz + 8.0 * (double)(A.n + 1) + 16.0 * (double)A.n;
}

template <int L, int U, bool NT, bool CW, bool XCD = false>
static void launch_wvec1(hipStream_t s, const Csr& A, const double* x, double* y) {
    const size_t lds = sizeof(double) * kWinX;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_csr_wvec<L, U, NT, CW, XCD>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    AHIP_LAUNCH((k_csr_wvec<L, U, NT, CW, XCD>), dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s,
                       A.w_sb_tile0, A.w_tiles, A.w_sb_c0, A.w_sb_span, A.rowptr, A.col, A.w_colw,
                       A.val, x, y);
}

template <int L, int U>
static void launch_wvec(hipStream_t s, const Csr& A, const double* x, double* y, bool nt) {
    const bool cw = A.w_colw != nullptr && A.kernel != kCsrWVecNT;
    if (cw && A.kernel == kCsrWVecX) launch_wvec1<L, U, false, true, true>(s, A, x, y);
    else if (cw) launch_wvec1<L, U, false, true>(s, A, x, y);
    else if (nt) launch_wvec1<L, U, true, false>(s, A, x, y);
    else launch_wvec1<L, U, false, false>(s, A, x, y);
}

// AHIP_SELL_FIN=0: a finalize deferred into the SpMV gets a launch of its own
// before the full-storage SELL kernel instead of riding in it
static bool sell_fin() {
    static const bool on = [] {
        const char* e = getenv("AHIP_SELL_FIN");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool csr_sym_det_fallback(const Csr& A) {
    return A.kernel == kCsrSymSell && A.ss_val && !A.ss_det_all && deterministic();
}

void csr_spmv(hipStream_t s, const Csr& A, const double* x, double* y, FinQueue* q) {
    if (csr_sym_det_fallback(A)) {
        // the full CSR arrays stay resident under symmetric storage: the
        // fixed-order full-storage form the operator had before
        Csr F = A;
        F.kernel = A.s_val ? kCsrSell : (A.rblk ? kCsrStream : kCsrVector);
        csr_spmv(s, F, x, y, q);
        return;
    }
    if (A.kernel == kCsrSymSell && A.ss_val) {  // (carries a deferred finalize itself)
        csr_spmv_sym(s, A, x, y, q);
        return;
    }
    // the full-storage SELL kernel's default form (NT loads, U = 4) and its
    // multi-range form carry a deferred finalize in workgroup 0 (k_csr_sell
    // FIN); every other form has it launched first
    const bool sell_carry = A.kernel == kCsrSell && A.s_val && (A.w_rng || A.s_unroll == 10) && sell_fin();
    FinArgs fa{};
    size_t fin_lds = 0;
    // it must fit the window below the Arnoldi H staging (kFoldHMax^2 doubles)
    const bool carried =
        sell_carry && take_deferred_finalize(q, &fa, &fin_lds,
                                             sizeof(double) * (kWinX - kFoldHMax * kFoldHMax));
    if (!carried) flush_deferred_finalize(q, s);
    if (A.kernel == kCsrSell && A.s_val) {
        const size_t lds = sizeof(double) * kWinX;
        if (carried) {
            auto gof = [&](auto kern) {
                (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds);
                AHIP_LAUNCH(kern, dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s, A.s_sb_slice0,
                            A.s_ptr, A.s_row, A.w_sb_c0, A.w_sb_span, A.s_colw, A.s_val, x, y,
                            (const int64_t*)A.w_rng, fa);
            };
            if (A.w_rng) {
                if (fa.hs) gof(k_csr_sell_fin<true, 2>);
                else gof(k_csr_sell_fin<true, 1>);
            } else {
                if (fa.hs) gof(k_csr_sell_fin<false, 2>);
                else gof(k_csr_sell_fin<false, 1>);
            }
            return;
        }
        auto go = [&](auto kern) {  // k_csr_sell (one window range: no range table)
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds);
            AHIP_LAUNCH(kern, dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s, A.s_sb_slice0,
                               A.s_ptr, A.s_row, A.w_sb_c0, A.w_sb_span, A.s_colw, A.s_val, x, y,
                               (const int64_t*)nullptr);
        };
        auto go2 = [&](auto kern) {  // k_csr_sell2
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds);
            AHIP_LAUNCH(kern, dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s, A.s_sb_slice0,
                               A.s_ptr, A.s_row, A.w_sb_c0, A.w_sb_span, A.s_colw, A.s_val, x, y);
        };
        if (A.w_rng) {  // multi-range windows: only this form stages them
            (void)hipFuncSetAttribute((const void*)k_csr_sell<4, true, true, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            AHIP_LAUNCH((k_csr_sell<4, true, true, true>), dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s,
                        A.s_sb_slice0, A.s_ptr, A.s_row, A.w_sb_c0, A.w_sb_span, A.s_colw, A.s_val, x, y,
                        A.w_rng);
            return;
        }
        if (A.s_unroll == 4) go(k_csr_sell<4, true>);
        else if (A.s_unroll == 9) go(k_csr_sell<8, true, true>);   // non-temporal val/col
        else if (A.s_unroll == 10) go(k_csr_sell<4, true, true>);
        else if (A.s_unroll == 11) go(k_csr_sell<6, true, true>);
        else if (A.s_unroll == 2) go(k_csr_sell<2, true>);
        else if (A.s_unroll == 3) go(k_csr_sell<3, true>);
        else if (A.s_unroll == 6) go(k_csr_sell<6, true>);
        else if (A.s_unroll == 5) go2(k_csr_sell2<4, true>);  // two slices per wave
        else if (A.s_unroll == 7) go2(k_csr_sell2<2, true>);
        else go(k_csr_sell<8, true>);
        return;
    }
    if ((A.kernel == kCsrWVec || A.kernel == kCsrWVecNT || A.kernel == kCsrWVecX) && A.w_nsb > 0) {
        const bool nt = A.kernel == kCsrWVecNT;
        const double avg = A.n > 0 ? (double)A.nnz / (double)A.n : 1.0;
        if (avg <= 6) launch_wvec<4, 2>(s, A, x, y, nt);
        else if (avg <= 12) launch_wvec<8, 2>(s, A, x, y, nt);
        else if (avg <= 28) launch_wvec<8, 4>(s, A, x, y, nt);
        else if (avg <= 60) launch_wvec<16, 4>(s, A, x, y, nt);
        else if (avg <= 120) launch_wvec<32, 4>(s, A, x, y, nt);
        else launch_wvec<64, 4>(s, A, x, y, nt);
        return;
    }
    if ((A.kernel == kCsrWVecP3 || A.kernel == kCsrWVecP4) && A.w_nsb > 0 && A.w_colw) {
        const size_t lds = sizeof(double) * kWinX;
        const double avg = A.n > 0 ? (double)A.nnz / (double)A.n : 1.0;
        auto go = [&](auto kern) {
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            AHIP_LAUNCH(kern, dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s, A.w_sb_tile0, A.w_tiles,
                               A.w_sb_c0, A.w_sb_span, A.rowptr, A.col, A.w_colw, A.val, x, y);
        };
        const bool p4 = A.kernel == kCsrWVecP4;
        if (avg <= 28) p4 ? go(k_csr_wvecp<8, 4, 4, true>) : go(k_csr_wvecp<8, 4, 3, true>);
        else if (avg <= 60) p4 ? go(k_csr_wvecp<16, 4, 4, true>) : go(k_csr_wvecp<16, 4, 3, true>);
        else p4 ? go(k_csr_wvecp<32, 4, 4, true>) : go(k_csr_wvecp<32, 4, 3, true>);
        return;
    }
    if (A.kernel == kCsrWVec8 && A.w_nsb > 0) {  // fewer lanes per row, more loads per lane
        const double avg = A.n > 0 ? (double)A.nnz / (double)A.n : 1.0;
        if (avg <= 12) launch_wvec<4, 4>(s, A, x, y, false);
        else if (avg <= 28) launch_wvec<4, 8>(s, A, x, y, false);
        else if (avg <= 60) launch_wvec<8, 8>(s, A, x, y, false);
        else launch_wvec<16, 8>(s, A, x, y, false);
        return;
    }
    if ((A.kernel == kCsrWindow || A.kernel == kCsrWindowNT) && A.w_nsb > 0) {
        const size_t lds = sizeof(double) * (kWinX + kWinTile);
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)k_csr_window<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            (void)hipFuncSetAttribute((const void*)k_csr_window<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr = true;
        }
        if (A.kernel == kCsrWindowNT)
            AHIP_LAUNCH((k_csr_window<true>), dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s,
                               A.w_sb_tile0, A.w_tiles, A.w_sb_c0, A.w_sb_span, A.rowptr, A.col, A.val, x, y);
        else
            AHIP_LAUNCH((k_csr_window<false>), dim3((unsigned)A.w_nsb), dim3(kWinThreads), lds, s,
                               A.w_sb_tile0, A.w_tiles, A.w_sb_c0, A.w_sb_span, A.rowptr, A.col, A.val, x, y);
        return;
    }
    if (A.kernel != kCsrVector && A.rblk) {
        const dim3 g((unsigned)A.nrblk), b(kBlock);
        const bool nt = A.kernel == kCsrStreamNT;
        if (A.tile == 2048) {
            if (nt) AHIP_LAUNCH((k_csr_stream<2048, true>), g, b, 0, s, A.rblk, A.rowptr, A.col, A.val, x, y);
            else AHIP_LAUNCH((k_csr_stream<2048, false>), g, b, 0, s, A.rblk, A.rowptr, A.col, A.val, x, y);
        } else {
            if (nt) AHIP_LAUNCH((k_csr_stream<4096, true>), g, b, 0, s, A.rblk, A.rowptr, A.col, A.val, x, y);
            else AHIP_LAUNCH((k_csr_stream<4096, false>), g, b, 0, s, A.rblk, A.rowptr, A.col, A.val, x, y);
        }
        return;
    }
    const int G = A.group;
    const int rows_per_block = kBlock / G;
    int64_t g = (A.n + rows_per_block - 1) / rows_per_block;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    switch (G) {
        case 4: AHIP_LAUNCH(k_csr_vector<4>, dim3(g), dim3(kBlock), 0, s, A.n, A.rowptr, A.col, A.val, x, y); break;
        case 8: AHIP_LAUNCH(k_csr_vector<8>, dim3(g), dim3(kBlock), 0, s, A.n, A.rowptr, A.col, A.val, x, y); break;
        case 16: AHIP_LAUNCH(k_csr_vector<16>, dim3(g), dim3(kBlock), 0, s, A.n, A.rowptr, A.col, A.val, x, y); break;
        case 32: AHIP_LAUNCH(k_csr_vector<32>, dim3(g), dim3(kBlock), 0, s, A.n, A.rowptr, A.col, A.val, x, y); break;
        default: AHIP_LAUNCH(k_csr_vector<64>, dim3(g), dim3(kBlock), 0, s, A.n, A.rowptr, A.col, A.val, x, y); break;
    }
}

}  // namespace ahip::dev

// ------------------------------------------------------------ HBM probe ---
// Read-only streaming probe (sum of a large buffer) at 8- or 16-byte loads per
// lane: the achievable HBM read rate that the SpMV/Gram-Schmidt kernels are
// compared against.
namespace ahip::dev {
namespace {
template <int W>
__global__ __launch_bounds__(256) void k_probe(int64_t n8, const double* __restrict__ a,
                                               double* __restrict__ out) {
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    if constexpr (W == 16) {
        const double2* a2 = reinterpret_cast<const double2*>(a);
        const int64_t n16 = n8 / 2;
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
            const double2 v = a2[i];
            s += v.x + v.y;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) s += a[i];
    }
    if (s == 12345.678) out[0] = s;  // keep the loads alive
}
}  // namespace
}  // namespace ahip::dev

extern "C" double arpack_hip_stream_probe(int64_t nbytes, int width, int grid, int reps) {
    double* a = nullptr;
    double* o = nullptr;
    if (hipMalloc(&a, nbytes) || hipMalloc(&o, 8)) return -1.0;
    (void)hipMemset(a, 0, nbytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int64_t n8 = nbytes / 8;
    auto launch = [&]() {
        if (width == 16)
            AHIP_LAUNCH(ahip::dev::k_probe<16>, dim3(grid), dim3(256), 0, nullptr, n8, a, o);
        else
            AHIP_LAUNCH(ahip::dev::k_probe<8>, dim3(grid), dim3(256), 0, nullptr, n8, a, o);
    };
    launch();
    (void)hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(a);
    (void)hipFree(o);
    return (double)nbytes * reps / (ms * 1e-3) / 1e9;
}
