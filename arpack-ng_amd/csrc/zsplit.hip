// XCD column split of the complex CSR operator (config 5: n = 5e5, ~100
// random columns a row).  x (8 MB) does not fit one XCD's 4 MB L2, so the
// wave-per-row kernel's random gathers miss to the Infinity Cache (0.63 ms,
// 1.6 TB/s of algorithmic bytes).  Here the columns are cut into S slices of
// x (S = 8, or 4 when a quarter of x fits 2 MB, see zcsr_build_split);
// workgroup b works on slice b % S -- the hardware deals workgroups
// round-robin over the 8 XCDs, so every slice's gathers stay in the L2 of one
// XCD (S = 8) or of the two XCDs s and s + 4 (S = 4) --
// with 8 lanes a row on the slice's own CSR (slice-relative 16-bit columns,
// non-temporal matrix loads), and writes a partial y per slice; a second
// kernel sums the 8 partials in a fixed order.  tools/zspmv_split.hip: 0.41 ms
// against 0.63 (and 0.72 for the same split WITHOUT the XCD alignment: the
// alignment, not the split, is the gain); results within 5e-16 of the
// wave-per-row kernel (a different, fixed summation order).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "zcommon.hpp"
#include "zengine.hpp"

namespace ahip::zdev {

namespace {
using namespace zc;
constexpr int kMaxSlices = zc::kZMaxSlices;
constexpr int kLanes = 8;   // lanes per row (tools/zspmv_split.hip: 8 of 4/8/16)

template <int S>
__global__ void k_zsplit_count(int64_t n, int64_t sw, const int64_t* __restrict__ rp,
                               const int32_t* __restrict__ col, int32_t* __restrict__ cnt) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        int32_t c[S];
#pragma unroll
        for (int s = 0; s < S; ++s) c[s] = 0;
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) c[col[k] / sw]++;
#pragma unroll
        for (int s = 0; s < S; ++s) cnt[(int64_t)s * (n + 1) + r] = c[s];
    }
}

template <int S, class CT>
__global__ void k_zsplit_fill(int64_t n, int64_t sw, const int64_t* __restrict__ rp,
                              const int32_t* __restrict__ col, const double2* __restrict__ val,
                              const int32_t* __restrict__ srp, const int64_t* __restrict__ base,
                              CT* __restrict__ scol, double2* __restrict__ sval) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        int64_t pos[S];
#pragma unroll
        for (int s = 0; s < S; ++s) pos[s] = base[s] + srp[(int64_t)s * (n + 1) + r];
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {  // row order kept inside each slice
            const int s = (int)(col[k] / sw);
            scol[pos[s]] = (CT)(col[k] - s * sw);
            sval[pos[s]] = val[k];
            pos[s]++;
        }
    }
}

template <int S, class CT>
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
    const int s = (int)(blockIdx.x % S);  // the XCD (S = 4: one of two) this workgroup runs on
    const int64_t q = blockIdx.x / S, nq = gridDim.x / S;
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

template <int S>
__global__ void k_zsplit_combine(int64_t n, const double2* __restrict__ yp, double2* __restrict__ y,
                                 const int* __restrict__ gate) {
    if (gate && *gate) return;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256)
        y[r] = zc::slice_sum<S>(yp, n, r);
}

// ---- column-sorted tiles --------------------------------------------------
// Measured (tools/zspmv_probe.hip, config-5 operator): the CSR split spends
// 0.41 ms of which only 0.23-0.28 is its matrix stream -- the rest is the
// random 16-byte gather, which costs the address unit one cache line per lane
// whether or not the line is in L2 (a 64 KB gather window: 0.38 ms).  Here the
// entries of each (row block of kTileRows rows, slice) are sorted by column, so
// the 64 lanes of a wave gather from a few neighbouring lines of x, and every
// product is added into the block's row sums in LDS (ds_add_f64), written once
// as the slice's partial y: 0.226 ms, same results to 5e-16 (the LDS adds land
// in schedule order, so y is reproducible to rounding, not bitwise).
constexpr int kTileRows = 4096;  // 64 KB of LDS row sums: two blocks a CU
constexpr int kTileU = 4;        // entries a lane keeps in flight (default; AHIP_ZTILE_U=8 for A/B)

// Two encodings of a tile's column-sorted entries (segment q = slice * nrb +
// row block: entries [seg[q], seg[q + 1])):
//  * PK = false: idx = row << 20 | slice column (4 B) + the 16-B value: 20 B an entry;
//  * PK = true (packed, default where it fits): idx16 = row << 4 | dcol (2 B),
//    dcol = the column step from the previous entry of the same 64-entry
//    chunk (0 for a chunk's first), and one int32 base column a chunk: 18.06 B
//    an entry.  A segment starts on a chunk boundary, so every wave's load is
//    one whole chunk and the columns are its base plus a wave-wide inclusive
//    scan of the steps.  Steps above 15 get zero-valued filler entries between
//    them, and every segment is padded to whole chunks with zero values (both
//    at the segment's own columns; built only where they stay below 3% of the
//    entries, ztile_pack).
// Inclusive scan over the 64 lanes in DPP moves (VALU only: the first form,
// six __shfl_up's a scan, went through LDS beside the tile's LDS atomics and
// made the packed product 5% SLOWER than the 20-B one, profiles/r06c):
// Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8), then row 0's
// total into row 1 and row 2's into row 3 (row_bcast:15), then the first two
// rows' total into rows 2 and 3 (row_bcast:31).  Lanes without a source keep
// `old` = 0 (bound_ctrl off); rows outside a move's row mask add 0.
__device__ __forceinline__ int wave_iscan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

template <bool PK, int U, int T = 256>
__device__ __forceinline__ void tile_batch(int64_t e, const void* __restrict__ idx,
                                           const int32_t* __restrict__ cbase,
                                           const double2* __restrict__ val, int (&row)[U], int (&col)[U],
                                           double2 (&v)[U]) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    if constexpr (PK) {
        uint16_t id[U];
        int cb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every load of the batch issued first
            id[u] = __builtin_nontemporal_load(static_cast<const uint16_t*>(idx) + e + u * T);
            const dv2 w = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + e + u * T);
            v[u] = make_double2(w.x, w.y);
            // one base a wave: the chunk index is wave-uniform (a segment
            // starts on a chunk, a wave loads one whole chunk), so a scalar load
            cb[u] = cbase[__builtin_amdgcn_readfirstlane((int)((e + u * T) >> 6))];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            row[u] = id[u] >> 4;
            col[u] = cb[u] + wave_iscan(id[u] & 15);
        }
    } else {
        uint32_t id[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            id[u] = __builtin_nontemporal_load(static_cast<const uint32_t*>(idx) + e + u * T);
            const dv2 w = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + e + u * T);
            v[u] = make_double2(w.x, w.y);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            row[u] = (int)(id[u] >> 20);
            col[u] = (int)(id[u] & 0xfffffu);
        }
    }
}

// The tile walk of both products below: for each batch of entries, the x
// gathers of the slice, then add(row, re, im) per entry (LDS row sums).  A
// packed segment's length is a multiple of 64, so the tail loop's condition is
// uniform across a wave (its scan needs every lane).
template <bool PK, int TU, class Add, int T = 256>
__device__ __forceinline__ void tile_walk(int64_t e0, int64_t e1, const void* __restrict__ idx,
                                          const int32_t* __restrict__ cbase,
                                          const double2* __restrict__ val, const double2* __restrict__ xs,
                                          Add add) {
    int64_t e = e0 + threadIdx.x;
    for (; e + (TU - 1) * T < e1; e += TU * T) {
        int row[TU], col[TU];
        double2 v[TU];
        tile_batch<PK, TU, T>(e, idx, cbase, val, row, col, v);
        double2 xv[TU];
#pragma unroll
        for (int u = 0; u < TU; ++u) xv[u] = xs[col[u]];
#pragma unroll
        for (int u = 0; u < TU; ++u)
            add(row[u], v[u].x * xv[u].x - v[u].y * xv[u].y, v[u].x * xv[u].y + v[u].y * xv[u].x);
    }
    for (; e < e1; e += T) {
        int row[1], col[1];
        double2 v[1];
        tile_batch<PK, 1, T>(e, idx, cbase, val, row, col, v);
        const double2 xv = xs[col[0]];
        add(row[0], v[0].x * xv.x - v[0].y * xv.y, v[0].x * xv.y + v[0].y * xv.x);
    }
}

template <int S, bool PK, int TU, int T>
__device__ __forceinline__ void ztile_body(int64_t n, int64_t sw, const int64_t* __restrict__ seg,
                                           int64_t nrb, const void* __restrict__ idx,
                                           const int32_t* __restrict__ cbase,
                                           const double2* __restrict__ val,
                                           const double2* __restrict__ x, double2* __restrict__ yp,
                                           const int* __restrict__ gate) {
    if (gate && *gate) return;
    __shared__ double ylds[2 * kTileRows];
    const int s = (int)(blockIdx.x % S);  // the XCD (S = 4: one of two) this block runs on
    const int64_t rb = blockIdx.x / S;
    const int64_t r0 = rb * kTileRows;
    const int rows = (int)((n - r0) < kTileRows ? (n - r0) : kTileRows);
    for (int i = threadIdx.x; i < 2 * rows; i += T) ylds[i] = 0.0;
    __syncthreads();
    const int64_t q = s * nrb + rb;
    auto add = [&](int r, double re, double im) {
        atomicAdd(&ylds[2 * r], re);
        atomicAdd(&ylds[2 * r + 1], im);
    };
    tile_walk<PK, TU, decltype(add), T>(seg[q], seg[q + 1], idx, cbase, val, x + (int64_t)s * sw, add);
    __syncthreads();
    double2* y = yp + (int64_t)s * n + r0;
    for (int i = threadIdx.x; i < rows; i += T) y[i] = make_double2(ylds[2 * i], ylds[2 * i + 1]);
}

template <int S, bool PK, int TU = kTileU, int T = 256>
__global__ __launch_bounds__(T) void k_ztile(int64_t n, int64_t sw, const int64_t* __restrict__ seg,
                                               int64_t nrb, const void* __restrict__ idx,
                                               const int32_t* __restrict__ cbase,
                                               const double2* __restrict__ val,
                                               const double2* __restrict__ x,
                                               double2* __restrict__ yp, const int* __restrict__ gate) {
    ztile_body<S, PK, TU, T>(n, sw, seg, nrb, idx, cbase, val, x, yp, gate);
}

// the 1,024-thread packed walk held to 64 VGPRs (8 waves a SIMD: both LDS-sized
// workgroups of a CU resident) where TU would otherwise take more
template <int S, int TU>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_ztile_w8(
    int64_t n, int64_t sw, const int64_t* __restrict__ seg, int64_t nrb, const void* __restrict__ idx,
    const int32_t* __restrict__ cbase, const double2* __restrict__ val, const double2* __restrict__ x,
    double2* __restrict__ yp, const int* __restrict__ gate) {
    ztile_body<S, true, TU, 1024>(n, sw, seg, nrb, idx, cbase, val, x, yp, gate);
}

constexpr int kZMaxBlocks = 256;  // k_zabsmax's grid (<= k_ztile_det's block size)

// Deterministic mode's tile product (arpack_hip_set_deterministic): k_ztile
// with the row sums as 64-bit FIXED-POINT integers (the scheme of
// spmv_sym.hip's k_csr_ssell_det): every product's real and imaginary part
// (|.| <= 2 amax max|x| < 2^E, amax of this row block and slice, max|x| over
// x by k_zabsmax just before) becomes q = rint(p 2^(B-E)) -- one fma onto
// 1.5 * 2^52 -- and the LDS sums are exact integer adds, the same in any
// wave order; y_s = (double)(sum q) 2^(E-B).  B = min(51, 62 - bits(L)) for at
// most L entries a row in a slice.  The slice partials are summed in
// zc::slice_sum's fixed order as before.
template <int S, bool PK, int TU = kTileU, int T = 256>
__global__ __launch_bounds__(T) void k_ztile_det(int64_t n, int64_t sw, const int64_t* __restrict__ seg,
                                                   int64_t nrb, const void* __restrict__ idx,
                                                   const int32_t* __restrict__ cbase,
                                                   const double2* __restrict__ val,
                                                   const double2* __restrict__ x,
                                                   double2* __restrict__ yp, const int* __restrict__ gate,
                                                   const double* __restrict__ amax,
                                                   const unsigned long long* __restrict__ xmax, int bits) {
    if (gate && *gate) return;
    constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
    const unsigned long long kMagicBits = (unsigned long long)__double_as_longlong(kMagic);
    __shared__ unsigned long long ylds[2 * kTileRows];
    static_assert(T >= kZMaxBlocks, "one block maximum a thread");
    __shared__ unsigned long long wmax[T / 64];
    const int s = (int)(blockIdx.x % S);
    const int64_t rb = blockIdx.x / S;
    const int64_t r0 = rb * kTileRows;
    const int rows = (int)((n - r0) < kTileRows ? (n - r0) : kTileRows);
    for (int i = threadIdx.x; i < 2 * rows; i += T) ylds[i] = 0ull;
    {  // max|x| from k_zabsmax's kZMaxBlocks block maxima (one a thread; a
       // maximum, so the same in any order and at any block size)
        unsigned long long m = threadIdx.x < kZMaxBlocks ? xmax[threadIdx.x] : 0ull;
        for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
        if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    }
    __syncthreads();
    unsigned long long wm = wmax[0];
#pragma unroll
    for (int w = 1; w < T / 64; ++w) wm = max(wm, wmax[w]);
    const double X = __longlong_as_double((long long)wm);
    const int64_t q = s * nrb + rb;
    int ea = 0, ex = 0;
    (void)frexp(amax[q], &ea);
    (void)frexp(X, &ex);
    const int E = max(ea + ex + 1, bits - 1000);
    const double inv = ldexp(1.0, bits - E);
    const double sc = X <= DBL_MAX ? ldexp(1.0, E - bits) : __longlong_as_double(0x7ff8000000000000ll);
    __syncthreads();
    auto q64 = [&](double p) {
        const double f = fma(p, inv, kMagic);
        return (unsigned long long)__double_as_longlong(f) - kMagicBits;
    };
    auto add = [&](int r, double re, double im) {
        atomicAdd(&ylds[2 * r], q64(re));
        atomicAdd(&ylds[2 * r + 1], q64(im));
    };
    tile_walk<PK, TU, decltype(add), T>(seg[q], seg[q + 1], idx, cbase, val, x + (int64_t)s * sw, add);
    __syncthreads();
    double2* y = yp + (int64_t)s * n + r0;
    for (int i = threadIdx.x; i < rows; i += T)
        y[i] = make_double2((double)(long long)ylds[2 * i] * sc, (double)(long long)ylds[2 * i + 1] * sc);
}

// bits of max(|re x_i|, |im x_i|) over x (non-negative doubles order as their
// bit patterns, so a NaN wins): one maximum per block into xmax[block], which
// k_ztile_det's blocks reduce themselves (no atomics: 4,096 arrivals on one
// word cost 49 us, MI355X_MICROARCH.md "fanin")
__global__ __launch_bounds__(256) void k_zabsmax(int64_t n2, const double* __restrict__ x,
                                                 unsigned long long* __restrict__ xmax,
                                                 const int* __restrict__ gate) {
    if (gate && *gate) return;
    __shared__ unsigned long long w[4];
    unsigned long long m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
        m = max(m, (unsigned long long)__double_as_longlong(fabs(x[i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) xmax[blockIdx.x] = max(max(w[0], w[1]), max(w[2], w[3]));
}

// per (slice, row block) segment q: the largest |re|, |im| of its entries;
// *lmax: the most entries a row has in one slice
__global__ void k_ztile_amax(const int64_t* __restrict__ seg, const double* __restrict__ tval,
                             double* __restrict__ amax) {
    const int64_t q = blockIdx.x;
    double m = 0.0;
    for (int64_t k = 2 * seg[q] + threadIdx.x; k < 2 * seg[q + 1]; k += blockDim.x) m = fmax(m, fabs(tval[k]));
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    __shared__ double w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) amax[q] = fmax(fmax(w[0], w[1]), fmax(w[2], w[3]));
}
__global__ void k_zslice_lmax(int64_t n, int ns, const int32_t* __restrict__ srp, int* __restrict__ lmax) {
    int m = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        for (int s = 0; s < ns; ++s) {
            const int32_t* rp = srp + (int64_t)s * (n + 1);
            m = max(m, rp[r + 1] - rp[r]);
        }
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(lmax, m);
}

// sort keys (slice column), the row of every entry, and the segment bounds of
// the (slice, row block) segments in the slice-major entry order
template <class CT>
__global__ void k_ztile_keys(int64_t n, int ns, const int32_t* __restrict__ srp, const int64_t* __restrict__ base,
                             const CT* __restrict__ scol, uint32_t* __restrict__ key,
                             uint32_t* __restrict__ erow, uint32_t* __restrict__ perm) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        for (int s = 0; s < ns; ++s) {
            const int32_t* rp = srp + (int64_t)s * (n + 1);
            for (int64_t k = base[s] + rp[r]; k < base[s] + rp[r + 1]; ++k) {
                key[k] = (uint32_t)scol[k];
                erow[k] = (uint32_t)(r % kTileRows);
                perm[k] = (uint32_t)k;
            }
        }
    }
}
__global__ void k_ztile_segs(int64_t n, int nsl, int64_t nrb, const int32_t* __restrict__ srp,
                             const int64_t* __restrict__ base, int64_t* __restrict__ seg) {
    const int64_t ns = nsl * nrb;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= ns;
         q += (int64_t)gridDim.x * blockDim.x) {
        if (q == ns) {
            seg[q] = base[nsl];
            continue;
        }
        const int s = (int)(q / nrb);
        const int64_t rb = q % nrb;
        seg[q] = base[s] + srp[(int64_t)s * (n + 1) + rb * kTileRows];
    }
}
__global__ void k_ztile_gather(int64_t nnz, const uint32_t* __restrict__ perm,
                               const uint32_t* __restrict__ key_sorted, const uint32_t* __restrict__ erow,
                               const double2* __restrict__ sval, uint32_t* __restrict__ idx,
                               double2* __restrict__ tval) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = perm[k];
        idx[k] = (erow[p] << 20) | key_sorted[k];
        tval[k] = sval[p];
    }
}

// ---- packing (ztile_pack): the 20-B encoding -> the 18-B one -------------------
__device__ __forceinline__ int64_t seg_of(const int64_t* __restrict__ seg, int64_t nseg, int64_t k) {
    int64_t lo = 0, hi = nseg;  // the last q with seg[q] <= k
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (seg[mid] <= k) lo = mid;
        else hi = mid;
    }
    return lo;
}
// fillers before sorted entry k: steps above 15 inside a segment
__global__ void k_zpk_fills(int64_t nnz, const uint32_t* __restrict__ idx, const int64_t* __restrict__ seg,
                            int64_t nseg, int64_t* __restrict__ fills) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        int64_t f = 0;
        if (k < nnz) {
            const int64_t q = seg_of(seg, nseg, k);
            if (k > seg[q]) {
                const int32_t g = (int32_t)(idx[k] & 0xfffffu) - (int32_t)(idx[k - 1] & 0xfffffu);
                f = g > 15 ? (g + 14) / 15 - 1 : 0;
            }
        }
        fills[k] = f;
    }
}
// every entry at its packed position, its fillers just before it (columns
// col - 15 i, zero values; rows and values were zeroed)
__global__ void k_zpk_scatter(int64_t nnz, const uint32_t* __restrict__ idx, const double2* __restrict__ val,
                              const int64_t* __restrict__ seg, int64_t nseg, const int64_t* __restrict__ fscan,
                              const int64_t* __restrict__ poff, int32_t* __restrict__ pcol,
                              uint16_t* __restrict__ prow, double2* __restrict__ pval) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = seg_of(seg, nseg, k);
        // after the fillers of every entry up to and including k (its own
        // precede it): the inclusive count fscan[k + 1]
        const int64_t pos = poff[q] + (k - seg[q]) + (fscan[k + 1] - fscan[seg[q]]);
        const int32_t c = (int32_t)(idx[k] & 0xfffffu);
        pcol[pos] = c;
        prow[pos] = (uint16_t)(idx[k] >> 20);
        pval[pos] = val[k];
        const int64_t f = fscan[k + 1] - fscan[k];
        for (int64_t i = 1; i <= f; ++i) pcol[pos - i] = c - (int32_t)(15 * i);
    }
}
__global__ void k_zpk_segfill(int64_t nseg, const int64_t* __restrict__ seg, const int64_t* __restrict__ fscan,
                              int64_t* __restrict__ out) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= nseg;
         q += (int64_t)gridDim.x * blockDim.x)
        out[q] = fscan[seg[q]];
}
// a segment's padding to whole chunks: its last column, zero values
__global__ void k_zpk_pad(int64_t nseg, const int64_t* __restrict__ seg, const int64_t* __restrict__ fscan,
                          const int64_t* __restrict__ poff, int32_t* __restrict__ pcol) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nseg;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t len = (seg[q + 1] - seg[q]) + (fscan[seg[q + 1]] - fscan[seg[q]]);
        const int32_t last = len > 0 ? pcol[poff[q] + len - 1] : 0;
        for (int64_t p = poff[q] + len; p < poff[q + 1]; ++p) pcol[p] = last;
    }
}
// idx16 = row << 4 | step, one base column a 64-entry chunk; *bad counts steps
// outside [0, 15] (none by construction: the build checks)
__global__ void k_zpk_encode(int64_t stored, const int32_t* __restrict__ pcol, const uint16_t* __restrict__ prow,
                             uint16_t* __restrict__ idx16, int32_t* __restrict__ cbase, int* __restrict__ bad) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < stored;
         p += (int64_t)gridDim.x * blockDim.x) {
        int32_t d = 0;
        if ((p & 63) == 0) cbase[p >> 6] = pcol[p];
        else d = pcol[p] - pcol[p - 1];
        if (d < 0 || d > 15 || prow[p] >= kTileRows) {
            atomicAdd(bad, 1);
            d = 0;
        }
        idx16[p] = (uint16_t)((prow[p] << 4) | d);
    }
}

inline int grid1(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}
}  // namespace

void zcsr_free_split(ZCsr& A) {
    if (A.t_idx) (void)hipFree(A.t_idx);
    if (A.t_val) (void)hipFree(A.t_val);
    if (A.t_cbase) (void)hipFree(A.t_cbase);
    if (A.t_seg) (void)hipFree(A.t_seg);
    A.t_cbase = nullptr;
    A.t_seg = nullptr;
    A.t_pk = false;
    if (A.t_amax) (void)hipFree(A.t_amax);
    if (A.t_xmax) (void)hipFree(A.t_xmax);
    A.t_idx = nullptr;
    A.t_val = nullptr;
    A.t_amax = nullptr;
    A.t_xmax = nullptr;
    A.t_det = 0;
    A.tile = false;
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

// The packed (18-B) encoding of the sorted tiles (k_ztile PK): from the 20-B
// arrays A.t_idx / A.t_val over A.t_seg, which it replaces.  0: packed; 1: not
// built (AHIP_ZTILE_PACK=0, or fillers + padding above 3% of the entries --
// a sparse slice); < 0: error (the 20-B form stays).
static int ztile_pack(ZCsr& A, int64_t nseg) {
    static const bool off = [] {
        const char* e = getenv("AHIP_ZTILE_PACK");
        return e && e[0] == '0';
    }();
    if (off) return 1;
    const int64_t nnz = A.nnz;
    int64_t *fills = nullptr, *fscan = nullptr, *segf = nullptr, *poff = nullptr;
    int32_t *pcol = nullptr, *cbase = nullptr;
    uint16_t *prow = nullptr, *idx16 = nullptr;
    double2* pval = nullptr;
    int* bad = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto release = [&](bool outputs) {
        for (void* q : {(void*)fills, (void*)fscan, (void*)segf, (void*)pcol, (void*)prow, (void*)bad, tmp})
            if (q) (void)hipFree(q);
        if (outputs)
            for (void* q : {(void*)poff, (void*)idx16, (void*)pval, (void*)cbase})
                if (q) (void)hipFree(q);
    };
    const auto* idx = static_cast<const uint32_t*>(A.t_idx);
    if (hipMalloc(&fills, sizeof(int64_t) * (nnz + 1)) || hipMalloc(&fscan, sizeof(int64_t) * (nnz + 1)) ||
        hipMalloc(&segf, sizeof(int64_t) * (nseg + 1))) {
        release(true);
        return -2;
    }
    hipLaunchKernelGGL(k_zpk_fills, dim3(grid1(nnz + 1)), dim3(256), 0, nullptr, nnz, idx, A.t_seg, nseg, fills);
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, fills, fscan, (int)(nnz + 1)) != hipSuccess ||
        hipMalloc(&tmp, tmpb ? tmpb : 1) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, fills, fscan, (int)(nnz + 1)) != hipSuccess) {
        release(true);
        return -2;
    }
    hipLaunchKernelGGL(k_zpk_segfill, dim3(grid1(nseg + 1)), dim3(256), 0, nullptr, nseg, A.t_seg, fscan, segf);
    std::vector<int64_t> hseg((size_t)nseg + 1), hf((size_t)nseg + 1), hp((size_t)nseg + 1, 0);
    if (hipMemcpy(hseg.data(), A.t_seg, sizeof(int64_t) * (nseg + 1), hipMemcpyDeviceToHost) ||
        hipMemcpy(hf.data(), segf, sizeof(int64_t) * (nseg + 1), hipMemcpyDeviceToHost)) {
        release(true);
        return -2;
    }
    for (int64_t q = 0; q < nseg; ++q) {
        const int64_t len = (hseg[q + 1] - hseg[q]) + (hf[q + 1] - hf[q]);
        hp[q + 1] = hp[q] + (len + 63) / 64 * 64;
    }
    const int64_t stored = hp[nseg];
    if ((double)(stored - nnz) > 0.03 * (double)nnz || stored >= (int64_t(1) << 32)) {
        release(true);
        return 1;
    }
    const int64_t nch = stored / 64;
    if (hipMalloc(&poff, sizeof(int64_t) * (nseg + 1)) || hipMalloc(&pcol, sizeof(int32_t) * (stored + 1)) ||
        hipMalloc(&prow, sizeof(uint16_t) * (stored + 1)) || hipMalloc(&pval, 16 * (size_t)(stored + 1)) ||
        hipMalloc(&idx16, sizeof(uint16_t) * (stored + 1)) ||
        hipMalloc(&cbase, sizeof(int32_t) * (nch + 1)) || hipMalloc(&bad, sizeof(int)) ||
        hipMemcpy(poff, hp.data(), sizeof(int64_t) * (nseg + 1), hipMemcpyHostToDevice) ||
        hipMemset(prow, 0, sizeof(uint16_t) * (stored + 1)) || hipMemset(pval, 0, 16 * (size_t)(stored + 1)) ||
        hipMemset(bad, 0, sizeof(int))) {
        release(true);
        return -2;
    }
    hipLaunchKernelGGL(k_zpk_scatter, dim3(grid1(nnz)), dim3(256), 0, nullptr, nnz, idx,
                       (const double2*)A.t_val, A.t_seg, nseg, fscan, poff, pcol, prow, pval);
    hipLaunchKernelGGL(k_zpk_pad, dim3(grid1(nseg)), dim3(256), 0, nullptr, nseg, A.t_seg, fscan, poff, pcol);
    hipLaunchKernelGGL(k_zpk_encode, dim3(grid1(stored)), dim3(256), 0, nullptr, stored, pcol, prow, idx16,
                       cbase, bad);
    int hbad = 1;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess || hbad != 0) {
        release(true);
        return -1;
    }
    release(false);
    (void)hipFree(A.t_idx);
    (void)hipFree(A.t_val);
    (void)hipFree(A.t_seg);
    A.t_idx = idx16;
    A.t_val = reinterpret_cast<double*>(pval);
    A.t_seg = poff;
    A.t_cbase = cbase;
    A.t_stored = stored;
    A.t_pk = true;
    return 0;
}

// Column-sorted tiles from the slice CSR (A.split): a stable segmented radix sort
// of each (slice, row block) segment by column, then idx / val gathered in that
// order; the slice CSR's columns and values are released.  0: built; 1: not
// applicable (slice wider than 2^20 columns, AHIP_ZSPLIT=csr); < 0: error (the
// CSR split is kept).
static int ztile_build(ZCsr& A) {
    static const bool off = [] {
        const char* e = getenv("AHIP_ZSPLIT");
        return e && std::strcmp(e, "csr") == 0;
    }();
    const int64_t n = A.n, nnz = A.nnz;
    if (off || A.s_w >= (int64_t(1) << 20) || nnz <= 0 || nnz >= (int64_t(1) << 32)) return 1;
    const int64_t nrb = (n + kTileRows - 1) / kTileRows, nseg = A.s_n * nrb;
    uint32_t *key = nullptr, *key2 = nullptr, *erow = nullptr, *perm = nullptr, *perm2 = nullptr;
    int64_t* seg = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    int rc = 0;
    auto cleanup = [&]() {
        for (void* q : {(void*)key, (void*)key2, (void*)erow, (void*)perm, (void*)perm2, (void*)seg, tmp})
            if (q) (void)hipFree(q);
    };
    const size_t eb = sizeof(uint32_t) * (size_t)nnz;
    if (hipMalloc(&key, eb) || hipMalloc(&key2, eb) || hipMalloc(&erow, eb) || hipMalloc(&perm, eb) ||
        hipMalloc(&perm2, eb) || hipMalloc(&seg, sizeof(int64_t) * (nseg + 1)) ||
        hipMalloc(&A.t_idx, eb) || hipMalloc(&A.t_val, 16 * (size_t)nnz)) {
        // (A.t_idx: the 20-B form's uint32 entries until ztile_pack)
        rc = -2;
    } else {
        if (A.s_col16)
            hipLaunchKernelGGL(k_ztile_keys<uint16_t>, dim3(grid1(n)), dim3(256), 0, nullptr, n, A.s_n, A.s_rp,
                               A.s_base, (const uint16_t*)A.s_col, key, erow, perm);
        else
            hipLaunchKernelGGL(k_ztile_keys<int32_t>, dim3(grid1(n)), dim3(256), 0, nullptr, n, A.s_n, A.s_rp,
                               A.s_base, (const int32_t*)A.s_col, key, erow, perm);
        hipLaunchKernelGGL(k_ztile_segs, dim3(grid1(nseg + 1)), dim3(256), 0, nullptr, n, A.s_n, nrb, A.s_rp,
                           A.s_base, seg);
        int bits = 1;
        while ((int64_t(1) << bits) < A.s_w) ++bits;
        if (hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tmpb, key, key2, perm, perm2, (int)nnz,
                                                        (int)nseg, seg, seg + 1, 0, bits) != hipSuccess ||
            hipMalloc(&tmp, tmpb ? tmpb : 1) != hipSuccess ||
            hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tmpb, key, key2, perm, perm2, (int)nnz,
                                                        (int)nseg, seg, seg + 1, 0, bits) != hipSuccess) {
            rc = -1;
        } else {
            hipLaunchKernelGGL(k_ztile_gather, dim3(grid1(nnz)), dim3(256), 0, nullptr, nnz, perm2, key2, erow,
                               (const double2*)A.s_val, static_cast<uint32_t*>(A.t_idx),
                               (double2*)A.t_val);
            if (hipDeviceSynchronize() != hipSuccess) rc = -1;
            if (rc == 0) {  // the segment bounds stay with the tiles; the 18-B form where it fits
                A.t_seg = seg;
                seg = nullptr;
                A.t_stored = nnz;
                if (ztile_pack(A, nseg) < 0) rc = 0;  // (an error leaves the 20-B form, still valid)
            }
            // the deterministic form's scale inputs (optional: without them
            // deterministic mode keeps the CSR split)
            int* dl = nullptr;
            if (rc == 0 && hipMalloc(&A.t_amax, sizeof(double) * (size_t)nseg) == hipSuccess &&
                hipMalloc(&A.t_xmax, sizeof(unsigned long long) * kZMaxBlocks) == hipSuccess &&
                hipMalloc(&dl, sizeof(int)) == hipSuccess && hipMemset(dl, 0, sizeof(int)) == hipSuccess) {
                hipLaunchKernelGGL(k_ztile_amax, dim3((unsigned)nseg), dim3(256), 0, nullptr, A.t_seg, A.t_val,
                                   A.t_amax);
                hipLaunchKernelGGL(k_zslice_lmax, dim3(grid1(n)), dim3(256), 0, nullptr, n, A.s_n, A.s_rp, dl);
                std::vector<double> am((size_t)nseg);
                int L = 0;
                if (hipMemcpy(am.data(), A.t_amax, sizeof(double) * (size_t)nseg, hipMemcpyDeviceToHost) ==
                        hipSuccess &&
                    hipMemcpy(&L, dl, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess) {
                    int hb = 0;
                    while (hb < 31 && (1ll << hb) <= (long long)L) ++hb;
                    bool scaled = true;
                    for (double a : am) scaled = scaled && (a == 0.0 || (a >= 0x1p-900 && a <= 0x1p900));
                    A.t_bits = std::min(51, 62 - hb);
                    A.t_det = scaled && A.t_bits >= 40 ? 1 : 0;
                }
            }
            if (dl) (void)hipFree(dl);
        }
    }
    cleanup();
    if (rc != 0) {
        if (A.t_idx) (void)hipFree(A.t_idx);
        if (A.t_val) (void)hipFree(A.t_val);
        if (A.t_seg) (void)hipFree(A.t_seg);
        if (A.t_cbase) (void)hipFree(A.t_cbase);
        A.t_seg = nullptr;
        A.t_cbase = nullptr;
        A.t_pk = false;
        if (A.t_amax) (void)hipFree(A.t_amax);
        if (A.t_xmax) (void)hipFree(A.t_xmax);
        A.t_idx = nullptr;
        A.t_val = nullptr;
        A.t_amax = nullptr;
        A.t_xmax = nullptr;
        A.t_det = 0;
        return rc;
    }
    if (A.t_det) {  // the tiles replace the slice CSR's columns and values
        (void)hipFree(A.s_col);
        (void)hipFree(A.s_val);
        A.s_col = nullptr;
        A.s_val = nullptr;
    }  // (else the CSR split stays: deterministic mode's fixed-order form of this operator)
    A.t_nrb = nrb;
    A.tile = true;
    return 0;
}

int zcsr_build_split(ZCsr& A) {
    static const bool off = [] {
        const char* e = getenv("AHIP_ZSPLIT");
        return e && e[0] == '0';
    }();
    const int64_t n = A.n;
    if (off || n < (int64_t(1) << 18) || A.nnz < 32 * n) return 1;
    // 4 slices while a quarter of x fits 2 MB (half an XCD's L2; slice s on XCDs
    // s and s + 4), else 8: tools/ztile_probe.hip at config 5 (n = 5e5), 0.215 ms
    // a product against 0.237 with 8 slices -- half the partial-sum traffic, the
    // same column density per tile
    // (AHIP_ZSLICES=2|4|8 forces the count: A/B of the partial-sum traffic
    // against x's L2 footprint)
    static const int force_ns = [] {
        const char* e = getenv("AHIP_ZSLICES");
        const int v = e ? atoi(e) : 0;
        return v == 2 || v == 4 || v == 8 ? v : 0;
    }();
    const int ns = force_ns ? force_ns : (n + 3) / 4 * 16 <= (int64_t(2) << 20) ? 4 : 8;
    const int64_t sw = (n + ns - 1) / ns;
    A.s_n = ns;
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
    if (hipMalloc(&cnt, sizeof(int32_t) * ns * (n + 1)) ||
        hipMalloc(&A.s_rp, sizeof(int32_t) * ns * (n + 1)) ||
        hipMalloc(&A.s_base, sizeof(int64_t) * (ns + 1)))
        return fail(-2);
    if (ns == 2)
        hipLaunchKernelGGL(k_zsplit_count<2>, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr, A.col, cnt);
    else if (ns == 4)
        hipLaunchKernelGGL(k_zsplit_count<4>, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr, A.col, cnt);
    else
        hipLaunchKernelGGL(k_zsplit_count<8>, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr, A.col, cnt);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, cnt, A.s_rp, (int)(n + 1));
    if (hipMalloc(&tmp, tmpb ? tmpb : 1)) return fail(-2);
    int64_t hb[kMaxSlices + 1];
    hb[0] = 0;
    for (int s = 0; s < ns; ++s) {
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
    if (hb[ns] != A.nnz) return fail(-1);
    if (hipMemcpy(A.s_base, hb, sizeof(int64_t) * (ns + 1), hipMemcpyHostToDevice)) return fail(-1);
    (void)hipFree(cnt);
    cnt = nullptr;
    (void)hipFree(tmp);
    tmp = nullptr;
    if (hipMalloc(&A.s_col, cb * (A.nnz ? A.nnz : 1)) || hipMalloc(&A.s_val, 16 * (A.nnz ? A.nnz : 1)) ||
        hipMalloc(&A.s_y, 16 * (size_t)ns * n))
        return fail(-2);
    const auto* v2 = reinterpret_cast<const double2*>(A.val);
    auto fill = [&](auto kern, auto* sc) {
        hipLaunchKernelGGL(kern, dim3(grid1(n)), dim3(256), 0, nullptr, n, sw, A.rowptr, A.col, v2, A.s_rp,
                           A.s_base, sc, (double2*)A.s_val);
    };
    if (A.s_col16)
        ns == 2 ? fill(k_zsplit_fill<2, uint16_t>, (uint16_t*)A.s_col)
        : ns == 4 ? fill(k_zsplit_fill<4, uint16_t>, (uint16_t*)A.s_col)
                  : fill(k_zsplit_fill<8, uint16_t>, (uint16_t*)A.s_col);
    else
        ns == 2 ? fill(k_zsplit_fill<2, int32_t>, (int32_t*)A.s_col)
        : ns == 4 ? fill(k_zsplit_fill<4, int32_t>, (int32_t*)A.s_col)
                  : fill(k_zsplit_fill<8, int32_t>, (int32_t*)A.s_col);
    if (hipDeviceSynchronize() != hipSuccess) return fail(-1);
    A.split = true;
    (void)ztile_build(A);  // optional: the CSR split stays if the tiles cannot be built
    return 0;
}

namespace {
// Entries a lane of the packed tile walk keeps in flight: 6 at 1,024 threads
// (62 VGPRs, under the 64 that 8 waves a SIMD allow), 4 at 256 / 512; A/B:
// AHIP_ZTILE_U=8 (256 threads) | 2, 4, 5, 7, 8 (1,024 threads; 8 through
// k_ztile_w8).  Config 5 in mode 3 at 1,024 threads, same-box pairs
// (profiles/r06ab_ztile_unroll_ab.txt): 6 solves 3% faster than 4, 1-2% than 5,
// 2% than 7 and 7% than 8; 2 is 8% slower than 4.
constexpr int kTileU1k = 6;
int tile_u(int dflt) {
    static const int u = [] {
        const char* e = getenv("AHIP_ZTILE_U");
        return e && e[0] >= '2' && e[0] <= '8' ? e[0] - '0' : 0;
    }();
    return u ? u : dflt;
}
// Threads a packed tile workgroup: 1,024 (default), AHIP_ZTILE_T=256 | 512
// for A/B.  The 64 KB of LDS row sums hold two workgroups a CU whatever their
// size, so the size sets the waves a SIMD that keep entries in flight: 2, 4 or
// 8.  Config 5 in mode 3, same box (profiles/r06v_ztile_threads_ab.txt): 2.60
// / 2.70 / 2.52 ms a solve at 256 / 512 / 1,024 threads (51 VGPRs in each).
int tile_t() {
    static const int t = [] {
        const char* e = getenv("AHIP_ZTILE_T");
        const int v = e ? atoi(e) : 1024;
        return v == 256 || v == 512 ? v : 1024;
    }();
    return t;
}

template <int S>
void split_partials(hipStream_t s, const ZCsr& A, const double2* x2, double2* yp, const int* gate) {
    const dim3 tg((unsigned)(S * A.t_nrb)), tb(256);
    if (A.tile && !deterministic()) {  // (LDS-atomic row sums: not bitwise run to run)
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, tg, tb, 0, s, A.n, A.s_w, A.t_seg, A.t_nrb, A.t_idx, A.t_cbase,
                               (const double2*)A.t_val, x2, yp, gate);
        };
        if (A.t_pk && tile_t() == 512) {
            hipLaunchKernelGGL((k_ztile<S, true, kTileU, 512>), tg, dim3(512), 0, s, A.n, A.s_w, A.t_seg,
                               A.t_nrb, A.t_idx, A.t_cbase, (const double2*)A.t_val, x2, yp, gate);
        } else if (A.t_pk && tile_t() == 1024) {
            auto go1k = [&](auto kern) {
                hipLaunchKernelGGL(kern, tg, dim3(1024), 0, s, A.n, A.s_w, A.t_seg, A.t_nrb, A.t_idx,
                                   A.t_cbase, (const double2*)A.t_val, x2, yp, gate);
            };
            const int u = tile_u(kTileU1k);
            if (u == 2)
                go1k(k_ztile<S, true, 2, 1024>);
            else if (u == 5)
                go1k(k_ztile<S, true, 5, 1024>);
            else if (u == 6)
                go1k(k_ztile<S, true, 6, 1024>);
            else if (u == 7)
                go1k(k_ztile<S, true, 7, 1024>);
            else if (u == 8)
                go1k(k_ztile_w8<S, 8>);
            else
                hipLaunchKernelGGL((k_ztile<S, true, kTileU, 1024>), tg, dim3(1024), 0, s, A.n,
                                   A.s_w, A.t_seg, A.t_nrb, A.t_idx, A.t_cbase,
                                   (const double2*)A.t_val, x2, yp, gate);
        } else if (A.t_pk) {  // 256 threads (U = 8: AHIP_ZTILE_U A/B, with AHIP_ZTILE_T=256)
            tile_u(kTileU) == 8 ? go(k_ztile<S, true, 8>) : go(k_ztile<S, true>);
        } else {
            go(k_ztile<S, false>);
        }
        return;
    }
    if (A.tile && A.t_det) {  // deterministic: the fixed-point tile form (else the CSR split, kept)
        // (t_xmax, like s_y, is the operator's scratch: one stream per ZCsr,
        // include/arpack_hip.h -- ADVICE r05)
        hipLaunchKernelGGL(k_zabsmax, dim3(kZMaxBlocks), dim3(256), 0, s, 2 * A.n,
                           reinterpret_cast<const double*>(x2), A.t_xmax, gate);
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, tg, tb, 0, s, A.n, A.s_w, A.t_seg, A.t_nrb, A.t_idx, A.t_cbase,
                               (const double2*)A.t_val, x2, yp, gate, A.t_amax, A.t_xmax, A.t_bits);
        };
        auto det1k = [&](auto kern) {  // the default tile's block size (bitwise the same sums)
            hipLaunchKernelGGL(kern, tg, dim3(1024), 0, s, A.n, A.s_w, A.t_seg, A.t_nrb, A.t_idx,
                               A.t_cbase, (const double2*)A.t_val, x2, yp, gate, A.t_amax, A.t_xmax,
                               A.t_bits);
        };
        if (A.t_pk && tile_t() == 1024 && tile_u(kTileU1k) == 4)
            det1k(k_ztile_det<S, true, 4, 1024>);
        else if (A.t_pk && tile_t() == 1024)  // six entries a lane: 64 VGPRs
            det1k(k_ztile_det<S, true, kTileU1k, 1024>);
        else if (A.t_pk)
            go(k_ztile_det<S, true>);
        else
            go(k_ztile_det<S, false>);
        return;
    }
    const int g = 1024;  // 128 workgroups a slice at S = 8 (tools/zspmv_split.hip)
    if (A.s_col16)
        hipLaunchKernelGGL((k_zsplit_spmv<S, uint16_t>), dim3(g), dim3(256), 0, s, A.n, A.s_w, A.s_rp,
                           A.s_base, (const uint16_t*)A.s_col, (const double2*)A.s_val, x2, yp, gate);
    else
        hipLaunchKernelGGL((k_zsplit_spmv<S, int32_t>), dim3(g), dim3(256), 0, s, A.n, A.s_w, A.s_rp,
                           A.s_base, (const int32_t*)A.s_col, (const double2*)A.s_val, x2, yp, gate);
}
}  // namespace

double zcsr_split_matrix_bytes(const ZCsr& A) {
    if (A.tile && A.t_pk) return 18.0 * (double)A.t_stored + 4.0 * (double)(A.t_stored / 64);
    return 20.0 * (double)A.nnz;
}

const double* zcsr_split_partials(hipStream_t s, const ZCsr& A, const double* x, const int* gate) {
    if (!A.split) return nullptr;
    const auto* x2 = reinterpret_cast<const double2*>(x);
    auto* yp = reinterpret_cast<double2*>(A.s_y);
    if (A.s_n == 2) split_partials<2>(s, A, x2, yp, gate);
    else if (A.s_n == 4) split_partials<4>(s, A, x2, yp, gate);
    else split_partials<8>(s, A, x2, yp, gate);
    return A.s_y;
}

void zcsr_split_spmv(hipStream_t s, const ZCsr& A, const double* x, double* y, const int* gate) {
    const auto* yp = reinterpret_cast<const double2*>(zcsr_split_partials(s, A, x, gate));
    auto* y2 = reinterpret_cast<double2*>(y);
    if (A.s_n == 2) hipLaunchKernelGGL(k_zsplit_combine<2>, dim3(2048), dim3(256), 0, s, A.n, yp, y2, gate);
    else if (A.s_n == 4) hipLaunchKernelGGL(k_zsplit_combine<4>, dim3(2048), dim3(256), 0, s, A.n, yp, y2, gate);
    else hipLaunchKernelGGL(k_zsplit_combine<8>, dim3(2048), dim3(256), 0, s, A.n, yp, y2, gate);
}

}  // namespace ahip::zdev
