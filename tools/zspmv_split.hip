// Config-5 complex SpMV (n = 5e5, ~100 random columns per row, complex128):
// one wave per row over the whole x (x = 8 MB does not fit an XCD's 4 MB L2,
// so the random gathers miss to the Infinity Cache) against an XCD column
// split: the columns are cut into 8 slices of 1 MB of x, workgroup b works on
// slice b % 8 (the hardware deals workgroups round-robin over the 8 XCDs, so
// every slice's gathers stay in one XCD's L2), 16 lanes per row, a partial y
// per slice, then a fixed-order combine of the 8 partials.
//   hipcc -O3 --offload-arch=gfx950 tools/zspmv_split.hip -o tools/zspmv_split && tools/zspmv_split
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);           \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double wsum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void k_zcsr(int64_t n, const int64_t* __restrict__ rp,
                                              const int32_t* __restrict__ col,
                                              const double2* __restrict__ val,
                                              const double2* __restrict__ x, double2* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
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

// slice s = blockIdx % 8; G lanes per row; rows of the slice CSR (rp32: offsets
// into the slice's own arrays), 16-bit columns relative to the slice start
template <int G, bool XCD = true>
__global__ __launch_bounds__(256) void k_zcsr_split(int64_t n, int64_t sw,
                                                    const int32_t* __restrict__ rps,  // 8 x (n+1)
                                                    const int64_t* __restrict__ base, // 8 slice offsets
                                                    const uint16_t* __restrict__ colr,
                                                    const double2* __restrict__ val,
                                                    const double2* __restrict__ x,
                                                    double2* __restrict__ yp) {       // 8 x n
    // XCD: slice = blockIdx % 8 (the XCD the workgroup lands on); else contiguous
    // block ranges per slice (every XCD gathers from every slice: control)
    const int s = XCD ? (int)(blockIdx.x & 7) : (int)(blockIdx.x / (gridDim.x >> 3));
    const int64_t q = XCD ? blockIdx.x >> 3 : blockIdx.x % (gridDim.x >> 3), nq = gridDim.x >> 3;
    const int lane = threadIdx.x & (G - 1);
    const int64_t rows_per_block = 256 / G;
    const int32_t* rp = rps + (int64_t)s * (n + 1);
    const int64_t b0 = base[s];
    const double2* xs = x + (int64_t)s * sw;
    double2* y = yp + (int64_t)s * n;
    for (int64_t r = q * rows_per_block + threadIdx.x / G; r < n; r += nq * rows_per_block) {
        double re = 0.0, im = 0.0;
        const int64_t k1 = b0 + rp[r + 1];
        for (int64_t k = b0 + rp[r] + lane; k < k1; k += G) {
            typedef double dv2 __attribute__((ext_vector_type(2)));
            const dv2 vv = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + k);
            const double2 v = make_double2(vv.x, vv.y);
            const double2 p = cmul(v, xs[__builtin_nontemporal_load(&colr[k])]);
            re += p.x;
            im += p.y;
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) {
            re += __shfl_xor(re, o, G);
            im += __shfl_xor(im, o, G);
        }
        if (lane == 0) y[r] = make_double2(re, im);
    }
}

// as k_zcsr_split, two entries per lane per iteration (both gathers in flight)
template <int G>
__global__ __launch_bounds__(256) void k_zcsr_split2(int64_t n, int64_t sw,
                                                     const int32_t* __restrict__ rps,
                                                     const int64_t* __restrict__ base,
                                                     const uint16_t* __restrict__ colr,
                                                     const double2* __restrict__ val,
                                                     const double2* __restrict__ x,
                                                     double2* __restrict__ yp) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    const int s = blockIdx.x & 7;
    const int64_t q = blockIdx.x >> 3, nq = gridDim.x >> 3;
    const int lane = threadIdx.x & (G - 1);
    const int64_t rows_per_block = 256 / G;
    const int32_t* rp = rps + (int64_t)s * (n + 1);
    const int64_t b0 = base[s];
    const double2* xs = x + (int64_t)s * sw;
    double2* y = yp + (int64_t)s * n;
    for (int64_t r = q * rows_per_block + threadIdx.x / G; r < n; r += nq * rows_per_block) {
        double re = 0.0, im = 0.0;
        const int64_t k1 = b0 + rp[r + 1];
        for (int64_t k = b0 + rp[r] + lane; k < k1; k += 2 * G) {
            const bool two = k + G < k1;
            const int c0 = __builtin_nontemporal_load(&colr[k]);
            const int c1 = two ? (int)__builtin_nontemporal_load(&colr[k + G]) : c0;
            const dv2 v0 = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + k);
            const dv2 v1 = two ? __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + k + G) : dv2{0.0, 0.0};
            const double2 x0 = xs[c0], x1 = xs[c1];
            re += v0.x * x0.x - v0.y * x0.y;
            im += v0.x * x0.y + v0.y * x0.x;
            re += v1.x * x1.x - v1.y * x1.y;
            im += v1.x * x1.y + v1.y * x1.x;
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) {
            re += __shfl_xor(re, o, G);
            im += __shfl_xor(im, o, G);
        }
        if (lane == 0) y[r] = make_double2(re, im);
    }
}

// SELL-64 per column slice: within windows of 4096 rows the slice's rows are
// sorted by length and cut into chunks of 64 (one row per lane); chunk c has
// width w_c, entries column-step-major (val[o_c + k*64 + lane]), the chunk's
// original rows in perm; no row pointers on the critical path.  Workgroup b
// takes slice b % 8; its waves take the slice's chunks.
template <int U>
__global__ __launch_bounds__(256) void k_zsell_split(int64_t n, int64_t sw,
                                                     const int64_t* __restrict__ cbase,  // 9: first chunk of each slice
                                                     const int64_t* __restrict__ coff,   // chunk offsets (+1)
                                                     const int32_t* __restrict__ perm,   // 64 per chunk
                                                     const uint16_t* __restrict__ colr,
                                                     const double2* __restrict__ val,
                                                     const double2* __restrict__ x,
                                                     double2* __restrict__ yp) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    const int s = blockIdx.x & 7;
    const int64_t q = blockIdx.x >> 3, nq = gridDim.x >> 3;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double2* xs = x + (int64_t)s * sw;
    double2* y = yp + (int64_t)s * n;
    for (int64_t c = cbase[s] + q * 4 + wave; c < cbase[s + 1]; c += nq * 4) {
        const int64_t o = coff[c];
        const int w = (int)((coff[c + 1] - o) >> 6);
        double re = 0.0, im = 0.0;
        int k = 0;
        for (; k + U <= w; k += U) {
            int cl[U];
            dv2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cl[u] = __builtin_nontemporal_load(&colr[o + (int64_t)(k + u) * 64 + lane]);
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + o + (int64_t)(k + u) * 64 + lane);
            }
            double2 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) xv[u] = xs[cl[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                re += v[u].x * xv[u].x - v[u].y * xv[u].y;
                im += v[u].x * xv[u].y + v[u].y * xv[u].x;
            }
        }
        for (; k < w; ++k) {
            const int cl = __builtin_nontemporal_load(&colr[o + (int64_t)k * 64 + lane]);
            const dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + o + (int64_t)k * 64 + lane);
            const double2 xv = xs[cl];
            re += v.x * xv.x - v.y * xv.y;
            im += v.x * xv.y + v.y * xv.x;
        }
        const int r = perm[c * 64 + lane];
        if (r >= 0) y[r] = make_double2(re, im);
    }
}

__global__ void k_combine8(int64_t n, const double2* __restrict__ yp, double2* __restrict__ y) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        double2 a[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) a[s] = yp[(int64_t)s * n + r];
        const double re = ((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x));
        const double im = ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y));
        y[r] = make_double2(re, im);
    }
}

static uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

int main() {
    const int64_t n = 500000, per = 100;
    // host CSR: sorted random columns (duplicates merged), diagonal present
    std::vector<int64_t> rp(n + 1, 0);
    std::vector<int32_t> col;
    std::vector<double2> val;
    col.reserve(n * (per + 1));
    val.reserve(n * (per + 1));
    for (int64_t i = 0; i < n; ++i) {
        std::vector<uint32_t> c(per + 1);
        for (int k = 0; k < per; ++k) c[k] = mix32(mix32((uint32_t)i ^ 5u) + k * 0x9E3779B9u) % n;
        c[per] = (uint32_t)i;
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (uint32_t cc : c) {
            col.push_back((int32_t)cc);
            const uint32_t h = mix32(cc * 2654435761u ^ (uint32_t)i);
            val.push_back(make_double2((double)(h >> 21) * 0x1p-10 - 1.0 + (cc == i ? 100.0 : 0.0),
                                       (double)(mix32(h) >> 21) * 0x1p-10 - 1.0));
        }
        rp[i + 1] = (int64_t)col.size();
    }
    const int64_t nnz = rp[n];
    // column split into 8 slices
    const int64_t sw = (n + 7) / 8;
    std::vector<int32_t> rps(8 * (n + 1), 0);
    std::vector<int64_t> base(8, 0);
    std::vector<uint16_t> colr(nnz);
    std::vector<double2> vals(nnz);
    {
        std::vector<int64_t> cnt(8, 0);
        for (int64_t k = 0; k < nnz; ++k) cnt[col[k] / sw]++;
        for (int s = 1; s < 8; ++s) base[s] = base[s - 1] + cnt[s - 1];
        std::vector<int64_t> pos(base);
        for (int64_t i = 0; i < n; ++i) {
            for (int s = 0; s < 8; ++s) rps[s * (n + 1) + i] = (int32_t)(pos[s] - base[s]);
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int s = col[k] / sw;
                colr[pos[s]] = (uint16_t)(col[k] - s * sw);
                vals[pos[s]] = val[k];
                pos[s]++;
            }
        }
        for (int s = 0; s < 8; ++s) rps[s * (n + 1) + n] = (int32_t)(pos[s] - base[s]);
    }
    // SELL-64 per slice (padding entries: column 0, value 0)
    std::vector<int64_t> cbase(9, 0), coff;
    std::vector<int32_t> perm;
    std::vector<uint16_t> scol;
    std::vector<double2> sval;
    {
        const int64_t win = 4096;
        for (int s = 0; s < 8; ++s) {
            cbase[s] = (int64_t)coff.size();
            for (int64_t r0 = 0; r0 < n; r0 += win) {
                const int64_t r1 = std::min(n, r0 + win);
                std::vector<int64_t> rows;
                for (int64_t r = r0; r < r1; ++r) rows.push_back(r);
                auto len = [&](int64_t r) { return (int64_t)rps[s * (n + 1) + r + 1] - rps[s * (n + 1) + r]; };
                std::stable_sort(rows.begin(), rows.end(), [&](int64_t a, int64_t b) { return len(a) > len(b); });
                for (size_t c0 = 0; c0 < rows.size(); c0 += 64) {
                    const int64_t w = len(rows[c0]);
                    const int64_t o = (int64_t)sval.size();
                    coff.push_back(o);
                    sval.resize(o + w * 64, make_double2(0.0, 0.0));
                    scol.resize(o + w * 64, 0);
                    for (int l = 0; l < 64; ++l) {
                        if (c0 + l >= rows.size()) { perm.push_back(-1); continue; }
                        const int64_t r = rows[c0 + l];
                        perm.push_back((int32_t)r);
                        const int64_t kb = base[s] + rps[s * (n + 1) + r];
                        for (int64_t k = 0; k < len(r); ++k) {
                            sval[o + k * 64 + l] = vals[kb + k];
                            scol[o + k * 64 + l] = colr[kb + k];
                        }
                    }
                }
            }
        }
        cbase[8] = (int64_t)coff.size();
        coff.push_back((int64_t)sval.size());
        printf("SELL split: %ld chunks, padding %.1f%%\n", (long)cbase[8],
               100.0 * ((double)sval.size() / (double)nnz - 1.0));
    }
    int64_t *d_cbase, *d_coff;
    int32_t* d_perm;
    uint16_t* d_scol;
    double2* d_sval;
    CK(hipMalloc(&d_cbase, 8 * 9));
    CK(hipMalloc(&d_coff, 8 * coff.size()));
    CK(hipMalloc(&d_perm, 4 * perm.size()));
    CK(hipMalloc(&d_scol, 2 * scol.size()));
    CK(hipMalloc(&d_sval, 16 * sval.size()));
    CK(hipMemcpy(d_cbase, cbase.data(), 8 * 9, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_coff, coff.data(), 8 * coff.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_perm, perm.data(), 4 * perm.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_scol, scol.data(), 2 * scol.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sval, sval.data(), 16 * sval.size(), hipMemcpyHostToDevice));
    std::vector<double2> x(n);
    for (int64_t i = 0; i < n; ++i) x[i] = make_double2(std::sin(0.001 * i), std::cos(0.002 * i));
    int64_t *d_rp, *d_base;
    int32_t *d_col, *d_rps;
    uint16_t* d_colr;
    double2 *d_val, *d_vals, *d_x, *d_y, *d_y2, *d_yp;
    CK(hipMalloc(&d_rp, 8 * (n + 1)));
    CK(hipMalloc(&d_col, 4 * nnz));
    CK(hipMalloc(&d_val, 16 * nnz));
    CK(hipMalloc(&d_rps, 4 * 8 * (n + 1)));
    CK(hipMalloc(&d_base, 8 * 8));
    CK(hipMalloc(&d_colr, 2 * nnz));
    CK(hipMalloc(&d_vals, 16 * nnz));
    CK(hipMalloc(&d_x, 16 * n));
    CK(hipMalloc(&d_y, 16 * n));
    CK(hipMalloc(&d_y2, 16 * n));
    CK(hipMalloc(&d_yp, 16 * 8 * n));
    CK(hipMemcpy(d_rp, rp.data(), 8 * (n + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), 4 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_val, val.data(), 16 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_rps, rps.data(), 4 * 8 * (n + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_base, base.data(), 8 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_colr, colr.data(), 2 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vals, vals.data(), 16 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), 16 * n, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto f) {
        f();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) f();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 20;
    };
    const double algo = 20.0 * nnz + 8.0 * (n + 1) + 32.0 * n;  // val + col + rowptr + x + y
    const float t0 = timeit([&] { k_zcsr<<<65536, 256>>>(n, d_rp, d_col, d_val, d_x, d_y); });
    printf("nnz %ld  wave-per-row     %.3f ms  %.0f GB/s algorithmic\n", (long)nnz, t0, algo / t0 / 1e6);
    std::vector<double2> y0(n), y1(n);
    CK(hipMemcpy(y0.data(), d_y, 16 * n, hipMemcpyDeviceToHost));
    for (int g : {256, 512, 1024, 2048}) {
        auto chk = [&]() {
            (void)hipMemcpy(y1.data(), d_y2, 16 * n, hipMemcpyDeviceToHost);
            double err = 0, sc = 0;
            for (int64_t i = 0; i < n; ++i) {
                err = std::max(err, std::hypot(y1[i].x - y0[i].x, y1[i].y - y0[i].y));
                sc = std::max(sc, std::hypot(y0[i].x, y0[i].y));
            }
            return err / sc;
        };
        auto run = [&](auto kern) {
            return timeit([&] {
                kern<<<g, 256>>>(n, sw, d_rps, d_base, d_colr, d_vals, d_x, d_yp);
                k_combine8<<<2048, 256>>>(n, d_yp, d_y2);
            });
        };
        const float a4 = run(k_zcsr_split<4>), a8 = run(k_zcsr_split<8>), a16 = run(k_zcsr_split<16>);
        const float b4 = run(k_zcsr_split2<4>), b8 = run(k_zcsr_split2<8>);
        const double e = chk();
        printf("grid %5d  G4 %.3f  G8 %.3f  G16 %.3f  | x2: G4 %.3f  G8 %.3f ms  (max rel diff %.1e)\n", g, a4,
               a8, a16, b4, b8, e);
        auto runs = [&](auto kern) {
            return timeit([&] {
                kern<<<g, 256>>>(n, sw, d_cbase, d_coff, d_perm, d_scol, d_sval, d_x, d_yp);
                k_combine8<<<2048, 256>>>(n, d_yp, d_y2);
            });
        };
        const float s2 = runs(k_zsell_split<2>), s4 = runs(k_zsell_split<4>), s8 = runs(k_zsell_split<8>);
        const float nx = run(k_zcsr_split<8, false>);
        printf("           CSR split G8 without the XCD alignment (control) %.3f ms\n", nx);
        const double e2 = chk();
        printf("           SELL split U2 %.3f  U4 %.3f  U8 %.3f ms  (max rel diff %.1e)\n", s2, s4, s8, e2);
    }
    return 0;
}
