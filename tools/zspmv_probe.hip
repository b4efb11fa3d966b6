// PROBE of the config-5 complex SpMV (see k_probe below).  Setup copied from
// tools/zspmv_split.hip.
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


// Probe: what bounds the XCD-split kernel?  MODE 0 = the product as shipped;
// 1 = every gather folded into the first 4096 columns of the slice (64 KB of x:
// L1/L2-resident); 2 = no gather at all (x[0]); 3 = MODE 0 with the column
// loads issued one iteration ahead.  Same matrix stream in every mode.
template <int G, int MODE>
__global__ __launch_bounds__(256) void k_probe(int64_t n, int64_t sw, const int32_t* __restrict__ rps,
                                               const int64_t* __restrict__ base,
                                               const uint16_t* __restrict__ colr,
                                               const double2* __restrict__ val,
                                               const double2* __restrict__ x,
                                               double2* __restrict__ yp) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    const int s = (int)(blockIdx.x & 7);
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
        for (int64_t k = b0 + rp[r] + lane; k < k1; k += G) {
            const dv2 vv = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + k);
            int c = __builtin_nontemporal_load(&colr[k]);
            if (MODE == 1) c &= 4095;
            if (MODE == 2) c = 0;
            const double2 xv = xs[c];
            re += vv.x * xv.x - vv.y * xv.y;
            im += vv.x * xv.y + vv.y * xv.x;
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) {
            re += __shfl_xor(re, o, G);
            im += __shfl_xor(im, o, G);
        }
        if (lane == 0) y[r] = make_double2(re, im);
    }
}


// Column-sorted tiles: the entries of (row block of RB rows, column slice s) are
// sorted by column, so neighbouring lanes gather neighbouring x entries (a wave
// touches a few cache lines instead of 64); each entry's product is added into
// the block's row sums in LDS (ds_add_f64), written out once per block as the
// slice's partial y.  idx = row_local << 16 | slice-relative column.
template <int U>
__global__ __launch_bounds__(256) void k_ztile(int64_t n, int64_t sw, int rb_rows,
                                               const int64_t* __restrict__ boff,
                                               const uint32_t* __restrict__ idx,
                                               const double2* __restrict__ val,
                                               const double2* __restrict__ x,
                                               double2* __restrict__ yp) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    extern __shared__ double ylds[];  // 2 * rb_rows
    const int s = (int)(blockIdx.x & 7);
    const int64_t rb = blockIdx.x >> 3;
    const int64_t r0 = rb * rb_rows;
    const int rows = (int)((n - r0) < rb_rows ? (n - r0) : rb_rows);
    for (int i = threadIdx.x; i < 2 * rows; i += 256) ylds[i] = 0.0;
    __syncthreads();
    const double2* xs = x + (int64_t)s * sw;
    const int64_t e0 = boff[blockIdx.x], e1 = boff[blockIdx.x + 1];
    int64_t e = e0 + threadIdx.x;
    for (; e + (U - 1) * 256 < e1; e += U * 256) {
        uint32_t id[U];
        dv2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            id[u] = __builtin_nontemporal_load(&idx[e + u * 256]);
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + e + u * 256);
        }
        double2 xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = xs[id[u] & 0xffffu];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = (int)(id[u] >> 16);
            atomicAdd(&ylds[2 * r], v[u].x * xv[u].x - v[u].y * xv[u].y);
            atomicAdd(&ylds[2 * r + 1], v[u].x * xv[u].y + v[u].y * xv[u].x);
        }
    }
    for (; e < e1; e += 256) {
        const uint32_t id = idx[e];
        const dv2 v = reinterpret_cast<const dv2*>(val)[e];
        const double2 xv = xs[id & 0xffffu];
        const int r = (int)(id >> 16);
        atomicAdd(&ylds[2 * r], v.x * xv.x - v.y * xv.y);
        atomicAdd(&ylds[2 * r + 1], v.x * xv.y + v.y * xv.x);
    }
    __syncthreads();
    double2* y = yp + (int64_t)s * n + r0;
    for (int i = threadIdx.x; i < rows; i += 256) y[i] = make_double2(ylds[2 * i], ylds[2 * i + 1]);
}


// k_ztile with the next batch's index/value loads issued before this batch's
// gathers (software pipelined) and a block of T threads
template <int U, int T>
__global__ __launch_bounds__(T) void k_ztile_pipe(int64_t n, int64_t sw, int rb_rows,
                                                  const int64_t* __restrict__ boff,
                                                  const uint32_t* __restrict__ idx,
                                                  const double2* __restrict__ val,
                                                  const double2* __restrict__ x,
                                                  double2* __restrict__ yp) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    extern __shared__ double ylds[];
    const int s = (int)(blockIdx.x & 7);
    const int64_t r0 = (int64_t)(blockIdx.x >> 3) * rb_rows;
    const int rows = (int)((n - r0) < rb_rows ? (n - r0) : rb_rows);
    for (int i = threadIdx.x; i < 2 * rows; i += T) ylds[i] = 0.0;
    __syncthreads();
    const double2* xs = x + (int64_t)s * sw;
    const int64_t e0 = boff[blockIdx.x], e1 = boff[blockIdx.x + 1];
    int64_t e = e0 + threadIdx.x;
    uint32_t id[U];
    dv2 v[U];
    auto load = [&](int64_t b) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = b + u * T;
            id[u] = q < e1 ? __builtin_nontemporal_load(&idx[q]) : 0u;
            v[u] = q < e1 ? __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + q) : dv2{0.0, 0.0};
        }
    };
    load(e);
    for (; e < e1; e += U * T) {
        uint32_t idc[U];
        dv2 vc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { idc[u] = id[u]; vc[u] = v[u]; }
        load(e + U * T);
        double2 xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = xs[idc[u] & 0xffffu];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (e + u * T < e1) {
                const int r = (int)(idc[u] >> 16);
                atomicAdd(&ylds[2 * r], vc[u].x * xv[u].x - vc[u].y * xv[u].y);
                atomicAdd(&ylds[2 * r + 1], vc[u].x * xv[u].y + vc[u].y * xv[u].x);
            }
        }
    }
    __syncthreads();
    double2* y = yp + (int64_t)s * n + r0;
    for (int i = threadIdx.x; i < rows; i += T) y[i] = make_double2(ylds[2 * i], ylds[2 * i + 1]);
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
    double2 *d_vals, *d_x, *d_yp;
    int32_t* d_rps;
    int64_t* d_base;
    uint16_t* d_colr;
    CK(hipMalloc(&d_rps, 4 * 8 * (n + 1)));
    CK(hipMalloc(&d_base, 8 * 8));
    CK(hipMalloc(&d_colr, 2 * nnz));
    CK(hipMalloc(&d_vals, 16 * nnz));
    CK(hipMalloc(&d_x, 16 * n));
    CK(hipMalloc(&d_yp, 16 * 8 * n));
    CK(hipMemcpy(d_rps, rps.data(), 4 * 8 * (n + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_base, base.data(), 8 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_colr, colr.data(), 2 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vals, vals.data(), 16 * nnz, hipMemcpyHostToDevice));
    std::vector<double2> x(n);
    for (int64_t i = 0; i < n; ++i) x[i] = make_double2(std::sin(0.001 * i), std::cos(0.002 * i));
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
    const double stream = 18.0 * nnz + 4.0 * 8 * (n + 1) + 16.0 * 8 * n;  // val + colr + rps + partials
    // column-sorted tile layout (block b = rb * 8 + s), for RB = 2048 and 4096
    for (int RB : {4096, 8192}) {
        for (int sorted = 0; sorted < 2; ++sorted) {
            const int64_t nrb = (n + RB - 1) / RB;
            std::vector<int64_t> boff(8 * nrb + 1, 0);
            std::vector<uint32_t> tidx;
            std::vector<double2> tval;
            tidx.reserve(nnz);
            tval.reserve(nnz);
            for (int64_t rb = 0; rb < nrb; ++rb)
                for (int s = 0; s < 8; ++s) {
                    const int64_t b = rb * 8 + s;
                    boff[b] = (int64_t)tidx.size();
                    std::vector<std::pair<uint32_t, double2>> ent;
                    for (int64_t r = rb * RB; r < std::min(n, (rb + 1) * RB); ++r)
                        for (int64_t k = base[s] + rps[s * (n + 1) + r]; k < base[s] + rps[s * (n + 1) + r + 1]; ++k)
                            ent.push_back({(uint32_t)((r - rb * RB) << 16) | colr[k], vals[k]});
                    if (sorted)
                        std::stable_sort(ent.begin(), ent.end(), [](const auto& a, const auto& b2) {
                            return (a.first & 0xffffu) < (b2.first & 0xffffu);
                        });
                    for (auto& pr : ent) {
                        tidx.push_back(pr.first);
                        tval.push_back(pr.second);
                    }
                }
            boff[8 * nrb] = (int64_t)tidx.size();
            int64_t* d_boff;
            uint32_t* d_tidx;
            double2* d_tval;
            CK(hipMalloc(&d_boff, 8 * boff.size()));
            CK(hipMalloc(&d_tidx, 4 * tidx.size()));
            CK(hipMalloc(&d_tval, 16 * tval.size()));
            CK(hipMemcpy(d_boff, boff.data(), 8 * boff.size(), hipMemcpyHostToDevice));
            CK(hipMemcpy(d_tidx, tidx.data(), 4 * tidx.size(), hipMemcpyHostToDevice));
            CK(hipMemcpy(d_tval, tval.data(), 16 * tval.size(), hipMemcpyHostToDevice));
            const unsigned grid = (unsigned)(8 * nrb);
            const size_t lds = 16 * (size_t)RB;
            auto runt = [&](auto kern) {
                return timeit([&] {
                    kern<<<grid, 256, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp);
                });
            };
            if (lds > 65536) {
                CK(hipFuncSetAttribute((const void*)k_ztile<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                CK(hipFuncSetAttribute((const void*)k_ztile<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                CK(hipFuncSetAttribute((const void*)k_ztile<6>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            }
            const float t1 = runt(k_ztile<2>), t4 = runt(k_ztile<4>), t8 = runt(k_ztile<6>);
            if (RB == 4096 && sorted) {
                const float p2 = timeit([&] { k_ztile_pipe<2, 256><<<grid, 256, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp); });
                const float p4 = timeit([&] { k_ztile_pipe<4, 256><<<grid, 256, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp); });
                const float q4 = timeit([&] { k_ztile_pipe<4, 512><<<grid, 512, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp); });
                const float q2 = timeit([&] { k_ztile_pipe<2, 512><<<grid, 512, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp); });
                const float w4 = timeit([&] { k_ztile_pipe<4, 1024><<<grid, 1024, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp); });
                printf("pipelined RB 4096 sorted: T256 U2 %.3f U4 %.3f | T512 U2 %.3f U4 %.3f | T1024 U4 %.3f ms\n", p2, p4, q2, q4, w4);
            }
            // check against the CSR-split probe (MODE 0) partials
            std::vector<double2> ya(8 * n), yb(8 * n);
            CK(hipMemcpy(ya.data(), d_yp, 16 * 8 * n, hipMemcpyDeviceToHost));
            k_probe<8, 0><<<1024, 256>>>(n, sw, d_rps, d_base, d_colr, d_vals, d_x, d_yp);
            CK(hipMemcpy(yb.data(), d_yp, 16 * 8 * n, hipMemcpyDeviceToHost));
            double err = 0, sc = 0;
            for (int64_t i = 0; i < 8 * n; ++i) {
                err = std::max(err, std::hypot(ya[i].x - yb[i].x, ya[i].y - yb[i].y));
                sc = std::max(sc, std::hypot(yb[i].x, yb[i].y));
            }
            printf("tile RB %d %s: U2 %.3f  U4 %.3f  U6 %.3f ms  (max rel diff %.1e)\n", RB,
                   sorted ? "column-sorted" : "row order   ", t1, t4, t8, err / sc);
            CK(hipFree(d_boff));
            CK(hipFree(d_tidx));
            CK(hipFree(d_tval));
        }
    }
    for (int g : {1024, 2048, 4096}) {
        auto run = [&](auto kern) {
            return timeit([&] { kern<<<g, 256>>>(n, sw, d_rps, d_base, d_colr, d_vals, d_x, d_yp); });
        };
        const float m0 = run(k_probe<8, 0>), m1 = run(k_probe<8, 1>), m2 = run(k_probe<8, 2>);
        const float m4 = run(k_probe<4, 0>), m16 = run(k_probe<16, 0>);
        printf("grid %5d  G8: gather %.3f  local-gather %.3f  no-gather %.3f ms | G4 %.3f G16 %.3f  "
               "(stream %.0f GB/s at no-gather)\n", g, m0, m1, m2, m4, m16, stream / m2 / 1e6);
    }
    return 0;
}
