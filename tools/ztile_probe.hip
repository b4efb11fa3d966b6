// PROBE: the config-5 column-sorted tile SpMV (csrc/zsplit.hip k_ztile) over
// its two layout parameters -- the number of column slices S (8 = one per XCD,
// x slice 1 MB; 4 = two XCDs per slice, x slice 2 MB, still inside a 4 MB L2,
// half the partial-sum traffic) and the rows of a tile RB (LDS 16 B a row:
// smaller tiles, more resident workgroups per CU, more bytes in flight) -- and
// the entries a lane keeps in flight (U).  Workgroup b: slice b % S, row block
// b / S, so with S = 4 slice s runs on XCDs s and s + 4 (b % 8).
// Output: ms per product (slices + combine of the S partials), checked against
// a host CSR product.
//   hipcc -O3 --offload-arch=gfx950 tools/ztile_probe.hip -o tools/ztile_probe && tools/ztile_probe
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

typedef double dv2 __attribute__((ext_vector_type(2)));

template <int S, int U, int T = 256>
__global__ __launch_bounds__(T) void k_tile(int64_t n, int64_t sw, int rb_rows,
                                              const int64_t* __restrict__ boff,
                                              const uint32_t* __restrict__ idx,
                                              const double2* __restrict__ val,
                                              const double2* __restrict__ x,
                                              double2* __restrict__ yp) {
    extern __shared__ double ylds[];  // 2 * rb_rows
    const int s = (int)(blockIdx.x % S);
    const int64_t r0 = (int64_t)(blockIdx.x / S) * rb_rows;
    const int rows = (int)((n - r0) < rb_rows ? (n - r0) : rb_rows);
    for (int i = threadIdx.x; i < 2 * rows; i += T) ylds[i] = 0.0;
    __syncthreads();
    const double2* xs = x + (int64_t)s * sw;
    const int64_t e0 = boff[blockIdx.x], e1 = boff[blockIdx.x + 1];
    int64_t e = e0 + threadIdx.x;
    for (; e + (U - 1) * T < e1; e += U * T) {
        uint32_t id[U];
        dv2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            id[u] = __builtin_nontemporal_load(&idx[e + u * T]);
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(val) + e + u * T);
        }
        double2 xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = xs[id[u] & 0xfffffu];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = (int)(id[u] >> 20);
            atomicAdd(&ylds[2 * r], v[u].x * xv[u].x - v[u].y * xv[u].y);
            atomicAdd(&ylds[2 * r + 1], v[u].x * xv[u].y + v[u].y * xv[u].x);
        }
    }
    for (; e < e1; e += T) {
        const uint32_t id = idx[e];
        const dv2 v = reinterpret_cast<const dv2*>(val)[e];
        const double2 xv = xs[id & 0xfffffu];
        const int r = (int)(id >> 20);
        atomicAdd(&ylds[2 * r], v.x * xv.x - v.y * xv.y);
        atomicAdd(&ylds[2 * r + 1], v.x * xv.y + v.y * xv.x);
    }
    __syncthreads();
    double2* y = yp + (int64_t)s * n + r0;
    for (int i = threadIdx.x; i < rows; i += T) y[i] = make_double2(ylds[2 * i], ylds[2 * i + 1]);
}

template <int S>
__global__ void k_combine(int64_t n, const double2* __restrict__ yp, double2* __restrict__ y) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        double2 a = yp[r];
#pragma unroll
        for (int s = 1; s < S; ++s) {
            const double2 b = yp[(int64_t)s * n + r];
            a.x += b.x;
            a.y += b.y;
        }
        y[r] = a;
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
    std::vector<double2> x(n), yref(n);
    for (int64_t i = 0; i < n; ++i) x[i] = make_double2(std::sin(0.001 * i), std::cos(0.002 * i));
    for (int64_t i = 0; i < n; ++i) {
        double re = 0, im = 0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            const double2 a = val[k], b = x[col[k]];
            re += a.x * b.x - a.y * b.y;
            im += a.x * b.y + a.y * b.x;
        }
        yref[i] = make_double2(re, im);
    }
    double2 *d_x, *d_yp, *d_y;
    CK(hipMalloc(&d_x, 16 * n));
    CK(hipMalloc(&d_yp, 16 * 8 * n));
    CK(hipMalloc(&d_y, 16 * n));
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
    auto probe = [&](auto SC, int RB) -> int {
        constexpr int S = decltype(SC)::value;
        const int64_t sw = (n + S - 1) / S;
        const int64_t nrb = (n + RB - 1) / RB;
        std::vector<int64_t> boff(S * nrb + 1, 0);
        std::vector<uint32_t> tidx;
        std::vector<double2> tval;
        tidx.reserve(nnz);
        tval.reserve(nnz);
        std::vector<std::vector<std::pair<uint32_t, double2>>> ent(S);
        for (int64_t rb = 0; rb < nrb; ++rb) {
            for (auto& e : ent) e.clear();
            for (int64_t r = rb * RB; r < std::min(n, (rb + 1) * RB); ++r)
                for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
                    const int s = (int)(col[k] / sw);
                    ent[s].push_back({(uint32_t)((r - rb * RB) << 20) | (uint32_t)(col[k] - s * sw), val[k]});
                }
            for (int s = 0; s < S; ++s) {
                boff[rb * S + s] = (int64_t)tidx.size();
                std::stable_sort(ent[s].begin(), ent[s].end(), [](const auto& a, const auto& b) {
                    return (a.first & 0xfffffu) < (b.first & 0xfffffu);
                });
                for (auto& pr : ent[s]) {
                    tidx.push_back(pr.first);
                    tval.push_back(pr.second);
                }
            }
        }
        boff[S * nrb] = (int64_t)tidx.size();
        int64_t* d_boff;
        uint32_t* d_tidx;
        double2* d_tval;
        CK(hipMalloc(&d_boff, 8 * boff.size()));
        CK(hipMalloc(&d_tidx, 4 * tidx.size()));
        CK(hipMalloc(&d_tval, 16 * tval.size()));
        CK(hipMemcpy(d_boff, boff.data(), 8 * boff.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_tidx, tidx.data(), 4 * tidx.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_tval, tval.data(), 16 * tval.size(), hipMemcpyHostToDevice));
        const unsigned grid = (unsigned)(S * nrb);
        const size_t lds = 16 * (size_t)RB;
        float t[3];
        int q = 0;
        auto one = [&](auto kern) {
            t[q++] = timeit([&] {
                kern<<<grid, 256, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp);
                k_combine<S><<<2048, 256>>>(n, d_yp, d_y);
            });
        };
        one(k_tile<S, 2>);
        one(k_tile<S, 4>);
        one(k_tile<S, 8>);
        float t512[2];
        {
            auto one512 = [&](auto kern, int qq) {
                t512[qq] = timeit([&] {
                    kern<<<grid, 512, lds>>>(n, sw, RB, d_boff, d_tidx, d_tval, d_x, d_yp);
                    k_combine<S><<<2048, 256>>>(n, d_yp, d_y);
                });
            };
            one512(k_tile<S, 2, 512>, 0);
            one512(k_tile<S, 4, 512>, 1);
        }
        const float tc = timeit([&] { k_combine<S><<<2048, 256>>>(n, d_yp, d_y); });
        std::vector<double2> y(n);
        CK(hipMemcpy(y.data(), d_y, 16 * n, hipMemcpyDeviceToHost));
        double err = 0, sc = 0;
        for (int64_t i = 0; i < n; ++i) {
            err = std::max(err, std::hypot(y[i].x - yref[i].x, y[i].y - yref[i].y));
            sc = std::max(sc, std::hypot(yref[i].x, yref[i].y));
        }
        printf("S %d RB %5d (%5u groups, LDS %2zu KB): U2 %.3f  U4 %.3f  U8 %.3f | T512 U2 %.3f U4 %.3f ms a "
               "product (combine %.3f)  rel err %.1e\n", S, RB, grid, lds / 1024, t[0], t[1], t[2], t512[0],
               t512[1], tc, err / sc);
        CK(hipFree(d_boff));
        CK(hipFree(d_tidx));
        CK(hipFree(d_tval));
        return 0;
    };
    for (int RB : {2048, 4096}) {
        if (probe(std::integral_constant<int, 8>{}, RB)) return 1;
        if (probe(std::integral_constant<int, 4>{}, RB)) return 1;
    }
    return 0;
}
