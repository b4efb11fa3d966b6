// HIP kernels (gfx950 / CDNA4) for the n-length half of the IRL/IRA cycle.
//
// All of these are HBM-bandwidth bound (<= 2 flop/byte): the
// design goal is one coalesced pass over V per Gram-Schmidt sweep, with every
// reduction done as per-block partials (fixed order, no float atomics, so the
// result is bitwise reproducible run to run) plus a single-block finalize.
//
//   place      v_j = r/rnorm                          SRC/dsaitr.f:438-464
//   dots       [V' u ; w' u]   (CGS coefficients)     SRC/dsaitr.f:551-575
//   update     r = r - V c, fused with the DGKS        SRC/dsaitr.f:582-583,
//              coefficients [V' r ; r' r] of the       680-692 (speculative: the
//              NEXT sweep, which the reference takes   reference re-orthogonalises
//              in ~99.8% of steps)                     in 430 of 431 steps)
//   finalize   partial sums -> scalars + the DGKS decision (0.717 rule)
//   vq_update  V <- V*Q, r <- sigma*r + beta*v_{kev+1} SRC/dsapps.f:450-493
//   larnv      dlarnv(idist=2) continuation on device  SRC/dgetv0.f:234-236
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "device.hpp"
#include "passes.hpp"
#include "reduce.hpp"
#include "finalize.hpp"

namespace ahip::dev {

namespace {

constexpr double kSafminD = DBL_MIN;

// ------------------------------------------------------------------ place ---
template <class R>
__global__ __launch_bounds__(kBlock) void k_place(int64_t n, const R* __restrict__ r,
                                                  R* __restrict__ vcol, R* __restrict__ copy1,
                                                  R* __restrict__ sc, LzState* __restrict__ st,
                                                  int j) {
    if (st->abort) return;
    const double rn = st->rnorm;
    if (!(rn > 0.0)) {  // invariant subspace: restart needed (SRC/dsaitr.f:378)
        if (blockIdx.x == 0 && threadIdx.x == 0) { st->abort = 1; st->abort_j = j; }
        return;
    }
    // v = r * (1/rnorm), or dlascl's careful factors when rnorm < safmin
    double m0 = 1.0 / rn, m1 = 1.0, m2 = 1.0;
    if (rn < kSafminD) {
        // dlascl('G', cfrom=rn, cto=1): rn*safmin underflows, so scale up first
        const double big = 1.0 / kSafminD;
        m0 = big;
        const double c2 = rn * big;
        m1 = 1.0 / c2;
        m2 = 1.0;
    }
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const R v = (R)((double)r[i] * m0 * m1 * m2);
        vcol[i] = v;
        if (copy1) copy1[i] = v;
        if (sc) sc[i] = (R)((double)sc[i] * m0 * m1 * m2);
    }
}

// ------------------------------------------------------------------- dots ---
// Exact compile-time column count J (branch-free unrolled loads: all J column
// loads of a row are in flight together).  WM: 0 no w'u, 1 w == u, 2 w != u.
template <class R, int J, int WM, int POL = kPolNt>
__global__ __launch_bounds__(kBlock) void k_dots(int64_t n, int j0, const R* __restrict__ V,
                                                 int64_t ld, const R* __restrict__ u,
                                                 const R* __restrict__ w,
                                                 double* __restrict__ part, int pstride, int wslot,
                                                 const LzState* __restrict__ st, int gate) {
    if (gate_closed(st, gate)) return;
    double acc[J > 0 ? J : 1];
#pragma unroll
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    double aw = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const R* Vb = V + (int64_t)j0 * ld;
    // Software-pipelined: the next row's J+1 loads are issued before the
    // current row is consumed.  Without it the compiler serialises each
    // load->FMA pair for some J (26..29 here: one load in flight per wave,
    // 4.1 TB/s measured); the per-thread row order -- hence the rounding -- is
    // unchanged.
    constexpr int JL = J > 0 ? J : 1;
    double cur[JL], cu = 0.0, cw = 0.0;
    auto load = [&](int64_t it, double (&dst)[JL], double& du, double& dw) {
        const int64_t r = POL == kPolNtRev ? n - 1 - it : it;  // see VPol
#pragma unroll
        for (int k = 0; k < J; ++k) dst[k] = vld<POL>(Vb + r + (int64_t)k * ld);
        du = u[r];
        if constexpr (WM == 2) dw = w[r];
    };
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) load(i, cur, cu, cw);
    for (; i < n; i += stride) {
        double nxt[JL], nu = 0.0, nw = 0.0;
        if (i + stride < n) load(i + stride, nxt, nu, nw);
        if constexpr (WM == 1) aw += cu * cu;
        if constexpr (WM == 2) aw += cw * cu;
#pragma unroll
        for (int k = 0; k < J; ++k) acc[k] += cur[k] * cu;
#pragma unroll
        for (int k = 0; k < J; ++k) cur[k] = nxt[k];
        cu = nu;
        cw = nw;
    }
    constexpr int JJ = J > 0 ? J : 1;
    block_partials<JJ>(acc, J, aw, WM != 0, part, j0, wslot);
}

// ----------------------------------------------------------------- update ---
// rout = rin - V(:,0:J) c ; SPEC: partials of [V' rout ; rout' rout] from the
// same pass (the V row stays in registers: one HBM read of V serves both).
// POL = kPolNtRev: sweep the rows last-to-first.  The preceding V pass (the CGS dots)
// ended on the last rows, which the 256 MB Infinity Cache still holds, so a
// reversed sweep starts on cache hits (and the next forward pass on this one's
// last rows).
//
// Chained Lanczos steps (free-running engine, kFinCgsChained):
//   chained: V(:,J-1) holds the RAW residual r (v_j = r / rnorm not formed; the
//            SpMV ran on r): the pass normalises it in place (the same product
//            k_place forms) and takes w = vscale * (A r);
//   raw1/2:  also store rout there (the next step's raw column, and the x
//            buffer of a row-distributed SpMV); with the gate closed (no DGKS
//            sweep this step) the pass only copies rin to them.
template <class R, int J, bool SPEC, int POL = kPolNt>
__global__ __launch_bounds__(kBlock) void k_update_fused(
    int64_t n, R* __restrict__ V, int64_t ld, const double* __restrict__ c,
    const R* rin, R* rout, double* __restrict__ part, int pstride,
    const LzState* __restrict__ st, int gate, int chained, R* __restrict__ raw1,
    R* __restrict__ raw2) {
    if (st->abort) return;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    if (gate >= 0 && st->dgks != gate) {
        if (raw1)
            for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
                const R r = rin[i];
                raw1[i] = r;
                if (raw2) raw2[i] = r;
            }
        return;
    }
    const double vs = chained ? st->vscale : 1.0;  // exact no-op when not chained
    double acc[J];
#pragma unroll
    for (int k = 0; k < J; ++k) acc[k] = 0.0;
    double rr = 0.0;
    for (int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x; it < n; it += stride) {
        const int64_t i = POL == kPolNtRev ? n - 1 - it : it;
        double vrow[J];
#pragma unroll
        for (int k = 0; k < J; ++k) vrow[k] = vld<POL>(V + i + (int64_t)k * ld);
        const double win = (double)rin[i];
        if (chained) {  // v_j = r * (1/rnorm), stored as k_place would
            const R v = (R)(vrow[J - 1] * vs);
            V[i + (int64_t)(J - 1) * ld] = v;
            vrow[J - 1] = (double)v;
        }
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < J; ++k) s += vrow[k] * c[k];
        const R r = (R)(win * vs - s);
        rout[i] = r;
        if (raw1) raw1[i] = r;
        if (raw2) raw2[i] = r;
        if constexpr (SPEC) {
            const double rd = (double)r;
            rr += rd * rd;
#pragma unroll
            for (int k = 0; k < J; ++k) acc[k] += vrow[k] * rd;
        }
    }
    if constexpr (SPEC) block_partials<J>(acc, J, rr, true, part, 0, J);
}

// generic (any j): no fused dots
template <class R>
__global__ __launch_bounds__(kBlock) void k_update_generic(int64_t n, int j,
                                                           const R* __restrict__ V, int64_t ld,
                                                           const double* __restrict__ c,
                                                           const R* rin, R* rout,
                                                           const LzState* __restrict__ st,
                                                           int gate) {
    if (gate_closed(st, gate)) return;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        double s = 0.0;
        for (int k = 0; k < j; ++k) s += (double)V[i + (int64_t)k * ld] * c[k];
        rout[i] = (R)((double)rin[i] - s);
    }
}

// --------------------------------------------------------------- finalize ---
// Fixed-order sum of one slot's nblk per-block partials -> sums[slot].
__global__ __launch_bounds__(256) void k_reduce_slots(const double* __restrict__ part, int nblk,
                                                      double* __restrict__ sums,
                                                      const LzState* __restrict__ st, int gate) {
    if (gate_closed(st, gate)) return;
    __shared__ double red[4];
    const double* p = part + (int64_t)blockIdx.x * nblk;
    double s = 0.0;
    for (int b = threadIdx.x; b < nblk; b += 256) s += p[b];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

template <bool HS>
__global__ __launch_bounds__(1024) void k_finalize(FinArgs a) { finalize_block_dyn<HS>(a); }

template <class R>
__global__ void k_zero_if(int64_t n, R* r, const LzState* st) {
    if (st->abort || !st->zero) return;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) r[i] = 0.0;
}

// -------------------------------------------------------------- V*Q update --
// NTS: non-temporal stores of the kev+1 new columns and r.  tools/vq_bench.hip
// (this pass's shape, 31 columns read + 12 written, n = 1e7): plain stores
// 0.683 ms = 5.04 TB/s -- what this kernel reaches -- non-temporal 0.610 ms
// = 5.64 TB/s; reads alone 0.351 ms = 7.06 TB/s.
template <class R, int MAXK, int POL = kPolNt, bool NTS = false>
__global__ __launch_bounds__(kBlock) void k_vq_update(int64_t n, R* V, int64_t ld,
                                                      int kplusp, int kev,
                                                      const double* __restrict__ Q, int ldq,
                                                      double sigmak, double betak,
                                                      R* __restrict__ r,
                                                      double* __restrict__ part, int pstride) {
    // Q(:, 0:kev] staged in LDS once per block: the per-row sums then read it
    // with broadcast LDS loads instead of waiting on ~330 scalar-cache loads
    // per row batch (the scalar-load waits held this kernel at 4.45 TB/s)
    __shared__ double sq[MAXK * (MAXK + 1)];
    for (int e = threadIdx.x; e < kplusp * (kev + 1); e += kBlock)
        sq[e] = Q[e % kplusp + (int64_t)(e / kplusp) * ldq];
    __syncthreads();
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const bool next = betak > 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        double v[MAXK];
#pragma unroll
        for (int k = 0; k < MAXK; ++k)
            v[k] = (k < kplusp) ? (double)vld<POL>(V + i + (int64_t)k * ld) : 0.0;
        double vnext = 0.0;
        if (next) {
            const double* q = sq + kev * kplusp;
#pragma unroll
            for (int k = 0; k < MAXK; ++k)
                if (k < kplusp) vnext += v[k] * q[k];
        }
        auto st_ = [](R* p, R x) {
            if constexpr (NTS) __builtin_nontemporal_store(x, p);
            else *p = x;
        };
        for (int l = 0; l < kev; ++l) {
            const double* q = sq + l * kplusp;
            double o = 0.0;
#pragma unroll
            for (int k = 0; k < MAXK; ++k)
                if (k < kplusp) o += v[k] * q[k];
            st_(V + i + (int64_t)l * ld, (R)o);
        }
        double ri = sigmak * (double)r[i];
        if (next) {
            const R vn = (R)vnext;
            st_(V + i + (int64_t)kev * ld, vn);
            ri += betak * (double)vn;
        }
        const R rs = (R)ri;
        st_(r + i, rs);
        rr += (double)rs * (double)rs;
    }
    double acc[1] = {0.0};
    block_partials<1>(acc, 0, rr, true, part, 0, 0);
}

template <class R>
__global__ __launch_bounds__(kBlock) void k_vq_update_generic(
    int64_t n, R* V, int64_t ld, int kplusp, int kev, const double* __restrict__ Q,
    int ldq, double sigmak, double betak, R* __restrict__ r, double* __restrict__ tmp,
    double* __restrict__ part, int pstride) {
    // kplusp > 64: each thread keeps its row's kev+1 outputs in its own column
    // of the preallocated scratch (tmp[l * S + tid], S = grid threads, coalesced)
    // while V's row is read in column order; same summation order as k_vq_update
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool next = betak > 0.0;
    for (int64_t i = tid; i < n; i += stride) {
        for (int l = 0; l <= kev; ++l) tmp[l * stride + tid] = 0.0;
        for (int k = 0; k < kplusp; ++k) {
            const double vk = (double)V[i + (int64_t)k * ld];
            for (int l = 0; l <= kev; ++l) tmp[l * stride + tid] += vk * Q[k + (int64_t)l * ldq];
        }
        for (int l = 0; l < kev; ++l) V[i + (int64_t)l * ld] = (R)tmp[l * stride + tid];
        double ri = sigmak * (double)r[i];
        if (next) {
            const R vn = (R)tmp[kev * stride + tid];
            V[i + (int64_t)kev * ld] = vn;
            ri += betak * (double)vn;
        }
        const R rs = (R)ri;
        r[i] = rs;
        rr += (double)rs * (double)rs;
    }
    double acc[1] = {0.0};
    block_partials<1>(acc, 0, rr, true, part, 0, 0);
}

// Z = V(:,0:k) * M(k x nz) for k > 128, alias-safe through the per-thread
// scratch columns (tmp[l * S + tid], S = grid threads)
template <class R>
__global__ __launch_bounds__(kBlock) void k_vq_gemm_generic(int64_t n, const R* V, int64_t ld,
                                                            int k, int nz,
                                                            const double* __restrict__ M, R* Z,
                                                            int64_t ldz, double* __restrict__ tmp) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (int64_t i = tid; i < n; i += stride) {
        for (int l = 0; l < nz; ++l) tmp[l * stride + tid] = 0.0;
        for (int t = 0; t < k; ++t) {
            const double vt = (double)V[i + (int64_t)t * ld];
            for (int l = 0; l < nz; ++l) tmp[l * stride + tid] += vt * M[t + (int64_t)l * k];
        }
        for (int l = 0; l < nz; ++l) Z[i + (int64_t)l * ldz] = (R)tmp[l * stride + tid];
    }
}

// Z = V(:,0:k) * M(k x nz) ; row-local, so Z may alias V (rows held in registers)
template <class R, int MAXK>
__global__ __launch_bounds__(kBlock) void k_vq_gemm(int64_t n, const R* V, int64_t ld,
                                                    int k, int nz, const double* __restrict__ M,
                                                    R* Z, int64_t ldz) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        double v[MAXK];
#pragma unroll
        for (int t = 0; t < MAXK; ++t) v[t] = (t < k) ? V[i + (int64_t)t * ld] : 0.0;
        for (int l = 0; l < nz; ++l) {
            double o = 0.0;
#pragma unroll
            for (int t = 0; t < MAXK; ++t)
                if (t < k) o += v[t] * M[t + (int64_t)l * k];
            Z[i + (int64_t)l * ldz] = (R)o;
        }
    }
}

// ------------------------------------------------------------------ larnv ---
// 48-bit multiplicative congruential generator of LAPACK dlaruv:
// x_{m} = seed * a^m mod 2^48, a = 33952834046453; dlarnv(idist=2) returns
// 2*x/2^48 - 1 (exact in double: 48 bits < 53).
constexpr uint64_t kLcgA = 33952834046453ull;
constexpr uint64_t kMask48 = (1ull << 48) - 1;

__device__ __host__ __forceinline__ uint64_t mulmod48(uint64_t a, uint64_t b) {
    return (a * b) & kMask48;
}

// seed * a^steps mod 2^48 (host)
uint64_t lcg_pow(uint64_t seed, uint64_t steps) {
    uint64_t base = kLcgA, p = 1;
    while (steps) {
        if (steps & 1) p = mulmod48(p, base);
        base = mulmod48(base, base);
        steps >>= 1;
    }
    return mulmod48(seed, p);
}

__global__ void k_larnv(int64_t n, uint64_t seed, int64_t offset, double* __restrict__ x) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        // a^(i+1) by square-and-multiply
        uint64_t e = (uint64_t)(i + offset) + 1, base = kLcgA, p = 1;
        while (e) {
            if (e & 1) p = mulmod48(p, base);
            base = mulmod48(base, base);
            e >>= 1;
        }
        const uint64_t xm = mulmod48(seed, p);
        x[i] = 2.0 * ((double)xm * 0x1p-48) - 1.0;
    }
}

// slarnv(idist=2) in single precision (LAPACK slaruv): the same 48-bit stream,
// converted with REAL arithmetic X = R*(IT1 + R*(IT2 + R*(IT3 + R*IT4))),
// R = 1/4096 (unfused, as the Fortran evaluates it), then 2X - 1.  With 24-bit
// floats X rounds to 1.0 about once in 2^25 draws; slaruv then bumps every seed
// digit by 2 and redraws, which shifts the rest of its 64-draw batch and every
// later batch.  The closed form below flags the first such index (atomicMin) and
// the launcher regenerates the vector sequentially on the host (slarnv_host).
__device__ __host__ inline float slaruv_real(uint64_t xm) {
#pragma clang fp contract(off)
    const float r = 1.0f / 4096.0f;
    const float i1 = (float)((xm >> 36) & 4095), i2 = (float)((xm >> 24) & 4095);
    const float i3 = (float)((xm >> 12) & 4095), i4 = (float)(xm & 4095);
    return r * (i1 + r * (i2 + r * (i3 + r * i4)));
}

__global__ void k_larnv_f(int64_t n, uint64_t seed, int64_t offset, float* __restrict__ x,
                          unsigned long long* __restrict__ flag) {
#pragma clang fp contract(off)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t e = (uint64_t)(i + offset) + 1, base = kLcgA, p = 1;
        while (e) {
            if (e & 1) p = mulmod48(p, base);
            base = mulmod48(base, base);
            e >>= 1;
        }
        const float u = slaruv_real(mulmod48(seed, p));
        if (u == 1.0f) atomicMin(flag, (unsigned long long)i);
        x[i] = 2.0f * u - 1.0f;
    }
}

// ------------------------------------------------------------ elementwise ---
template <class R>
__global__ void k_copy(int64_t n, const R* __restrict__ s, R* __restrict__ d) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
}
template <class R>
__global__ void k_scal(int64_t n, double a, R* x) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = (R)((double)x[i] * a);
}
template <class R>
__global__ void k_fill(int64_t n, double a, R* x) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = (R)a;
}
template <class R>
__global__ void k_axpby(int64_t n, double alpha, R* y, double beta, const R* x) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        y[i] = (R)(alpha * (double)y[i] + beta * (double)x[i]);
}

// Z(:,l) += x * w[l]  (dseupd purification, SRC/dseupd.f:840-857)
template <class R>
__global__ void k_ger_cols(int64_t n, int k, const R* __restrict__ x,
                           const double* __restrict__ w, R* Z, int64_t ldz) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double xi = x[i];
        for (int l = 0; l < k; ++l)
            Z[i + (int64_t)l * ldz] = (R)((double)Z[i + (int64_t)l * ldz] + xi * w[l]);
    }
}

inline int grid_for(int64_t n, int per_block = kBlock, int cap = 8192) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

}  // namespace

// ================================================================ launchers ==

// V-load policy (VPol): plain loads when the basis fits the Infinity Cache.
// The element size is taken as 8 B for both families: a float basis of the
// same n streams half the bytes but its passes are shorter in the same ratio.
bool choose_v_plain(int64_t n, int ncv, int elem) {
    static const int forced = [] {
        const char* e = getenv("AHIP_V_POLICY");
        if (!e) return -1;
        if (!strcmp(e, "plain")) return 1;
        if (!strcmp(e, "nt")) return 0;
        return -1;
    }();
    if (forced >= 0) return forced == 1;
    return (double)n * ncv * elem <= 400e6;
}

int choose_nblk(int64_t n) {
    // AHIP_NBLK: tuning knob for the partial-sum grid (default kMaxRedBlocks)
    static const int64_t cap = [] {
        const char* e = getenv("AHIP_NBLK");
        const long v = e ? atol(e) : 0;
        return (int64_t)(v >= 64 && v <= 8192 ? v : kMaxRedBlocks);
    }();
    int64_t b = (n + kBlock - 1) / kBlock;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (int)b;
}

static hipError_t ws_alloc(Workspace& ws, int64_t n, int ncv, hipStream_t s);

// on failure everything allocated so far is released (ws left empty)
hipError_t ws_create(Workspace& ws, int64_t n, int ncv, hipStream_t s) {
    const hipError_t e = ws_alloc(ws, n, ncv, s);
    if (e != hipSuccess) ws_destroy(ws);
    return e;
}

static hipError_t ws_alloc(Workspace& ws, int64_t n, int ncv, hipStream_t s) {
    ws.stream = s;
    ws.v_plain = choose_v_plain(n, ncv, 8);
    ws.nblk = choose_nblk(n);
    ws.stride = ncv + 2;
    hipError_t e;
    // two partial regions: the second holds a chained step's deferred DGKS sums
    if ((e = hipMalloc(&ws.part, sizeof(double) * 2 * (size_t)ws.nblk * ws.stride))) return e;
    if ((e = hipMalloc(&ws.sums, sizeof(double) * 2 * (size_t)ws.stride))) return e;
    if ((e = hipMalloc(&ws.coef, sizeof(double) * 4 * (size_t)ws.stride))) return e;
    if ((e = hipMalloc(&ws.rec, sizeof(double) * 2 * (size_t)(ncv + 1)))) return e;
    if ((e = hipMalloc(&ws.q, sizeof(double) * (size_t)ncv * ncv))) return e;
    if ((e = hipMalloc(&ws.hcol, sizeof(double) * (size_t)ncv * ncv))) return e;
    if (ncv > 64 &&  // per-thread output columns of the generic V*Q / gemm kernels
        (e = hipMalloc(&ws.scratch, sizeof(double) * (size_t)ws.nblk * kBlock * (ncv + 1))))
        return e;
    ws.defq = new FinQueue;
    if ((e = hipMalloc(&ws.st, sizeof(LzState)))) return e;
    if ((e = hipHostMalloc(&ws.st_host, sizeof(LzState)))) return e;
    if ((e = hipHostMalloc(&ws.host_scratch, sizeof(double) * (4 * (size_t)ws.stride + 2 * (ncv + 1)))))
        return e;
    if (ncv <= 64 && (e = hipHostMalloc(&ws.host_hcol, sizeof(double) * (size_t)ncv * ncv))) return e;
    if (ncv <= 64 && (e = hipHostMalloc(&ws.host_q, sizeof(double) * (size_t)ncv * ncv))) return e;
    memset(ws.st_host, 0, sizeof(LzState));
    {   // test hook: exercise the (rare) second DGKS refinement on every step
        const char* e = getenv("AHIP_FORCE_DGKS2");
        ws.st_host->force_dgks2 = (e && e[0] == '1') ? 1 : 0;
    }
    (void)hipMemcpyAsync(ws.st, ws.st_host, sizeof(LzState), hipMemcpyHostToDevice, s);
    (void)hipMemsetAsync(ws.coef, 0, sizeof(double) * 4 * (size_t)ws.stride, s);
    return hipSuccess;
}

void ws_destroy(Workspace& ws) {
    if (ws.part) (void)hipFree(ws.part);
    if (ws.sums) (void)hipFree(ws.sums);
    if (ws.coef) (void)hipFree(ws.coef);
    if (ws.rec) (void)hipFree(ws.rec);
    if (ws.q) (void)hipFree(ws.q);
    if (ws.hcol) (void)hipFree(ws.hcol);
    if (ws.scratch) (void)hipFree(ws.scratch);
    if (ws.st) (void)hipFree(ws.st);
    if (ws.st_host) (void)hipHostFree(ws.st_host);
    if (ws.host_scratch) (void)hipHostFree(ws.host_scratch);
    if (ws.host_hcol) (void)hipHostFree(ws.host_hcol);
    if (ws.host_q) (void)hipHostFree(ws.host_q);
    delete ws.defq;
    ws = Workspace{};
}

// Sweep direction of the V passes.  Each pass starts where the previous one
// ended, on the rows the 256 MB Infinity Cache still holds: within step j the
// CGS dots, the CGS update and the first DGKS update alternate, and so do
// consecutive steps (the SpMV between them streams its matrix with
// non-temporal loads).  AHIP_SWEEP=0: all forward; 1: only the updates
// alternate (dots forward); 2 (default): dots alternate per step too.
static bool dir_rev(int j, int which, bool is_dots) {
    static const int mode = [] {
        const char* e = getenv("AHIP_SWEEP");
        return e ? atoi(e) : 2;
    }();
    if (mode == 0) return false;
    const bool d = mode == 2 && (j & 1);  // the dots pass of step j
    if (is_dots) return d;
    return which % 2 == 0 ? !d : d;      // CGS / second DGKS update: opposite; first DGKS: same
}

template <class R>
void place(const Workspace& ws, int64_t n, const R* r, R* vcol, R* copy1, R* sc, int j) {
    ProfScope ps(kProfPlace, ws.stream,
                 (double)sizeof(R) * n * (2 + (copy1 != nullptr) + 2 * (sc != nullptr)));
    AHIP_LAUNCH(k_place<R>, dim3(grid_for(n)), dim3(kBlock), 0, ws.stream, n, r, vcol, copy1,
                       sc, ws.st, j);
}

template <class R, int WM, int POL = kPolNt>
static void launch_dots(const Workspace& ws, int64_t n, int j0, int jc, const R* V, int64_t ld,
                        const R* u, const R* w, int wslot, int gate) {
    const dim3 g(ws.nblk), b(kBlock);
    switch (jc) {
        case 0:
            AHIP_LAUNCH((k_dots<R, 0, WM>), g, b, 0, ws.stream, n, j0, V, ld, u, w, ws.part,
                               ws.stride, wslot, ws.st, gate);
            break;
#define AHIP_DOTS_CASE(J)                                                                          \
    case J:                                                                                        \
        AHIP_LAUNCH((k_dots<R, J, WM, POL>), g, b, 0, ws.stream, n, j0, V, ld, u, w,        \
                           ws.part, ws.stride, wslot, ws.st, gate);                                \
        break;
        AHIP_CASES_1_32(AHIP_DOTS_CASE)
#undef AHIP_DOTS_CASE
        default: break;
    }
}

template <class R>
void dots(const Workspace& ws, int64_t n, int j, const R* V, int64_t ld, const R* u, const R* w,
          int gate) {
    ProfScope ps(gate == 2 ? kProfOther : kProfDots, ws.stream,
                 gate == 2 ? 0.0 : (double)sizeof(R) * n * (j + 1 + (w != u)));
    if (j == 0) {
        if (w == u) launch_dots<R, 1>(ws, n, 0, 0, V, ld, u, w, 0, gate);
        else launch_dots<R, 2>(ws, n, 0, 0, V, ld, u, w, 0, gate);
        return;
    }
    // sweep direction alternates per Lanczos step (dir_rev, below)
    const bool rev = dir_rev(j, 0, true);
    for (int j0 = 0; j0 < j; j0 += 32) {
        const int jc = (j - j0 < 32) ? j - j0 : 32;
        if (j0 > 0) launch_dots<R, 0>(ws, n, j0, jc, V, ld, u, w, j, gate);
        else if (w == u && ws.v_plain) launch_dots<R, 1, kPolPlain>(ws, n, j0, jc, V, ld, u, w, j, gate);
        else if (w == u && rev) launch_dots<R, 1, kPolNtRev>(ws, n, j0, jc, V, ld, u, w, j, gate);
        else if (w == u) launch_dots<R, 1>(ws, n, j0, jc, V, ld, u, w, j, gate);
        else launch_dots<R, 2>(ws, n, j0, jc, V, ld, u, w, j, gate);
    }
}

template <class R>
void update(const Workspace& ws, int64_t n, int j, const R* V, int64_t ld, int which, const R* rin,
            R* rout, bool spec, int gate, const UpdateChain<R>& x) {
    const double* c = ws.coef + (size_t)which * ws.stride;
    ProfScope ps(gate == 2 ? kProfOther : kProfUpdate, ws.stream,
                 gate == 2 ? 0.0
                           : (double)sizeof(R) * n *
                                 (j + 2 + (x.chained ? 1 : 0) + (x.raw1 ? 1 : 0) + (x.raw2 ? 1 : 0)));
    const dim3 g(ws.nblk), b(kBlock);
    const bool rev = dir_rev(j, which, false);
    double* part = x.part ? x.part : ws.part;
    R* Vw = const_cast<R*>(V);  // written only by a chained pass (its column j)
    // fused up to j = 64 (ncv <= 64: dnaupd's C3 runs ncv = 40); the V row of a
    // fused pass lives in registers, so a wider J trades occupancy for
    // in-flight loads per wave (64 column loads per row at J = 64)
    if (j >= 1 && j <= 64) {
        auto go = [&](auto kern) {
            AHIP_LAUNCH(kern, g, b, 0, ws.stream, n, Vw, ld, c, rin, rout, part, ws.stride,
                               ws.st, gate, x.chained ? 1 : 0, x.raw1, x.raw2);
        };
        switch (j) {
#define AHIP_UPD_CASE(J)                                                                           \
    case J:                                                                                        \
        if (spec && ws.v_plain) go(k_update_fused<R, J, true, kPolPlain>);                         \
        else if (spec && rev) go(k_update_fused<R, J, true, kPolNtRev>);                           \
        else if (spec) go(k_update_fused<R, J, true>);                                             \
        else go(k_update_fused<R, J, false>);                                                      \
        break;
            AHIP_CASES_1_32(AHIP_UPD_CASE)
            AHIP_CASES_33_64(AHIP_UPD_CASE)
#undef AHIP_UPD_CASE
            default: break;
        }
    } else {  // (chained steps run only with ncv <= 64: the solver's choice)
        AHIP_LAUNCH(k_update_generic<R>, g, b, 0, ws.stream, n, j, V, ld, c, rin, rout, ws.st,
                           gate);
        if (spec) dots<R>(ws, n, j, V, ld, rout, rout, gate);
    }
}

namespace {
void launch_fin(hipStream_t s, const FinArgs& a, size_t lds) {
    // ncv up to kMaxNcv: the state and records plus 8002 sums pass 64 KB
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)k_finalize<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        return true;
    }();
    (void)attr;
    AHIP_LAUNCH(a.hs ? k_finalize<true> : k_finalize<false>, dim3(1), dim3(1024), lds, s, a);
}
}  // namespace

bool take_deferred_finalize(FinQueue* q, FinArgs* a, size_t* lds, size_t max_lds, bool allow_hs) {
    if (!q || !q->set) return false;
    if (q->lds > max_lds || (q->a.hs && !allow_hs)) return false;
    *a = q->a;
    *lds = q->lds;
    q->set = false;
    return true;
}

void flush_deferred_finalize(FinQueue* q, hipStream_t s) {
    if (!q || !q->set) return;
    q->set = false;
    ProfScope ps(kProfFinalize, s, 0.0);
    launch_fin(s, q->a, q->lds);
}

void finalize(const Workspace& ws, int m, FinPhase ph, int j, int rstart, int gate, bool from_sums,
              int m2, int rstart_prev, bool defer) {
    flush_deferred_finalize(ws.defq, ws.stream);  // (stream order: an earlier one runs first)
    // AHIP_FIN_DEFER=0: never deferred into the SpMV's combine
    static const bool defer_on = [] {
        const char* e = getenv("AHIP_FIN_DEFER");
        return !(e && e[0] == '0');
    }();
    // AHIP_FUSED_FIN=0: two launches (per-slot reduction, then the phase logic)
    static const bool fused = [] {
        const char* e = getenv("AHIP_FUSED_FIN");
        return !(e && e[0] == '0');
    }();
    const double* part2 = ws.part + (size_t)ws.nblk * ws.stride;  // region 2 (chained steps)
    const size_t lds = fin_lds_bytes(m + m2);  // state, records, sums (m + m2 <= kMaxNcv + 67)
    const bool hs = ph == kFinPostCgsFold && ws.hld && m - 1 <= kFoldHMax;
    auto args = [&](int fs) {
        return FinArgs{ws.part, ws.nblk, fs, m, (int)ph, j, rstart, gate, ws.sums, ws.coef,
                       ws.stride, ws.rec, ws.st, ws.hcol, ws.hld, part2, m2, rstart_prev,
                       hs ? 1 : 0, 1};
    };
    // (from_sums: the distributed path's phase logic on allreduced sums)
    if (defer && defer_on && (from_sums || fused) && ws.defq) {
        *ws.defq = FinQueue{args(from_sums ? 1 : 0), lds, true};
        return;
    }
    ProfScope ps(kProfFinalize, ws.stream, from_sums ? 0.0 : 8.0 * ws.nblk * (m + m2));
    auto fin = [&](int fs) { launch_fin(ws.stream, args(fs), lds); };
    if (!from_sums && fused) {  // one launch: the finalize block sums the partials itself
        fin(0);
        return;
    }
    if (!from_sums) {
        // stage 2a: one workgroup per slot sums that slot's nblk partials (coalesced;
        // region 2 follows region 1 in memory only when m == stride -- so two launches)
        AHIP_LAUNCH(k_reduce_slots, dim3(m), dim3(256), 0, ws.stream, ws.part, ws.nblk, ws.sums,
                           ws.st, gate);
        if (m2)
            AHIP_LAUNCH(k_reduce_slots, dim3(m2), dim3(256), 0, ws.stream, part2, ws.nblk,
                               ws.sums + m, ws.st, gate);
    }
    // stage 2b: the phase logic on the m + m2 sums (one small workgroup)
    fin(1);
}

template <class R>
void zero_if(const Workspace& ws, int64_t n, R* r) {
    ProfScope ps(kProfOther, ws.stream, 0.0);
    AHIP_LAUNCH(k_zero_if<R>, dim3(grid_for(n)), dim3(kBlock), 0, ws.stream, n, r, ws.st);
}

template <class R>
void vq_update(const Workspace& ws, int64_t n, R* V, int64_t ld, int kplusp, int kev, double sigmak,
               double betak, R* r) {
    const int g = ws.nblk;
    ProfScope ps(kProfVq, ws.stream,
                 (double)sizeof(R) * n * (kplusp + kev + (betak > 0.0) + 2));
    auto go = [&](auto kern) {
        AHIP_LAUNCH(kern, dim3(g), dim3(kBlock), 0, ws.stream, n, V, ld, kplusp, kev, ws.q,
                           kplusp, sigmak, betak, r, ws.part, ws.stride);
    };
    // AHIP_VQ_NTS=0: plain stores of the new columns (the V-load policy's
    // plain-load case keeps plain stores: there the next pass re-reads V from
    // the Infinity Cache)
    static const bool nts = [] {
        const char* e = getenv("AHIP_VQ_NTS");
        return !(e && e[0] == '0');
    }();
    if (kplusp <= 16) ws.v_plain ? go(k_vq_update<R, 16, kPolPlain>)
                      : nts ? go(k_vq_update<R, 16, kPolNt, true>) : go(k_vq_update<R, 16>);
    else if (kplusp <= 32) ws.v_plain ? go(k_vq_update<R, 32, kPolPlain>)
                           : nts ? go(k_vq_update<R, 32, kPolNt, true>) : go(k_vq_update<R, 32>);
    // 40 / 48: the ncv = 40 of configs 3 and 5 in 127 VGPRs (four waves a
    // SIMD) where MAXK = 64 takes 211 (two)
    else if (kplusp <= 40) ws.v_plain ? go(k_vq_update<R, 40, kPolPlain>)
                           : nts ? go(k_vq_update<R, 40, kPolNt, true>) : go(k_vq_update<R, 40>);
    else if (kplusp <= 48) ws.v_plain ? go(k_vq_update<R, 48, kPolPlain>)
                           : nts ? go(k_vq_update<R, 48, kPolNt, true>) : go(k_vq_update<R, 48>);
    else if (kplusp <= 64) ws.v_plain ? go(k_vq_update<R, 64, kPolPlain>)
                           : nts ? go(k_vq_update<R, 64, kPolNt, true>) : go(k_vq_update<R, 64>);
    else  // ws.scratch: nblk * kBlock * (ncv + 1) doubles, allocated by ws_create for ncv > 64
        AHIP_LAUNCH(k_vq_update_generic<R>, dim3(g), dim3(kBlock), 0, ws.stream, n, V, ld,
                           kplusp, kev, ws.q, kplusp, sigmak, betak, r, ws.scratch, ws.part,
                           ws.stride);
}

template <class R>
void vq_gemm(const Workspace& ws, int64_t n, const R* V, int64_t ld, int k, int nz, R* Z,
             int64_t ldz) {
    const int g = grid_for(n);
    if (k <= 16)
        AHIP_LAUNCH((k_vq_gemm<R, 16>), dim3(g), dim3(kBlock), 0, ws.stream, n, V, ld, k, nz,
                           ws.q, Z, ldz);
    else if (k <= 32)
        AHIP_LAUNCH((k_vq_gemm<R, 32>), dim3(g), dim3(kBlock), 0, ws.stream, n, V, ld, k, nz,
                           ws.q, Z, ldz);
    else if (k <= 64)
        AHIP_LAUNCH((k_vq_gemm<R, 64>), dim3(g), dim3(kBlock), 0, ws.stream, n, V, ld, k, nz,
                           ws.q, Z, ldz);
    else if (k <= 128)
        AHIP_LAUNCH((k_vq_gemm<R, 128>), dim3(g), dim3(kBlock), 0, ws.stream, n, V, ld, k, nz,
                           ws.q, Z, ldz);
    else  // grid = nblk: the scratch holds nblk * kBlock rows of ncv + 1 outputs
        AHIP_LAUNCH(k_vq_gemm_generic<R>, dim3(ws.nblk), dim3(kBlock), 0, ws.stream, n, V, ld,
                           k, nz, ws.q, Z, ldz, ws.scratch);
}

uint64_t larnv_uniform(const Workspace& ws, int64_t n, uint64_t seed48, double* x,
                       int64_t offset, int) {
    AHIP_LAUNCH(k_larnv, dim3(grid_for(n)), dim3(kBlock), 0, ws.stream, n, seed48, offset, x);
    return lcg_pow(seed48, (uint64_t)n);
}

// Sequential slarnv(idist=2, iseed, n, x) with slaruv's batches (64 draws;
// clarnv draws 128 = 64 complex per slaruv call) and its redraw rule (LAPACK
// slarnv.f / clarnv.f / slaruv.f); returns the updated 48-bit seed.
uint64_t slarnv_host(int64_t n, uint64_t seed, float* x, int batch) {
#pragma clang fp contract(off)
    // every seed digit + 2 (slaruv.f: I1..I4 = I1..I4 + 2 when X(I) = 1)
    const uint64_t bump = 2 * ((1ull << 36) + (1ull << 24) + (1ull << 12) + 1);
    for (int64_t iv = 0; iv < n; iv += batch) {
        const int il = (int)((n - iv) < batch ? (n - iv) : batch);
        uint64_t s = seed, p = 1, last = seed;
        for (int i = 0; i < il; ++i) {
            p = mulmod48(p, kLcgA);
            for (;;) {
                last = mulmod48(s, p);
                const float u = slaruv_real(last);
                if (u != 1.0f) {
                    x[iv + i] = 2.0f * u - 1.0f;
                    break;
                }
                s = (s + bump) & kMask48;
            }
        }
        seed = last;
    }
    return seed;
}

uint64_t larnv_uniform(const Workspace& ws, int64_t n, uint64_t seed48, float* x,
                       int64_t offset, int batch) {
    unsigned long long* flag = reinterpret_cast<unsigned long long*>(ws.host_scratch);
    const bool own = (flag == nullptr);
    if (own && hipHostMalloc(&flag, sizeof(unsigned long long)) != hipSuccess) flag = nullptr;
    bool redraw = true;  // no flag memory: take the sequential path
    if (flag) {
        *flag = ~0ull;  // pinned host memory, visible to the kernel
        AHIP_LAUNCH(k_larnv_f, dim3(grid_for(n)), dim3(kBlock), 0, ws.stream, n, seed48,
                           offset, x, flag);
        (void)hipStreamSynchronize(ws.stream);
        redraw = (*flag != ~0ull);
        if (own) (void)hipHostFree(flag);
    }
    if (!redraw) return lcg_pow(seed48, (uint64_t)n);
    // a draw rounded to 1.0: slaruv's redraw shifts the stream from there on
    std::vector<float> h((size_t)n);
    const uint64_t s = slarnv_host(n, seed48, h.data(), batch);
    (void)hipMemcpyAsync(x, h.data(), sizeof(float) * n, hipMemcpyHostToDevice, ws.stream);
    (void)hipStreamSynchronize(ws.stream);
    return s;
}

template <class R>
void copy(hipStream_t s, int64_t n, const R* src, R* dst) {
    AHIP_LAUNCH(k_copy<R>, dim3(grid_for(n)), dim3(kBlock), 0, s, n, src, dst);
}
template <class R>
void scal(hipStream_t s, int64_t n, double a, R* x) {
    AHIP_LAUNCH(k_scal<R>, dim3(grid_for(n)), dim3(kBlock), 0, s, n, a, x);
}
template <class R>
void fill(hipStream_t s, int64_t n, double a, R* x) {
    AHIP_LAUNCH(k_fill<R>, dim3(grid_for(n)), dim3(kBlock), 0, s, n, a, x);
}
template <class R>
void axpby(hipStream_t s, int64_t n, double alpha, R* y, double beta, const R* x) {
    AHIP_LAUNCH(k_axpby<R>, dim3(grid_for(n)), dim3(kBlock), 0, s, n, alpha, y, beta, x);
}

template <class R>
void ger_cols(hipStream_t s, int64_t n, int k, const R* x, const double* w, R* Z, int64_t ldz) {
    AHIP_LAUNCH(k_ger_cols<R>, dim3(grid_for(n)), dim3(kBlock), 0, s, n, k, x, w, Z, ldz);
}

#define AHIP_INST(R)                                                                               \
    template void place<R>(const Workspace&, int64_t, const R*, R*, R*, R*, int);                  \
    template void dots<R>(const Workspace&, int64_t, int, const R*, int64_t, const R*, const R*,   \
                          int);                                                                    \
    template void update<R>(const Workspace&, int64_t, int, const R*, int64_t, int, const R*, R*,  \
                            bool, int, const UpdateChain<R>&);                                     \
    template void zero_if<R>(const Workspace&, int64_t, R*);                                       \
    template void vq_update<R>(const Workspace&, int64_t, R*, int64_t, int, int, double, double,  \
                               R*);                                                                \
    template void vq_gemm<R>(const Workspace&, int64_t, const R*, int64_t, int, int, R*, int64_t); \
    template void copy<R>(hipStream_t, int64_t, const R*, R*);                                     \
    template void scal<R>(hipStream_t, int64_t, double, R*);                                       \
    template void fill<R>(hipStream_t, int64_t, double, R*);                                       \
    template void axpby<R>(hipStream_t, int64_t, double, R*, double, const R*);                    \
    template void ger_cols<R>(hipStream_t, int64_t, int, const R*, const double*, R*, int64_t);
AHIP_INST(double)
AHIP_INST(float)
#undef AHIP_INST

}  // namespace ahip::dev

// ---- test hook: a caller's in-flight GPU work (arpack_hip.h) -------------------
namespace {
__global__ void k_delayed_fill(double* __restrict__ dst, const double* __restrict__ src, double value,
                               int64_t count, long long ticks) {
    // every wave waits out the delay on the device wall clock (bounded: the
    // loop ends when the clock passes the mark), then the grid writes
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += stride)
        dst[k] = src ? src[k] : value;
}
}  // namespace

extern "C" int arpack_hip_test_delayed_fill(double* dst, const double* src, double value, int64_t count,
                                            int delay_us) {
    static hipStream_t s = nullptr;  // never destroyed: its last kernel may still run
    if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        return -1;
    const long long ticks = (long long)delay_us * khz / 1000;
    const int64_t g = std::min<int64_t>(std::max<int64_t>((count + 255) / 256, 1), 1024);
    hipLaunchKernelGGL(k_delayed_fill, dim3((unsigned)g), dim3(256), 0, s, dst, src, value, count, ticks);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
