// Device-resident complex Arnoldi step (znaitr, SRC/znaitr.f:355-830) for
// bmat = 'I': the complex twins of kernels.hip's place / dots / fused update /
// finalize, with every CGS and DGKS decision taken on the device
// (dev::LzState), so the free-running znaupd (OP = a device complex CSR) enqueues
// a whole restart cycle without a host round trip, and the RCI form synchronises
// once per step (at its return to the caller) instead of once per reduction.
//
//   zs_place   v_j = r / rnorm (zdscal, or zlascl's factors below safmin)
//   zs_dots    partials of [V(:,1:J)^H u ; u^H u]             (znaitr.f:567-577)
//   zs_update  r = rin - V h, fused with the partials of [V^H r ; r^H r]
//              (the DGKS coefficients of the next sweep)       (znaitr.f:585-590,
//                                                               675-690)
//   zs_finalize  fixed-order sums + the phase logic: h(1:j,j) recorded in hcol,
//              wnorm / rnorm, the 0.717 tests, <= 2 refinements (znaitr.f:651-780)
//   zfold_dots / zfold_update  the folded step (free-running mode 1, ncv <= 40):
//              step j-1's DGKS sweep applied inside step j's two passes, as the
//              real engine's fold.hip -- A r' = A r - V (H s) - s_J r' by the
//              Arnoldi relation A V_J = V_J H_J + r' e_J^T (H_J with the sweep's
//              correction in its last column), so OP runs on the raw residual r
//              and the sweep is no pass of its own: two V passes a step, not three
//
// Partial layout: complex slot c -> real slots 2c (Re), 2c+1 (Im) of
// part[slot * nblk + block]; the norm slot follows the j coefficients.
// Reductions are two-stage and fixed-order: bitwise reproducible run to run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdlib>

#include "zcommon.hpp"
#include "zengine.hpp"
#include "reduce.hpp"

namespace ahip::zdev {

namespace {
using namespace zc;
using dev::LzState;

__device__ __forceinline__ bool zgate_closed(const LzState* st, int gate) {
    if (st->abort) return true;
    return gate >= 0 && st->dgks != gate;
}

// Block-reduce NV per-thread values and store them as this block's partials in
// slots slot0 .. slot0+nv-1.
template <int NV>
__device__ __forceinline__ void zblock_partials(const double (&v)[NV], int nv, double* part,
                                                int slot0) {
    __shared__ double red[kB / 64][NV];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        if (k < nv) {
            const double s = wsum(v[k]);
            if (lane == 0) red[wave][k] = s;
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nv; k += kB) {
        const double s = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
        part[(size_t)(slot0 + k) * gridDim.x + blockIdx.x] = s;
    }
}

template <class R>
__global__ __launch_bounds__(kB) void k_zs_place(int64_t n, const typename C2<R>::T* __restrict__ r,
                                                 typename C2<R>::T* __restrict__ vcol,
                                                 typename C2<R>::T* __restrict__ copy1,
                                                 typename C2<R>::T* __restrict__ copy2,
                                                 double safmin, LzState* __restrict__ st, int j) {
    if (st->abort) return;
    const double rn = st->rnorm;
    if (!(rn > 0.0)) {  // invariant subspace: restart (SRC/znaitr.f:373)
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->abort = 1;
            st->abort_j = j;
        }
        return;
    }
    // zdscal(1/rnorm) (znaitr.f:440-442), or zlascl('General', rnorm, 1) below
    // safmin: rnorm * safmin underflows, so scale up by 1/safmin first
    double m0 = 1.0 / rn, m1 = 1.0;
    if (rn < safmin) {
        m0 = 1.0 / safmin;
        m1 = 1.0 / (rn * m0);
    }
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        const double2 x = d2(r[i]);
        const double2 v = make_double2(x.x * m0 * m1, x.y * m0 * m1);
        const auto vs = st2<R>(v);
        vcol[i] = vs;
        if (copy1) copy1[i] = vs;
        if (copy2) copy2[i] = vs;
    }
}

// [V(:,c0:c0+J)^H u ; (WM) u^H u]; the J column loads of a row issue together
template <class R, int J, bool WM>
__global__ __launch_bounds__(kB) void k_zs_dots(int64_t n, int c0,
                                                const typename C2<R>::T* __restrict__ V, int64_t ld,
                                                const typename C2<R>::T* __restrict__ u,
                                                double* __restrict__ part, int wslot,
                                                const LzState* __restrict__ st, int gate) {
    if (zgate_closed(st, gate)) return;
    double2 acc[J];
#pragma unroll
    for (int k = 0; k < J; ++k) acc[k] = make_double2(0.0, 0.0);
    double aw = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kB;
    const typename C2<R>::T* Vb = V + (int64_t)c0 * ld;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        double2 vr[J];
#pragma unroll
        for (int k = 0; k < J; ++k) vr[k] = ntld(Vb + i + (int64_t)k * ld);
        const double2 ui = d2(u[i]);
        if constexpr (WM) aw += ui.x * ui.x + ui.y * ui.y;
#pragma unroll
        for (int k = 0; k < J; ++k) {
            const double2 p = cmulc(vr[k], ui);
            acc[k].x += p.x;
            acc[k].y += p.y;
        }
    }
    constexpr int NV = 2 * J + 2;
    double v[NV];
#pragma unroll
    for (int k = 0; k < J; ++k) {
        v[2 * k] = acc[k].x;
        v[2 * k + 1] = acc[k].y;
    }
    v[2 * J] = aw;
    v[2 * J + 1] = 0.0;
    zblock_partials<NV>(v, 2 * J, part, 2 * c0);
    if constexpr (WM) {  // u^H u (real) into the norm slot
        double w2[2] = {aw, 0.0};
        __syncthreads();
        zblock_partials<2>(w2, 2, part, 2 * wslot);
    }
}

// rout = rin - V(:,0:J) c ; SPEC: partials of [V^H rout ; rout^H rout]
template <class R, int J, bool SPEC>
__global__ __launch_bounds__(kB) void k_zs_update(int64_t n, const typename C2<R>::T* __restrict__ V,
                                                  int64_t ld, const double2* __restrict__ c,
                                                  const typename C2<R>::T* rin,
                                                  typename C2<R>::T* rout, double* __restrict__ part,
                                                  const LzState* __restrict__ st, int gate) {
    if (zgate_closed(st, gate)) return;
    double2 acc[SPEC ? J : 1];
#pragma unroll
    for (int k = 0; k < (SPEC ? J : 1); ++k) acc[k] = make_double2(0.0, 0.0);
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        double2 vr[J];
#pragma unroll
        for (int k = 0; k < J; ++k) vr[k] = ntld(V + i + (int64_t)k * ld);
        double2 r = d2(rin[i]);
#pragma unroll
        for (int k = 0; k < J; ++k) {  // the zgemv order: r -= V(:,k) c(k), k ascending
            const double2 p = cmul(vr[k], c[k]);
            r.x -= p.x;
            r.y -= p.y;
        }
        const auto rs = st2<R>(r);
        rout[i] = rs;
        if constexpr (SPEC) {
            const double2 rd = d2(rs);
            rr += rd.x * rd.x + rd.y * rd.y;
#pragma unroll
            for (int k = 0; k < J; ++k) {
                const double2 p = cmulc(vr[k], rd);
                acc[k].x += p.x;
                acc[k].y += p.y;
            }
        }
    }
    if constexpr (SPEC) {
        constexpr int NV = 2 * J + 2;
        double v[NV];
#pragma unroll
        for (int k = 0; k < J; ++k) {
            v[2 * k] = acc[k].x;
            v[2 * k + 1] = acc[k].y;
        }
        v[2 * J] = rr;
        v[2 * J + 1] = 0.0;
        zblock_partials<NV>(v, NV, part, 0);
    }
}

// generic width (j > 40): rout = rin - V c, no fused partials
template <class R>
__global__ __launch_bounds__(kB) void k_zs_update_generic(int64_t n, int j,
                                                          const typename C2<R>::T* __restrict__ V,
                                                          int64_t ld, const double2* __restrict__ c,
                                                          const typename C2<R>::T* rin,
                                                          typename C2<R>::T* rout,
                                                          const LzState* __restrict__ st, int gate) {
    if (zgate_closed(st, gate)) return;
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        double2 r = d2(rin[i]);
        for (int k = 0; k < j; ++k) {
            const double2 p = cmul(d2(V[i + (int64_t)k * ld]), c[k]);
            r.x -= p.x;
            r.y -= p.y;
        }
        rout[i] = st2<R>(r);
    }
}

// The folded passes spread each row over L lanes (L = 1, 2 or 4): lane q of
// the row's group holds columns [q JQ, (q+1) JQ) of V (JQ = ceil(J / L)) and
// their accumulators -- a quarter of the registers at L = 4, so four waves a
// SIMD instead of one at J = 39.  Sums over a row's columns are each lane's
// sequential partial, then (p0 + p1) + (p2 + p3) across the group (xor
// shuffles: every lane of the group ends with the same bits).
template <int L>
__device__ __forceinline__ double gsum(double v) {
    if constexpr (L >= 2) v += __shfl_xor(v, 1, 64);
    if constexpr (L >= 4) v += __shfl_xor(v, 2, 64);
    return v;
}

// r' = r - V(:,0:J) s (rounded to the storage type as the DGKS update's store)
// and w = A r' = y - (V(:,0:J) t + c r') with t = H_J s, c = s_J; explicit fma,
// so k_zfold_dots and k_zfold_update form both bit-identically.  Without a
// pending sweep r' = r, w = y.  vr: this lane's JQ columns from c0.
template <class R, int J, int L>
__device__ __forceinline__ void zfold_rw(bool fold, const double2* vr, int c0,
                                         const double2* __restrict__ s,
                                         const double2* __restrict__ t, double2 c, double2& rp,
                                         double2& w) {
    if (!fold) return;
    constexpr int JQ = (J + L - 1) / L;
    double px = 0.0, py = 0.0;
#pragma unroll
    for (int kk = 0; kk < JQ; ++kk) {
        if (c0 + kk < J) {
            const double2 p = cmul(vr[kk], s[c0 + kk]);
            px += p.x;
            py += p.y;
        }
    }
    rp.x -= gsum<L>(px);
    rp.y -= gsum<L>(py);
    rp = d2(st2<R>(rp));
    double ax = 0.0, ay = 0.0;
#pragma unroll
    for (int kk = 0; kk < JQ; ++kk) {
        if (c0 + kk < J) {
            const double2 tk = t[c0 + kk];
            ax = fma(vr[kk].x, tk.x, fma(-vr[kk].y, tk.y, ax));
            ay = fma(vr[kk].x, tk.y, fma(vr[kk].y, tk.x, ay));
        }
    }
    ax = gsum<L>(ax);
    ay = gsum<L>(ay);
    ax = fma(c.x, rp.x, fma(-c.y, rp.y, ax));
    ay = fma(c.x, rp.y, fma(c.y, rp.x, ay));
    w.x -= ax;
    w.y -= ay;
}

// Block partials of a lane-split pass: accumulator kk of group lane q is column
// q JQ + kk (< J); `extra` (NE values, held by group lane 0) follows in slots
// 2J ...  Each column's sum over the block: the wave's lanes of the same q
// (xor offsets L .. 32), then the four waves in zblock_partials' order.
template <int J, int L, int NE>
__device__ __forceinline__ void zsplit_partials(const double2 (&acc)[(J + L - 1) / L],
                                                const double (&extra)[NE], double* part) {
    constexpr int JQ = (J + L - 1) / L, NV = 2 * J + NE;
    __shared__ double red[kB / 64][NV];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane % L;
    const int c0 = q * JQ;
#pragma unroll
    for (int kk = 0; kk < JQ; ++kk) {
        double x = acc[kk].x, y = acc[kk].y;
#pragma unroll
        for (int o = L; o < 64; o <<= 1) {
            x += __shfl_xor(x, o, 64);
            y += __shfl_xor(y, o, 64);
        }
        if (lane < L && c0 + kk < J) {
            red[wave][2 * (c0 + kk)] = x;
            red[wave][2 * (c0 + kk) + 1] = y;
        }
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        double x = extra[e];
#pragma unroll
        for (int o = L; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) red[wave][2 * J + e] = x;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < NV; k += kB) {
        const double v = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
        part[(size_t)k * gridDim.x + blockIdx.x] = v;
    }
}

// Folded step j = J + 1, first pass (reads only): r' and w in registers;
// partials of [V(:,0:J)^H w ; r'^H w] (complex slots 0..J) and (w^H w, r'^H r')
// (complex slot J + 1): the CGS sums of step j and step j-1's deferred
// refinement check (kFinCgsFolded).  s = coef slot 1, t = coef slot 3.
template <class R, int J, int L>
__global__ __launch_bounds__(kB) void k_zfold_dots(int64_t n, const typename C2<R>::T* __restrict__ V,
                                                   int64_t ld, const typename C2<R>::T* __restrict__ r,
                                                   const typename C2<R>::T* __restrict__ y,
                                                   const double2* __restrict__ s,
                                                   const double2* __restrict__ t,
                                                   double* __restrict__ part,
                                                   const LzState* __restrict__ st) {
    if (st->abort) return;
    constexpr int JQ = (J + L - 1) / L;
    const bool fold = st->fold != 0;
    const double2 c = fold ? s[J - 1] : make_double2(0.0, 0.0);
    const int q = threadIdx.x % L, c0 = q * JQ;
    double2 acc[JQ];
#pragma unroll
    for (int kk = 0; kk < JQ; ++kk) acc[kk] = make_double2(0.0, 0.0);
    double ex[4] = {0.0, 0.0, 0.0, 0.0};  // r'^H w (re, im), w^H w, r'^H r' (group lane 0)
    const int64_t stride = (int64_t)gridDim.x * (kB / L);
    for (int64_t i = ((int64_t)blockIdx.x * kB + threadIdx.x) / L; i < n; i += stride) {
        double2 vr[JQ];
#pragma unroll
        for (int kk = 0; kk < JQ; ++kk)
            vr[kk] = c0 + kk < J ? ntld(V + i + (int64_t)(c0 + kk) * ld) : make_double2(0.0, 0.0);
        double2 rp = d2(r[i]), w = d2(y[i]);
        zfold_rw<R, J, L>(fold, vr, c0, s, t, c, rp, w);
#pragma unroll
        for (int kk = 0; kk < JQ; ++kk) {
            const double2 p = cmulc(vr[kk], w);
            acc[kk].x += p.x;
            acc[kk].y += p.y;
        }
        if (q == 0) {
            const double2 p = cmulc(rp, w);
            ex[0] += p.x;
            ex[1] += p.y;
            ex[2] += w.x * w.x + w.y * w.y;
            ex[3] += rp.x * rp.x + rp.y * rp.y;
        }
    }
    zsplit_partials<J, L, 4>(acc, ex, part);
}

// Folded step j = J + 1, second pass: the same r' and w; v_j = r' vs -> V(:,J)
// (k_zs_place's product), r_j = w vs - V(:,0:J+1) h -> r (in place; h = coef
// slot 0), partials of [V(:,0:J+1)^H r_j ; r_j^H r_j] (the layout of
// k_zs_update's: the next sweep's coefficients).  Column J (= v_j, known to
// every lane of the group) is group lane 0's extra term.
template <class R, int J, int L>
__global__ __launch_bounds__(kB) void k_zfold_update(int64_t n, typename C2<R>::T* __restrict__ V,
                                                     int64_t ld, const double2* __restrict__ h,
                                                     const double2* __restrict__ s,
                                                     const double2* __restrict__ t,
                                                     const typename C2<R>::T* __restrict__ y,
                                                     typename C2<R>::T* r, double* __restrict__ part,
                                                     const LzState* __restrict__ st) {
    if (st->abort) return;
    constexpr int JQ = (J + L - 1) / L;
    const bool fold = st->fold != 0;
    const double2 c = fold ? s[J - 1] : make_double2(0.0, 0.0);
    const double vs = st->vscale;
    const double2 hj = h[J];
    const int q = threadIdx.x % L, c0 = q * JQ;
    double2 acc[JQ];
#pragma unroll
    for (int kk = 0; kk < JQ; ++kk) acc[kk] = make_double2(0.0, 0.0);
    double ex[4] = {0.0, 0.0, 0.0, 0.0};  // v_j^H r_j (re, im), r_j^H r_j, 0 (group lane 0)
    typename C2<R>::T* vj = V + (int64_t)J * ld;
    const int64_t stride = (int64_t)gridDim.x * (kB / L);
    for (int64_t i = ((int64_t)blockIdx.x * kB + threadIdx.x) / L; i < n; i += stride) {
        double2 vr[JQ];
#pragma unroll
        for (int kk = 0; kk < JQ; ++kk)
            vr[kk] = c0 + kk < J ? ntld(V + i + (int64_t)(c0 + kk) * ld) : make_double2(0.0, 0.0);
        double2 rp = d2(r[i]), w = d2(y[i]);
        zfold_rw<R, J, L>(fold, vr, c0, s, t, c, rp, w);
        const auto vst = st2<R>(make_double2(rp.x * vs, rp.y * vs));
        const double2 v = d2(vst);
        double px = 0.0, py = 0.0;  // this lane's part of V(:,0:J) h
#pragma unroll
        for (int kk = 0; kk < JQ; ++kk) {
            if (c0 + kk < J) {
                const double2 p = cmul(vr[kk], h[c0 + kk]);
                px += p.x;
                py += p.y;
            }
        }
        px = gsum<L>(px);
        py = gsum<L>(py);
        const double2 pj = cmul(v, hj);
        const double2 rn = make_double2(w.x * vs - px - pj.x, w.y * vs - py - pj.y);
        const auto rs = st2<R>(rn);
        if (q == 0) {
            vj[i] = vst;
            r[i] = rs;
        }
        const double2 rd = d2(rs);
#pragma unroll
        for (int kk = 0; kk < JQ; ++kk) {
            const double2 p = cmulc(vr[kk], rd);
            acc[kk].x += p.x;
            acc[kk].y += p.y;
        }
        if (q == 0) {
            const double2 p = cmulc(v, rd);
            ex[0] += p.x;
            ex[1] += p.y;
            ex[2] += rd.x * rd.x + rd.y * rd.y;
        }
    }
    zsplit_partials<J, L, 4>(acc, ex, part);
}

template <class R>
__global__ void k_zs_zero_if(int64_t n, typename C2<R>::T* r, const LzState* st) {
    if (st->abort || !st->zero) return;
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride)
        r[i] = st2<R>(make_double2(0.0, 0.0));
}

// Single-block finalize over m complex slots (2m real; slot m-1 = the norm).
// Stage 1: the sums into s_sum (reads no state: issued alongside the state
// load, as k_finalize does; the caller's barrier publishes them).
__device__ __forceinline__ void zs_fin_sums(const double* __restrict__ part, int nblk, int m) {
    extern __shared__ double s_sum[];  // 2m doubles
    const int mt = 2 * m, t = threadIdx.x;
    {   // 32 slots per round, 32 threads per slot in four chains (as k_finalize)
        const int sub = t & 31;
        for (int k0 = 0; k0 < mt; k0 += 32) {
            const int k = k0 + (t >> 5);
            double s = 0.0;
            if (k < mt) {
                s = dev::slot_partial(part + (int64_t)k * nblk, nblk, sub);
            }
#pragma unroll
            for (int off = 16; off > 0; off >>= 1) s += __shfl_xor(s, off, 32);
            if (sub == 0 && k < mt) s_sum[k] = s;
        }
    }
}

// Stage 2: the phase logic (st: the LDS copy of the state, gate checked).
__device__ __forceinline__ void zs_fin_body(int m, int phase, int j, int rstart,
                                            double* __restrict__ sums,
                                            double2* __restrict__ coef, int cstride,
                                            double* __restrict__ rec, LzState* st,
                                            double2* __restrict__ hcol, int hld) {
    extern __shared__ double s_sum[];  // 2m doubles
    const int mt = 2 * m, nt = blockDim.x, t = threadIdx.x;
    for (int k = t; k < mt; k += nt) sums[k] = s_sum[k];
    const int jm = m - 1;
    const double nrm = sqrt(fabs(s_sum[2 * jm]));
    if (phase == dev::kFinCgs) {  // h(1:j,j) = V^H w (znaitr.f:567-577)
        for (int k = t; k < jm; k += nt) {
            const double2 h = make_double2(s_sum[2 * k], s_sum[2 * k + 1]);
            coef[k] = h;
            hcol[(int64_t)(j - 1) * hld + k] = h;
        }
        if (t == 0) {
            st->zero = 0;
            st->dgks = 0;
            st->wnorm = nrm;
            st->beta = (j == 1 || rstart) ? 0.0 : st->rnorm;  // h(j,j-1)
            rec[j - 1] = st->beta;
        }
        return;
    }
    if (phase == dev::kFinNorm) {
        if (t == 0) st->rnorm = nrm;
        return;
    }
    if (phase == dev::kFinCgsFolded) {
        // step j of a folded cycle (sums of k_zfold_dots: slots 0..j-2 V^H w,
        // j-1 r'^H w, j (w^H w, r'^H r')): (1) step j-1's deferred first
        // refinement check on ||r'|| (a needed second one parks the cycle, the
        // host finishes it), (2) the CGS coefficients of v_j = r'/||r'||,
        // rescaled from the raw residual's sums (st.vscale)
        __shared__ int s_go;
        if (t == 0) {
            if (st->dgks == 1) {
                const double rn = sqrt(fabs(s_sum[2 * jm + 1]));
                if (rn > 0.717 * st->rnorm && !st->force_dgks2) {
                    st->rnorm = rn;
                    st->dgks = 0;
                } else {
                    st->nitref += 1;
                    st->rnorm = rn;
                    st->dgks = 2;
                    st->abort = 2;
                    st->abort_j = j - 1;
                }
            }
            const double rn = st->rnorm;
            int go = 0;
            if (st->abort) {
            } else if (!(rn > 0.0)) {  // invariant subspace at step j (znaitr.f:373)
                st->abort = 1;
                st->abort_j = j;
            } else if (rn < 1e-150 || rn > 1e150) {  // raw-vector range guard: the host
                st->abort = 3;                       // redoes step j with v_j formed first
                st->abort_j = j;
            } else {
                go = 1;
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go) return;
        const double vs = 1.0 / st->rnorm;  // k_zs_place's factor for rnorm >= safmin
        const int J = j - 1;
        for (int k = t; k < J; k += nt) {
            const double2 h = make_double2(s_sum[2 * k] * vs, s_sum[2 * k + 1] * vs);
            coef[k] = h;
            hcol[(int64_t)(j - 1) * hld + k] = h;
        }
        if (t == 0) {  // v_j^H w = vs^2 r'^H (A r')
            const double2 h = make_double2((s_sum[2 * J] * vs) * vs, (s_sum[2 * J + 1] * vs) * vs);
            coef[J] = h;
            hcol[(int64_t)(j - 1) * hld + J] = h;
            st->vscale = vs;
            st->zero = 0;
            st->dgks = 0;
            st->wnorm = sqrt(fabs(s_sum[2 * jm])) * vs;
            st->beta = (j == 1 || rstart) ? 0.0 : st->rnorm;
            rec[j - 1] = st->beta;
        }
        return;
    }
    if (phase == dev::kFinFoldCoef2) {  // a folded park's second sweep (host path)
        for (int k = t; k < jm; k += nt) {
            const double2 c = make_double2(s_sum[2 * k], s_sum[2 * k + 1]);
            coef[(int64_t)2 * cstride + k] = c;
            double2 h = hcol[(int64_t)(j - 1) * hld + k];
            h.x += c.x;
            h.y += c.y;
            hcol[(int64_t)(j - 1) * hld + k] = h;
        }
        return;
    }
    // refinement phases (znaitr.f:651-780): decision on rnorm = ||r||, then the
    // next sweep's coefficients V^H r into coef slot `take`
    __shared__ int s_take;
    const bool pfold = phase == dev::kFinPostCgsFold;
    if (t == 0) {
        int take = 0;
        if (phase == dev::kFinPostCgs || pfold) {
            st->rnorm = nrm;
            if (nrm > 0.717 * st->wnorm) {
                st->dgks = 0;
            } else {
                st->dgks = 1;
                st->nrorth += 1;
                take = 1;
            }
        } else if (phase == dev::kFinDgks1 || phase == dev::kFinDgks1Lazy) {
            if (nrm > 0.717 * st->rnorm && !st->force_dgks2) {
                st->rnorm = nrm;
                st->dgks = 0;
            } else {
                st->nitref += 1;
                st->rnorm = nrm;
                st->dgks = 2;
                take = 2;
                if (phase == dev::kFinDgks1Lazy) {
                    st->abort = 2;
                    st->abort_j = j;
                }
            }
        } else {  // kFinDgks2: a second failure gives up (r = 0)
            if (nrm > 0.717 * st->rnorm) {
                st->rnorm = nrm;
            } else {
                st->nitref += 1;
                st->zero = 1;
                st->rnorm = 0.0;
            }
            st->dgks = 0;
        }
        if (pfold) st->fold = take;
        s_take = take;
    }
    __syncthreads();
    // the correction of THIS sweep was added when its coefficients were taken;
    // the h(1:j,j) daxpy (znaitr.f:681) happens with the coefficients it used
    const int take = s_take;
    if (pfold && take) {
        // t = H_j s for the next step's fold, one row per thread: H(i, q) from
        // the records (rows 0..q of column q; this step's column is h + s, read
        // before the daxpy below), the real subdiagonal H(q+1, q) = rec[q+1]
        for (int i = t; i < jm; i += nt) {
            double tx = 0.0, ty = 0.0;
            for (int q = i > 0 ? i - 1 : 0; q < jm; ++q) {
                double2 hq;
                if (i <= q) {
                    hq = hcol[(int64_t)q * hld + i];
                    if (q == jm - 1) {
                        hq.x += s_sum[2 * i];
                        hq.y += s_sum[2 * i + 1];
                    }
                } else {
                    hq = make_double2(rec[q + 1], 0.0);
                }
                const double sx = s_sum[2 * q], sy = s_sum[2 * q + 1];
                tx = fma(hq.x, sx, fma(-hq.y, sy, tx));
                ty = fma(hq.x, sy, fma(hq.y, sx, ty));
            }
            coef[(int64_t)3 * cstride + i] = make_double2(tx, ty);
        }
        __syncthreads();
    }
    if (take) {
        for (int k = t; k < jm; k += nt) {
            const double2 c = make_double2(s_sum[2 * k], s_sum[2 * k + 1]);
            coef[(int64_t)take * cstride + k] = c;
            double2 h = hcol[(int64_t)(j - 1) * hld + k];
            h.x += c.x;
            h.y += c.y;
            hcol[(int64_t)(j - 1) * hld + k] = h;
        }
    }
}

// The state is read once into LDS and written back once (as k_finalize): the
// phase logic is one thread's chain of dependent state accesses.
__global__ __launch_bounds__(1024) void k_zs_finalize(const double* __restrict__ part, int nblk, int m,
                                                      int phase, int j, int rstart, int gate,
                                                      double* __restrict__ sums,
                                                      double2* __restrict__ coef, int cstride,
                                                      double* __restrict__ rec,
                                                      LzState* __restrict__ st,
                                                      double2* __restrict__ hcol, int hld) {
    __shared__ LzState s_st;
    if (threadIdx.x == 0) s_st = *st;
    zs_fin_sums(part, nblk, m);  // overlaps the state load
    __syncthreads();
    if (zgate_closed(&s_st, gate)) return;
    zs_fin_body(m, phase, j, rstart, sums, coef, cstride, rec, &s_st, hcol, hld);
    __syncthreads();
    if (threadIdx.x == 0) *st = s_st;
}

inline int sgrid(const Ws& ws) { return ws.nblk; }

}  // namespace

template <class R>
void step_place(const Ws& ws, int64_t n, const R* r, R* vcol, R* copy1, R* copy2, double safmin,
                int j) {
    using T = typename C2<R>::T;
    int64_t g = (n + kB - 1) / kB;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_zs_place<R>, dim3((unsigned)g), dim3(kB), 0, ws.stream, n,
                       reinterpret_cast<const T*>(r), reinterpret_cast<T*>(vcol),
                       reinterpret_cast<T*>(copy1), reinterpret_cast<T*>(copy2), safmin, ws.st, j);
}

#define AHIP_ZS_C16(M) \
    M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15) M(16)
#define AHIP_ZS_C32(M) \
    M(17) M(18) M(19) M(20) M(21) M(22) M(23) M(24) M(25) M(26) M(27) M(28) M(29) M(30) M(31) M(32)
#define AHIP_ZS_C39(M) M(33) M(34) M(35) M(36) M(37) M(38) M(39)
#define AHIP_ZS_C40(M) AHIP_ZS_C39(M) M(40)

template <class R>
void step_dots(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, const R* u, int gate) {
    using T = typename C2<R>::T;
    const T* V2 = reinterpret_cast<const T*>(V);
    const T* u2 = reinterpret_cast<const T*>(u);
    const dim3 g(sgrid(ws)), b(kB);
    if (j == 0) {
        hipLaunchKernelGGL((k_zs_dots<R, 1, true>), g, b, 0, ws.stream, n, 0, V2, (int64_t)0, u2,
                           ws.part, 0, ws.st, gate);  // J = 1 over column 0 is unused: norm only
        return;
    }
    for (int c0 = 0; c0 < j; c0 += 16) {  // 16 complex columns per pass over u
        const int jc = j - c0 < 16 ? j - c0 : 16;
        const bool wm = c0 == 0;
        switch (jc) {
#define AHIP_ZS_DOTS(J)                                                                            \
    case J:                                                                                        \
        if (wm)                                                                                    \
            hipLaunchKernelGGL((k_zs_dots<R, J, true>), g, b, 0, ws.stream, n, c0, V2, ld, u2,     \
                               ws.part, j, ws.st, gate);                                           \
        else                                                                                       \
            hipLaunchKernelGGL((k_zs_dots<R, J, false>), g, b, 0, ws.stream, n, c0, V2, ld, u2,    \
                               ws.part, j, ws.st, gate);                                           \
        break;
            AHIP_ZS_C16(AHIP_ZS_DOTS)
#undef AHIP_ZS_DOTS
            default: break;
        }
    }
}

// widest fused update; AHIP_ZFUSE_MAX=32 restores the round-2 split above 32
// columns (read per call: a test compares both forms in one process)
static int fused_max() {
    const char* e = getenv("AHIP_ZFUSE_MAX");
    const int v = e ? atoi(e) : 40;
    return v >= 1 && v <= 40 ? v : 40;
}

template <class R>
void step_update(const Ws& ws, int64_t n, int j, const R* V, int64_t ld, int which, const R* rin,
                 R* rout, bool spec, int gate) {
    using T = typename C2<R>::T;
    const T* V2 = reinterpret_cast<const T*>(V);
    const double2* c = reinterpret_cast<const double2*>(ws.coef) + (size_t)which * ws.cstride;
    const T* ri = reinterpret_cast<const T*>(rin);
    T* ro = reinterpret_cast<T*>(rout);
    const dim3 g(sgrid(ws)), b(kB);
    // up to 40 columns (config 5's ncv) the update and the next sweep's partials
    // share one pass: the row's V entries stay in registers (J = 40: 256 VGPRs +
    // 82 AGPRs, no scratch); the sums are those of step_dots over rout, term for
    // term, so the partials are the same either way
    if (j >= 1 && j <= fused_max()) {
        switch (j) {
#define AHIP_ZS_UPD(J)                                                                             \
    case J:                                                                                        \
        if (spec)                                                                                  \
            hipLaunchKernelGGL((k_zs_update<R, J, true>), g, b, 0, ws.stream, n, V2, ld, c, ri,    \
                               ro, ws.part, ws.st, gate);                                          \
        else                                                                                       \
            hipLaunchKernelGGL((k_zs_update<R, J, false>), g, b, 0, ws.stream, n, V2, ld, c, ri,   \
                               ro, ws.part, ws.st, gate);                                          \
        break;
            AHIP_ZS_C16(AHIP_ZS_UPD)
            AHIP_ZS_C32(AHIP_ZS_UPD)
            AHIP_ZS_C40(AHIP_ZS_UPD)
#undef AHIP_ZS_UPD
            default: break;
        }
    } else {  // wider bases: plain update, then the partials in separate passes
        hipLaunchKernelGGL(k_zs_update_generic<R>, g, b, 0, ws.stream, n, j, V2, ld, c, ri, ro, ws.st,
                           gate);
        if (spec) step_dots<R>(ws, n, j, V, ld, rout, gate);
    }
}

// lanes a row of the fold passes: the row's complex V entries and accumulators
// per lane stay at <= 10 each (two or more waves a SIMD)
constexpr int zfold_lanes(int J) { return J >= 12 ? 4 : J >= 6 ? 2 : 1; }

// folded step j (2 <= j <= kZFoldMax + 1; J = j - 1 formed columns): complex128 only
// (the free-running complex engine is znaupd's)
void step_fold_dots(const Ws& ws, int64_t n, int j, const double* V, int64_t ld, const double* r,
                    const double* y) {
    const double2* V2 = reinterpret_cast<const double2*>(V);
    const double2* r2 = reinterpret_cast<const double2*>(r);
    const double2* y2 = reinterpret_cast<const double2*>(y);
    const double2* s = reinterpret_cast<const double2*>(ws.coef) + ws.cstride;
    const double2* tt = reinterpret_cast<const double2*>(ws.coef) + 3 * (size_t)ws.cstride;
    const dim3 g(sgrid(ws)), b(kB);
    switch (j - 1) {
#define AHIP_ZF_DOTS(J)                                                                            \
    case J:                                                                                        \
        hipLaunchKernelGGL((k_zfold_dots<double, J, zfold_lanes(J)>), g, b, 0, ws.stream, n, V2, ld, \
                           r2, y2, s, tt, ws.part, ws.st);                                         \
        break;
        AHIP_ZS_C16(AHIP_ZF_DOTS)
        AHIP_ZS_C32(AHIP_ZF_DOTS)
        AHIP_ZS_C39(AHIP_ZF_DOTS)
#undef AHIP_ZF_DOTS
        default: break;
    }
}

void step_fold_update(const Ws& ws, int64_t n, int j, double* V, int64_t ld, const double* y,
                      double* r) {
    double2* V2 = reinterpret_cast<double2*>(V);
    const double2* y2 = reinterpret_cast<const double2*>(y);
    double2* r2 = reinterpret_cast<double2*>(r);
    const double2* h = reinterpret_cast<const double2*>(ws.coef);
    const double2* s = h + ws.cstride;
    const double2* tt = h + 3 * (size_t)ws.cstride;
    const dim3 g(sgrid(ws)), b(kB);
    switch (j - 1) {
#define AHIP_ZF_UPD(J)                                                                             \
    case J:                                                                                        \
        hipLaunchKernelGGL((k_zfold_update<double, J, zfold_lanes(J)>), g, b, 0, ws.stream, n, V2, ld, \
                           h, s, tt, y2, r2, ws.part, ws.st);                                      \
        break;
        AHIP_ZS_C16(AHIP_ZF_UPD)
        AHIP_ZS_C32(AHIP_ZF_UPD)
        AHIP_ZS_C39(AHIP_ZF_UPD)
#undef AHIP_ZF_UPD
        default: break;
    }
}

void step_finalize(const Ws& ws, int m, dev::FinPhase ph, int j, int rstart, int gate) {
    hipLaunchKernelGGL(k_zs_finalize, dim3(1), dim3(1024), sizeof(double) * 2 * (size_t)m, ws.stream,
                       ws.part, ws.nblk, m, (int)ph, j, rstart, gate, ws.sums,
                       reinterpret_cast<double2*>(ws.coef), ws.cstride, ws.rec, ws.st,
                       reinterpret_cast<double2*>(ws.hcol), ws.hld);
}

template <class R>
void step_zero_if(const Ws& ws, int64_t n, R* r) {
    using T = typename C2<R>::T;
    int64_t g = (n + kB - 1) / kB;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_zs_zero_if<R>, dim3((unsigned)g), dim3(kB), 0, ws.stream, n,
                       reinterpret_cast<T*>(r), ws.st);
}

#define AHIP_ZSINST(R)                                                                             \
    template void step_place<R>(const Ws&, int64_t, const R*, R*, R*, R*, double, int);           \
    template void step_dots<R>(const Ws&, int64_t, int, const R*, int64_t, const R*, int);         \
    template void step_update<R>(const Ws&, int64_t, int, const R*, int64_t, int, const R*, R*,   \
                                 bool, int);                                                       \
    template void step_zero_if<R>(const Ws&, int64_t, R*);
AHIP_ZSINST(double)
AHIP_ZSINST(float)
#undef AHIP_ZSINST

}  // namespace ahip::zdev
