// The folded Lanczos step (free-running dsaupd; sym.cpp saitr):
// step j-1's DGKS sweep applied inside step j's two passes over V.
//   k_fold_dots    r' and w = A r' in registers, [V' w ; r'' w ; w'w], r''r'
//   k_fold_update  the same r' and w, v_j = r'/rnorm, r_j = w/rnorm - V h,
//                  [V' r_j ; r_j' r_j]
// Reference: SRC/dsaitr.f:569-583 (CGS), :680-692 (DGKS), :438-474 (v_j, OP).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device.hpp"
#include "passes.hpp"

namespace ahip::dev {

namespace {

// ------------------------------------------------------------------- fold ---
// w = A r' of a folded step from y = A r (r: the residual before its DGKS
// sweep, r' = r - V s after it): A r' = y - A V s and, by the Lanczos relation
// A V_J = V_J T_J + r' e_J', A V s = V_J (T_J s) + s_J r'.  t = T_J s, c = s_J.
// Explicit fma: the fold pass and the update pass evaluate it bit-identically.
template <int JN>
__device__ __forceinline__ double fold_w(double y, const double* vrow, const double* __restrict__ t,
                                         double c, double rp) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < JN; ++k) a = fma(vrow[k], t[k], a);
    a = fma(c, rp, a);
    return y - a;
}

// r' = r - V(:,0:J) s of a folded step (explicit fma: k_fold_dots and
// k_fold_update form it bit-identically)
template <int J>
__device__ __forceinline__ double fold_r(double r, const double* vrow, const double* __restrict__ s) {
    double sv = 0.0;
#pragma unroll
    for (int k = 0; k < J; ++k) sv = fma(vrow[k], s[k], sv);
    return r - sv;
}

// Folded step j (device.hpp fold_dots): J = j-1 formed columns V(:,0:J); the
// pass forms r' and w in registers -- a pure read pass: stores in a read
// stream cost far more than their bytes (tools/stream_bench.hip: one written
// n-vector takes a 1.6 GB read pass from 6.8 to 6.0 TB/s), so r' is formed
// again by k_fold_update, which stores v_j -- and the partials of
// [V(:,0:J)' w ; r'' w ; w'w] (slots 0..J+1) and r''r' (region 2, slot 0).
// Without a pending sweep (st.fold == 0) r' = r and w = y exactly.
template <class R, int J, int POL = kPolNt>
__global__ __launch_bounds__(kBlock) void k_fold_dots(int64_t n, R* __restrict__ V, int64_t ld,
                                                      const R* __restrict__ r,
                                                      const R* __restrict__ y,
                                                      const double* __restrict__ s,
                                                      const double* __restrict__ t,
                                                      double* __restrict__ part, int pstride,
                                                      const LzState* __restrict__ st) {
    if (st->abort) return;
    const bool fold = st->fold != 0;
    const double c = fold ? s[J - 1] : 0.0;
    double acc[J + 2];
#pragma unroll
    for (int k = 0; k < J + 2; ++k) acc[k] = 0.0;
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x; it < n; it += stride) {
        const int64_t i = POL == kPolNtRev ? n - 1 - it : it;
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

// Folded step j, second pass (J = j-1 formed columns; V(:,J) receives v_j):
//   r' = r - V(:,0:J) s, w = y - V t - c r'       (as k_fold_dots; st.fold)
//   v_j = r' * vscale -> V(:,J)                     (k_place's product)
//   r_j = w * vscale - V(:,0:J+1) h -> r (in place) and x2 (a distributed SpMV's x)
//   partials of [V(:,0:J+1)' r_j ; r_j' r_j]        (region 1, J+2 slots)
// h = coef slot 0, s = slot 1, t = slot 3.  NTS: non-temporal stores.
template <class R, int J, int POL = kPolNt, bool NTS = false>
__global__ __launch_bounds__(kBlock) void k_fold_update(int64_t n, R* __restrict__ V, int64_t ld,
                                                        const double* __restrict__ h,
                                                        const double* __restrict__ s,
                                                        const double* __restrict__ t,
                                                        const R* __restrict__ y, R* r,
                                                        R* __restrict__ x2,
                                                        double* __restrict__ part,
                                                        const LzState* __restrict__ st) {
    if (st->abort) return;
    const bool fold = st->fold != 0;
    const double c = fold ? s[J - 1] : 0.0;
    const double vs = st->vscale;
    double acc[J + 1];
#pragma unroll
    for (int k = 0; k < J + 1; ++k) acc[k] = 0.0;
    double rr = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    R* vj = V + (int64_t)J * ld;
    auto st_ = [](R* p, R v) {
        if constexpr (NTS) __builtin_nontemporal_store(v, p);
        else *p = v;
    };
    for (int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x; it < n; it += stride) {
        const int64_t i = POL == kPolNtRev ? n - 1 - it : it;
        double vrow[J + 1];
#pragma unroll
        for (int k = 0; k < J; ++k) vrow[k] = vld<POL>(V + i + (int64_t)k * ld);
        double rp = (double)r[i], w = (double)y[i];
        if (fold) {
            rp = (double)(R)fold_r<J>(rp, vrow, s);
            w = fold_w<J>(w, vrow, t, c, rp);
        }
        const R v = (R)(rp * vs);
        st_(vj + i, v);
        vrow[J] = (double)v;
        double sh = 0.0;
#pragma unroll
        for (int k = 0; k < J + 1; ++k) sh += vrow[k] * h[k];
        const R rn = (R)(w * vs - sh);
        st_(r + i, rn);
        if (x2) st_(x2 + i, rn);
        const double rd = (double)rn;
        rr += rd * rd;
#pragma unroll
        for (int k = 0; k < J + 1; ++k) acc[k] += vrow[k] * rd;
    }
    block_partials<J + 1>(acc, J + 1, rr, true, part, 0, J + 1);
}

}  // namespace

template <class R>
void fold_dots(const Workspace& ws, int64_t n, int j, R* V, int64_t ld, const R* r, const R* y) {
    // j = step (2 <= j <= 64): V(:,0:j-1) formed, V(:,j-1) receives r'
    ProfScope ps(kProfDots, ws.stream, (double)sizeof(R) * n * (j + 1));
    const dim3 g(ws.nblk), b(kBlock);
    const double* s = ws.coef + ws.stride;
    const double* t = ws.coef + 3 * (size_t)ws.stride;
    auto go = [&](auto kern) {
        AHIP_LAUNCH(kern, g, b, 0, ws.stream, n, V, ld, r, y, s, t, ws.part, ws.stride, ws.st);
    };
    switch (j - 1) {
#define AHIP_FOLD_CASE(J)                                                                          \
    case J:                                                                                        \
        if (ws.v_plain) go(k_fold_dots<R, J, kPolPlain>);                                          \
        else go(k_fold_dots<R, J>);                                                                \
        break;
        AHIP_CASES_1_32(AHIP_FOLD_CASE)
        AHIP_CASES_33_64(AHIP_FOLD_CASE)
#undef AHIP_FOLD_CASE
        default: break;
    }
}

template <class R>
void fold_update(const Workspace& ws, int64_t n, int j, R* V, int64_t ld, const R* y, R* r, R* x2) {
    // non-temporal stores of v_j and r_j (AHIP_FOLD_NTS=0: plain): same-box A/B
    // 47.5 vs 46.5 iters/s -- the SpMV and the fold pass that follow run faster
    static const bool nts = [] {
        const char* e = getenv("AHIP_FOLD_NTS");
        return !(e && e[0] == '0');
    }();
    ProfScope ps(kProfUpdate, ws.stream, (double)sizeof(R) * n * (j + 3 + (x2 ? 1 : 0)));
    const dim3 g(ws.nblk), b(kBlock);
    const double* h = ws.coef;
    const double* s = ws.coef + ws.stride;
    const double* t = ws.coef + 3 * (size_t)ws.stride;
    auto go = [&](auto kern) {
        AHIP_LAUNCH(kern, g, b, 0, ws.stream, n, V, ld, h, s, t, y, r, x2, ws.part, ws.st);
    };
    switch (j - 1) {
#define AHIP_FOLDU_CASE(J)                                                                         \
    case J:                                                                                        \
        if (ws.v_plain) nts ? go(k_fold_update<R, J, kPolPlain, true>)                             \
                            : go(k_fold_update<R, J, kPolPlain>);                                  \
        else nts ? go(k_fold_update<R, J, kPolNtRev, true>) : go(k_fold_update<R, J, kPolNtRev>);  \
        break;
        AHIP_CASES_1_32(AHIP_FOLDU_CASE)
        AHIP_CASES_33_64(AHIP_FOLDU_CASE)
#undef AHIP_FOLDU_CASE
        default: break;
    }
}

template void fold_dots<double>(const Workspace&, int64_t, int, double*, int64_t, const double*,
                                const double*);
template void fold_dots<float>(const Workspace&, int64_t, int, float*, int64_t, const float*,
                               const float*);
template void fold_update<double>(const Workspace&, int64_t, int, double*, int64_t, const double*,
                                  double*, double*);
template void fold_update<float>(const Workspace&, int64_t, int, float*, int64_t, const float*,
                                 float*, float*);

}  // namespace ahip::dev
