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
    // refinement phases (znaitr.f:651-780): decision on rnorm = ||r||, then the
    // next sweep's coefficients V^H r into coef slot `take`
    __shared__ int s_take;
    if (t == 0) {
        int take = 0;
        if (phase == dev::kFinPostCgs) {
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
        s_take = take;
    }
    __syncthreads();
    // the correction of THIS sweep was added when its coefficients were taken;
    // the h(1:j,j) daxpy (znaitr.f:681) happens with the coefficients it used
    const int take = s_take;
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
#define AHIP_ZS_C40(M) M(33) M(34) M(35) M(36) M(37) M(38) M(39) M(40)

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
