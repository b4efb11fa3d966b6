// The single-block finalize of the n-length passes' partial sums: fixed-order
// slot sums and the phase logic of the Lanczos / Arnoldi step (the 0.717
// DGKS decisions of SRC/dsaitr.f:634-781, taken on the device).  Shared by
// kernels.hip (k_finalize) and spmv_sym.hip (a finalize deferred into the
// symmetric SpMV's combine kernel).
#pragma once
#include <hip/hip_runtime.h>

#include "device.hpp"
#include "passes.hpp"
#include "reduce.hpp"

namespace ahip::dev {
namespace {

constexpr int kFoldRecMax = 2 * 66;  // T records staged for the fold's t (j <= 64)
constexpr int kFoldHMax = 64;        // HS: H(0:j, 0:j) staged for the Arnoldi fold's t = H s

// The finalize's workgroup-shared state, in LDS the launch provides (dynamic
// LDS of k_finalize / the combine kernel, or a window of the SpMV kernel that
// carries a deferred finalize): the state copy, the fold's T records, the
// decisions, then the m + m2 sums.
struct FinLds {
    LzState st;
    double rec[kFoldRecMax];
    int take, take2, go, pad_;
    double sum[1];  // m + m2 doubles from here
};
__host__ __device__ constexpr size_t fin_lds_bytes(int mt) {
    return sizeof(FinLds) + sizeof(double) * (size_t)(mt > 1 ? mt - 1 : 0);
}

// One refinement decision (SRC/dsaitr.f:634-781) on the sums of [V'r ; r'r]
// (jm = index of r'r) for step jj; returns `take` (which coefficient slot the
// next sweep uses, 0 for none).  Thread 0 only.
__device__ int refine_decision(int phase, const double* ss, int jm, int jj, int rstart_jj,
                               LzState* st, double* rec, bool defer = false) {
    const double rn = sqrt(fabs(ss[jm]));
    int take = 0;
    if (phase == kFinPostCgs) {
        st->rnorm = rn;
        if (rn > 0.717 * st->wnorm) {
            st->dgks = 0;
        } else {
            st->dgks = 1;
            st->nrorth += 1;
            take = 1;
        }
    } else if (phase == kFinDgks1 || phase == kFinDgks1Lazy) {
        if (rn > 0.717 * st->rnorm && !st->force_dgks2) {
            st->rnorm = rn;
            st->dgks = 0;
        } else {
            st->nitref += 1;
            st->rnorm = rn;
            st->dgks = 2;
            take = 2;
            if (phase == kFinDgks1Lazy) {  // rare: the host runs the second sweep
                st->abort = 2;
                st->abort_j = jj;
            }
        }
    } else {  // kFinDgks2
        if (rn > 0.717 * st->rnorm) {
            st->rnorm = rn;
        } else {
            st->nitref += 1;
            st->zero = 1;
            st->rnorm = 0.0;
        }
        st->dgks = 0;
    }
    if (take && !defer) {  // defer: a folded park; kFinFoldCoef2 does this on the host path
        st->alpha += ss[jm - 1];
        if (jj == 1 || rstart_jj) st->beta = 0.0;
    }
    rec[2 * (jj - 1)] = st->alpha;
    rec[2 * (jj - 1) + 1] = st->beta;
    return take;
}

// Single-block finalize: fixed-order sums of the per-block partials (region 1:
// m slots of `part`; region 2: m2 slots of `part2`, only for kFinCgsChained)
// and the phase logic.  from_sums: the m + m2 sums are already in `sums`
// (reduced, and allreduced across ranks).
// Stage 1 (fin_sums): the m + m2 sums into the dynamic-LDS s_sum.  It reads
// nothing of the state, so k_finalize issues it before the state load has
// returned (the two memory round trips overlap); the caller's barrier
// publishes s_sum.
__device__ __forceinline__ void fin_sums(const double* __restrict__ part, int nblk, int from_sums,
                                         int m, const double* __restrict__ sums,
                                         const double* __restrict__ part2, int m2,
                                         double* s_sum) {
    // the m + m2 (<= 2 ncv + 4) sums are staged in LDS sized by the launch, so
    // any ncv the argument checks accept fits
    const int nt = blockDim.x;
    const int mt = m + m2;
    if (from_sums) {  // already reduced (and allreduced across ranks) in `sums`
        for (int k = threadIdx.x; k < mt; k += nt) s_sum[k] = sums[k];
    } else {
        // 32 slots per round, 32 threads (half a wave) per slot: thread `sub`
        // sums blocks sub, sub+32, ... in four independent chains (coalesced
        // 256-B rows of the k-major partials), then the half wave reduces
        const int sub = threadIdx.x & 31;
        for (int k0 = 0; k0 < mt; k0 += 32) {
            const int k = k0 + (threadIdx.x >> 5);
            double s = 0.0;
            if (k < mt) {
                const double* p = k < m ? part + (int64_t)k * nblk : part2 + (int64_t)(k - m) * nblk;
                s = slot_partial(p, nblk, sub);
            }
#pragma unroll
            for (int off = 16; off > 0; off >>= 1) s += __shfl_xor(s, off, 32);
            if (sub == 0 && k < mt) s_sum[k] = s;
        }
    }
}

// Stage 2: the phase logic on s_sum; st is the block's LDS copy of the state
// (k_finalize), already checked against the gate.
__device__ __forceinline__ void fin_body(int m, int phase, int j, int rstart,
                                         double* __restrict__ sums, double* __restrict__ coef,
                                         int cstride, double* __restrict__ rec, LzState* st,
                                         double* __restrict__ hcol, int hld, int m2,
                                         int rstart_prev, FinLds* L,
                                         const double* s_h = nullptr) {
    double* const s_sum = L->sum;
    double* const s_rec = L->rec;
    int& s_take2 = L->take2;
    int& s_go = L->go;
    int& s_take = L->take;
    const int nt = blockDim.x;
    const int mt = m + m2;
    const int t = threadIdx.x;
    for (int k = t; k < mt; k += nt) sums[k] = s_sum[k];
    const int jm = m - 1;  // index of the w'u / r'r slot
    if (phase == kFinCgsChained || phase == kFinCgsFolded) {
        // (1) the first DGKS refinement of step j-1, deferred to here: region 2
        //     holds its [V_{j-1}' r ; r'r] (SRC/dsaitr.f:730-771) -- folded: r'r only
        const bool folded = phase == kFinCgsFolded;
        if (t == 0) {
            s_take2 = 0;
            if (st->dgks == 1)
                s_take2 = refine_decision(kFinDgks1Lazy, s_sum + m, m2 - 1, j - 1, rstart_prev, st,
                                          rec, folded);
            // (2) v_j = r / rnorm was NOT formed: the SpMV ran on the raw residual
            //     (A r = rnorm * A v_j), so the CGS sums are rescaled here and the
            //     update pass normalises V(:,j) in place (scale st->vscale)
            const double rn = st->rnorm;
            s_go = 0;
            if (st->abort) {
            } else if (!(rn > 0.0)) {  // invariant subspace at step j (SRC/dsaitr.f:378)
                st->abort = 1;
                st->abort_j = j;
            } else if (rn < 1e-150 || rn > 1e150) {  // raw-vector range guard: the host
                st->abort = 3;                       // redoes step j with v_j formed first
                st->abort_j = j;
            } else {
                s_go = 1;
            }
        }
        __syncthreads();
        if (s_take2 && !folded) {  // the parked second refinement's coefficients (host path)
            for (int k = t; k < m2 - 1; k += nt) {
                coef[2 * cstride + k] = s_sum[m + k];
                if (hld) hcol[(int64_t)(j - 2) * hld + k] += s_sum[m + k];
            }
        }
        if (!s_go) return;
        const double vs = 1.0 / st->rnorm;  // k_place's factor for rnorm >= safmin
        for (int k = t; k < jm - 1; k += nt) {  // h(k) = V_k' w = vs * V_k' (A r)
            const double h = s_sum[k] * vs;
            coef[k] = h;
            if (hld) hcol[(int64_t)(j - 1) * hld + k] = h;
        }
        if (t == 0) {
            const double hj = (s_sum[jm - 1] * vs) * vs;  // v_j' w = vs^2 r' (A r)
            coef[jm - 1] = hj;
            if (hld) hcol[(int64_t)(j - 1) * hld + jm - 1] = hj;
            st->vscale = vs;
            st->zero = 0;
            st->dgks = 0;
            st->wnorm = sqrt(fabs(s_sum[jm])) * vs;
            st->alpha = hj;
            st->beta = (j == 1 || rstart) ? 0.0 : st->rnorm;
            rec[2 * (j - 1)] = st->alpha;
            rec[2 * (j - 1) + 1] = st->beta;
        }
        return;
    }
    if (phase == kFinCgs) {
        for (int k = t; k < jm; k += nt) {
            coef[k] = s_sum[k];
            if (hld) hcol[(int64_t)(j - 1) * hld + k] = s_sum[k];  // h(1:j,j) (dnaitr.f:566)
        }
        if (t == 0) {
            st->vscale = 1.0;
            st->zero = 0;
            st->dgks = 0;
            st->wnorm = sqrt(fabs(s_sum[jm]));
            st->alpha = s_sum[jm - 1];
            st->beta = (j == 1 || rstart) ? 0.0 : st->rnorm;
            rec[2 * (j - 1)] = st->alpha;
            rec[2 * (j - 1) + 1] = st->beta;
        }
        return;
    }
    if (phase == kFinNorm) {
        if (t == 0) st->rnorm = sqrt(fabs(s_sum[jm]));
        return;
    }
    if (phase == kFinRaw) return;
    if (phase == kFinCoef) {
        for (int k = t; k < jm; k += nt) coef[k] = s_sum[k];
        return;
    }
    if (phase == kFinFoldCoef2) {  // a folded park's second sweep (host path)
        for (int k = t; k < jm; k += nt) {
            coef[2 * cstride + k] = s_sum[k];
            if (hld) hcol[(int64_t)(j - 1) * hld + k] += s_sum[k];  // daxpy into h(1:j,j)
        }
        if (t == 0) {
            st->alpha += s_sum[jm - 1];
            if (j == 1 || rstart) st->beta = 0.0;
            rec[2 * (j - 1)] = st->alpha;
            rec[2 * (j - 1) + 1] = st->beta;
        }
        return;
    }
    // refinement phases share the "speculative coefficients" layout
    const bool pfold = phase == kFinPostCgsFold;
    if (t == 0) {
        s_take = refine_decision(pfold ? (int)kFinPostCgs : phase, s_sum, jm, j, rstart, st, rec);
        if (pfold) {
            // t = T_j s for the next step's fold: T tridiagonal, alpha_k = rec[2(k-1)]
            // (step j's includes s_j), beta_k = rec[2(k-1)+1] = T(k, k-1); the
            // records come from the LDS copy (step j's just updated)
            st->fold = s_take;
            s_rec[2 * (j - 1)] = st->alpha;
            s_rec[2 * (j - 1) + 1] = st->beta;
        }
    }
    __syncthreads();
    const int take = s_take;
    if (pfold && take && !hld) {
        // t = T s, one row per thread (Arnoldi: H s below); the same three
        // terms in the same order as a serial loop
        for (int k = t; k < jm; k += nt) {
            double tk = s_rec[2 * k] * s_sum[k];
            if (k > 0) tk = fma(s_rec[2 * k + 1], s_sum[k - 1], tk);
            if (k + 1 < jm) tk = fma(s_rec[2 * (k + 1) + 1], s_sum[k + 1], tk);
            coef[3 * cstride + k] = tk;
        }
    }
    if (pfold && take && hld) {
        // Arnoldi: t = H_j s with the full upper-Hessenberg records (column q of
        // H: hcol rows 0..q, subdiagonal H(q+1,q) = rec[2q+3]); this step's
        // column is h + s, read before the daxpy below adds s to it
        // (s_h: H(0:jm, 0:jm) staged in LDS by k_finalize<true> -- the same
        // values in the same order, without a global-memory latency per term)
        for (int i = t; i < jm; i += nt) {
            double ti = 0.0;
            for (int q = i > 0 ? i - 1 : 0; q < jm; ++q) {
                const double hc = s_h ? s_h[q * jm + i] : hcol[(int64_t)q * hld + i];
                double hiq;
                if (q == jm - 1) hiq = hc + s_sum[i];
                else if (i <= q) hiq = hc;
                else hiq = s_rec[2 * q + 3];
                ti = fma(hiq, s_sum[q], ti);
            }
            coef[3 * cstride + i] = ti;
        }
        __syncthreads();
    }
    if (take) {
        for (int k = t; k < jm; k += nt) {
            coef[take * cstride + k] = s_sum[k];
            if (hld) hcol[(int64_t)(j - 1) * hld + k] += s_sum[k];  // daxpy into h(1:j,j) (dnaitr.f:681)
        }
    }
}

// Single-block finalize.  The state is read once into LDS and written back
// once: the phase logic is one thread's chain of dependent accesses, which on
// the global copy (last written by another XCD's finalize) cost a memory
// latency each.
// The whole finalize, as the single workgroup of k_finalize runs it -- also
// run by workgroup 0 of the symmetric SpMV's combine kernel when a finalize is
// deferred into it (spmv_sym.hip; FinArgs).  Any block size; its loops stride
// by blockDim.x.  L: fin_lds_bytes(m + m2) of LDS; s_h (HS only): the Arnoldi
// fold's H(0:jm, 0:jm), kFoldHMax^2 doubles of LDS.
template <bool HS>
__device__ __forceinline__ void finalize_block(const FinArgs& a, FinLds* L, double* s_h) {
    if (threadIdx.x == 0) L->st = *a.st;
    if (a.phase == kFinPostCgsFold && 2 * (a.j + 1) <= kFoldRecMax)
        for (int k = threadIdx.x; k < 2 * (a.j + 1); k += blockDim.x) L->rec[k] = a.rec[k];
    if constexpr (HS) {
        const int jm = a.m - 1;
        for (int k = threadIdx.x; k < jm * jm; k += blockDim.x)
            s_h[k] = a.hcol[(int64_t)(k / jm) * a.hld + k % jm];
    }
    // the partials' loads go out with the state's: one memory latency, not two
    // (a closed gate discards the sums unwritten)
    fin_sums(a.part, a.nblk, a.from_sums, a.m, a.sums, a.part2, a.m2, L->sum);
    __syncthreads();
    if (gate_closed(&L->st, a.gate)) return;
    fin_body(a.m, a.phase, a.j, a.rstart, a.sums, a.coef, a.cstride, a.rec, &L->st, a.hcol, a.hld,
             a.m2, a.rstart_prev, L, HS ? s_h : nullptr);
    __syncthreads();
    if (threadIdx.x == 0) *a.st = L->st;
}

// The launch's dynamic LDS as the finalize's (k_finalize, the combine kernel);
// HS (Arnoldi kFinPostCgsFold, j <= kFoldHMax): H's first j columns and rows,
// read once in parallel (coalesced) for the t = H s loop; the 32 KB are static,
// so only that variant carries them.
template <bool HS>
__device__ __forceinline__ void finalize_block_dyn(const FinArgs& a) {
    extern __shared__ double fin_dyn[];
    __shared__ double s_h[HS ? kFoldHMax * kFoldHMax : 1];
    finalize_block<HS>(a, reinterpret_cast<FinLds*>(fin_dyn), s_h);
}

}  // namespace
}  // namespace ahip::dev
