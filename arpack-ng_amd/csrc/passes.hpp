// Device helpers shared by the n-length pass kernels (kernels.hip: dots,
// update, V*Q; fold.hip: the folded Lanczos step): the V-load policy, wave /
// block reductions into the k-major partials, the profiler scope of a
// launcher and the compile-time column-count dispatch.
#pragma once
#include <hip/hip_runtime.h>

#include "device.hpp"

namespace ahip::dev {
namespace {

// Loads of the Krylov basis V in the Gram-Schmidt and V*Q passes.  Policy POL:
//   kPolNt / kPolNtRev  non-temporal, sweeping rows first-to-last / last-to-first:
//            a basis of several hundred MB or more is streamed from HBM; the NT
//            hint keeps the 1-2.4 GB sweep from evicting the n-vectors every pass
//            re-reads (w, r) from the caches (+3.2% cycle rate at n = 1e7), and
//            alternating directions start each pass on rows the previous one left
//            in the 256 MB Infinity Cache;
//   kPolPlain  plain loads: a basis that fits the Infinity Cache (<= ~400 MB)
//            is re-read from it by the next pass (same-box A/B: +7% cycle rate at
//            n = 1e6, +4% at 1.25e6 rows, -2.7% at 2.5e6 and 1e7 -- hence the
//            size rule in ws_create, AHIP_V_POLICY=nt|plain to override).
enum VPol : int { kPolNt = 0, kPolNtRev = 1, kPolPlain = 2 };
template <int POL, class T>
__device__ __forceinline__ T vld(const T* p) {
    if constexpr (POL == kPolPlain) return *p;
    else return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Reduce CH per-thread accumulators over the block and write them (plus an
// optional extra value) as this block's partial row.
template <int CH>
__device__ __forceinline__ void block_partials(double (&acc)[CH], int jc, double extra,
                                               bool with_extra, double* part, int col0,
                                               int extra_slot) {
    // k-major layout part[slot * nblk + block]: the finalize reads each slot
    // as one contiguous (coalesced) run
    __shared__ double red[kBlock / 64][CH + 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        if (k < jc) {
            const double s = wave_sum(acc[k]);
            if (lane == 0) red[wave][k] = s;
        }
    }
    if (with_extra) {
        const double s = wave_sum(extra);
        if (lane == 0) red[wave][CH] = s;
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < jc) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][t];
        part[(size_t)(col0 + t) * gridDim.x + blockIdx.x] = s;
    }
    if (with_extra && t == kBlock - 1) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][CH];
        part[(size_t)extra_slot * gridDim.x + blockIdx.x] = s;
    }
}

__device__ __forceinline__ bool gate_closed(const LzState* st, int gate) {
    if (st->abort) return true;
    return gate >= 0 && st->dgks != gate;
}

}  // namespace

namespace {
struct ProfScope {  // kernel-mode span (prof_arm) around one launcher when profiling is on
    ProfClass c;
    hipStream_t s;
    double bytes;
    ProfScope(ProfClass cc, hipStream_t ss, double b) : c(cc), s(ss), bytes(b) { prof_arm(c, s); }
    ~ProfScope() { prof_disarm(c, bytes); }
};
}  // namespace


}  // namespace ahip::dev

#define AHIP_CASES_1_32(M) \
    M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15) M(16) \
    M(17) M(18) M(19) M(20) M(21) M(22) M(23) M(24) M(25) M(26) M(27) M(28) M(29) M(30) M(31) M(32)
#define AHIP_CASES_33_64(M) \
    M(33) M(34) M(35) M(36) M(37) M(38) M(39) M(40) M(41) M(42) M(43) M(44) M(45) M(46) M(47) M(48) \
    M(49) M(50) M(51) M(52) M(53) M(54) M(55) M(56) M(57) M(58) M(59) M(60) M(61) M(62) M(63) M(64)

