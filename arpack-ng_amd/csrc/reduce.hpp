// Shared device helper of the single-block finalize kernels (kernels.hip
// k_finalize, zstep.hip k_zs_finalize): the fixed-order sum of one slot's
// per-block partials, 32 threads (half a wave) per slot.
#pragma once
#include <hip/hip_runtime.h>

#include "device.hpp"

namespace ahip::dev {

// Thread `sub` (0..31) of the slot's half wave: the sum of p[sub], p[sub+32],
// ... in four chains over b = sub + 128 i (+32, +64, +96), then the half wave
// reduces.  For the common grid (nblk = kMaxRedBlocks) all 32 loads of the
// thread are issued before the first add -- one memory latency instead of
// eight dependent rounds -- with the same association as the generic loop,
// so both give the same bits.
__device__ __forceinline__ double slot_partial(const double* __restrict__ p, int nblk, int sub) {
    double s = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if (nblk == kMaxRedBlocks) {
        double v[kMaxRedBlocks / 32];
#pragma unroll
        for (int q = 0; q < kMaxRedBlocks / 32; ++q) v[q] = p[sub + 32 * q];
#pragma unroll
        for (int q = 0; q < kMaxRedBlocks / 32; q += 4) {
            s += v[q];
            s1 += v[q + 1];
            s2 += v[q + 2];
            s3 += v[q + 3];
        }
    } else {
        int b = sub;
        for (; b + 96 < nblk; b += 128) {
            s += p[b];
            s1 += p[b + 32];
            s2 += p[b + 64];
            s3 += p[b + 96];
        }
        for (; b < nblk; b += 32) s += p[b];
    }
    return (s + s1) + (s2 + s3);
}

}  // namespace ahip::dev
