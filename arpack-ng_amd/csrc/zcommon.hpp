// Complex helpers shared by the complex kernels (zkernels.hip, zstep.hip):
// interleaved (re, im) storage of complex128 (z*) / complex64 (c*) elements,
// complex128 arithmetic.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace ahip::zdev {
namespace zc {
constexpr int kB = 256;

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {  // conj(a) * b
    return make_double2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}

// storage of one complex element: double2 (complex128, z*) or float2
// (complex64, c*); arithmetic is always complex128
template <class R>
struct C2;
template <>
struct C2<double> {
    using T = double2;
};
template <>
struct C2<float> {
    using T = float2;
};
__device__ __forceinline__ double2 d2(double2 v) { return v; }
__device__ __forceinline__ double2 d2(float2 v) { return make_double2(v.x, v.y); }
template <class R>
__device__ __forceinline__ typename C2<R>::T st2(double2 v) {
    if constexpr (std::is_same_v<R, double>) return v;
    else return make_float2((float)v.x, (float)v.y);
}

// non-temporal load of one stored complex element (the basis sweeps)
typedef double zc_dv2 __attribute__((ext_vector_type(2)));
typedef float zc_fv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ntld(const double2* p) {
    const zc_dv2 v = __builtin_nontemporal_load(reinterpret_cast<const zc_dv2*>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ double2 ntld(const float2* p) {
    const zc_fv2 v = __builtin_nontemporal_load(reinterpret_cast<const zc_fv2*>(p));
    return make_double2(v.x, v.y);
}

// The split operator's S slice partials of row r (slice-major, n apart; S = 2,
// 4 or 8) summed in one fixed tree order: the split SpMV's combine (zsplit.hip)
// and the solver kernels that fuse it (zsolve.hip) produce bit-identical sums
constexpr int kZMaxSlices = 8;  // = XCDs
template <int S>
__device__ __forceinline__ double2 slice_sum(const double2* __restrict__ yp, int64_t n, int64_t r) {
    static_assert(S == 2 || S == 4 || S == 8, "2, 4 or 8 column slices");
    double2 a[S];
#pragma unroll
    for (int s = 0; s < S; ++s) a[s] = yp[(int64_t)s * n + r];
    if constexpr (S == 2)
        return make_double2(a[0].x + a[1].x, a[0].y + a[1].y);
    else if constexpr (S == 4)
        return make_double2((a[0].x + a[1].x) + (a[2].x + a[3].x), (a[0].y + a[1].y) + (a[2].y + a[3].y));
    else
        return make_double2(((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x)),
                            ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y)));
}

}  // namespace zc
}  // namespace ahip::zdev
