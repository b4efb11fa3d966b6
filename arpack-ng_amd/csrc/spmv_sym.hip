// Symmetric-storage SpMV y = A x for dsaupd's OP (A = A', declared by the
// caller through arpack_hip_csr_set_symmetric; MKL's SPARSE_MATRIX_TYPE_SYMMETRIC
// with the upper fill mode is the same contract).  Only the upper triangle
// (col >= row, diagonal included) is streamed from HBM: at the north-star
// operator that halves the val/col bytes of the dominant kernel of the cycle
// (SpMV ~50% of the cycle's bytes).
//
// y_i = sum_{j >= i} a_ij x_j  (row part, lane registers)
//     + sum_{k <  i} a_ki x_k  (transposed part: scattered from row k)
//
// Layout: SYMMETRIC SUPERBLOCKS.  Superblock b owns rows [r0, r1); the upper
// entries of those rows touch columns [r0, r0 + span) with span <= kSymWin (10240).
// A 1024-thread workgroup (one per CU; it walks a chain of consecutive
// superblocks, see k_csr_ssell) stages x[r0, r0+span) in LDS, zeroes an LDS y
// window of the same range, and streams the superblock's
// upper entries as SELL-64 slices (rows sorted by upper length, one row per
// lane, column-step-major: one 512-B val load + one 128-B 16-bit column load
// per wave and step).  Each entry feeds the row sum (x gathered from LDS) and,
// off the diagonal, one LDS atomic add a_ij x_i into y_lds[j].
// The y window then holds three ranges:
//   [0, pre)     rows that the previous superblock's window also reaches
//                (its spill): written to slot_hi, combined below
//   [pre, R)     complete rows: stored to y
//   [R, span)    this superblock's spill into the next one: slot_lo
// The analysis guarantees every spill lies inside the NEXT superblock's rows,
// so each combined row has exactly two partial sums; inside a chain the spill
// simply stays in LDS, and at chain heads a second small kernel stores
// y = lo + hi (a two-term sum is commutative, so the combine adds no order
// dependence of its own).
//
// Rounding: the transposed contributions arrive in LDS in wave-schedule order,
// so y is not bitwise reproducible run to run (|dy| ~ 1 ulp of the row's
// terms).  The full-storage kernel (spmv.hip, bitwise SciPy's csr_matvec) stays
// the default; this one is opt-in for operators the caller declares symmetric.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <type_traits>
#include <cstring>
#include <cstdint>
#include <vector>

#include "device.hpp"
#include "finalize.hpp"

namespace ahip::dev {

namespace {

constexpr int kSymThreads = 1024;
constexpr int kSymWin = 10240;  // doubles per LDS window (x and y: 2 x 80 KB = all 160 KB)

// Per row: the count of upper entries (diagonal included; bit 30 flags a
// column left of the block) and the largest column; over the matrix: the
// largest |a_ij| above the diagonal (as the bits of a non-negative double,
// which order like the unsigned integers).  Per column j (local, spill columns
// [n, n + spill_out) included): the strictly-upper entries (i < j) whose
// transposed terms the fixed-point form sums into word j -- its overflow
// headroom is the largest of these counts, whatever the pattern's symmetry.
__global__ void k_upper_stats(int64_t n, int64_t coff, const int64_t* __restrict__ rp,
                              const int32_t* __restrict__ col, const double* __restrict__ val,
                              int32_t* __restrict__ cnt, int32_t* __restrict__ cmax,
                              unsigned long long* __restrict__ amax, int32_t* __restrict__ ccol) {
    // amax[0]: the largest |a_ij| above the diagonal; amax[1]: the smallest
    // nonzero one (both as the bits of non-negative doubles)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    double am = 0.0, an = DBL_MAX;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int32_t c = 0, m = (int32_t)i, low = 0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            const int32_t j = (int32_t)(col[k] - coff);
            if (j >= i) {
                ++c;
                m = max(m, j);
                if (j > i) {
                    const double a = fabs(val[k]);
                    am = fmax(am, a);
                    if (a > 0.0) an = fmin(an, a);
                    atomicAdd(&ccol[j], 1);
                }
            }
            low |= j < 0;  // a column of the previous rank's block (halo_lo)
        }
        cnt[i] = c | (low << 30);
        cmax[i] = m;
    }
    for (int o = 32; o > 0; o >>= 1) {
        am = fmax(am, __shfl_xor(am, o, 64));
        an = fmin(an, __shfl_xor(an, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(amax, (unsigned long long)__double_as_longlong(am));
        atomicMin(amax + 1, (unsigned long long)__double_as_longlong(an));
    }
}

// one 64-thread block per slice, lane = row: the row's upper entries in CSR
// order; padding steps carry value 0 and the row's own (diagonal) column, so
// the kernel's off-diagonal test drops them without a length check
__global__ void k_symsell_fill(int64_t coff, const int64_t* __restrict__ sptr,
                               const int32_t* __restrict__ srow,
                               const int64_t* __restrict__ slice_r0, const int64_t* __restrict__ rp,
                               const int32_t* __restrict__ col, const double* __restrict__ val,
                               uint16_t* __restrict__ scolw, double* __restrict__ sval) {
    const int64_t s = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t base = sptr[s];
    const int w = (int)((sptr[s + 1] - base) >> 6);
    const int row = srow[s * 64 + lane];
    const int64_t r0 = slice_r0[s];
    const uint16_t pad = row >= 0 ? (uint16_t)(row - r0) : (uint16_t)0;
    int k = 0;
    if (row >= 0) {
        for (int64_t e = rp[row]; e < rp[row + 1]; ++e) {
            const int32_t j = (int32_t)(col[e] - coff);
            if (j < row) continue;
            sval[base + (int64_t)k * 64 + lane] = val[e];
            scolw[base + (int64_t)k * 64 + lane] = (uint16_t)(j - r0);
            ++k;
        }
    }
    for (; k < w; ++k) {
        sval[base + (int64_t)k * 64 + lane] = 0.0;
        scolw[base + (int64_t)k * 64 + lane] = pad;
    }
}

template <class T, bool NT>
__device__ __forceinline__ T ldg(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// One workgroup walks a CHAIN of `chain` consecutive superblocks (grid = the
// CU count, one resident workgroup per CU: the windows take all 160 KB of
// LDS).  A superblock's spill is the next one's window head, so inside a chain
// it stays in LDS: the x and y windows shift down by R and only the new x
// columns are loaded.  Only a chain's first superblock has head rows combined
// with another workgroup's (or rank's) spill through the slots, and only its
// last superblock's spill leaves through a slot.  Each wave streams its slices
// with the next slice's first chunk in flight, across superblock boundaries.
//
// ONE walk, two accumulators (DET):
//  * DET = false (default): the transposed terms a_ij x_i meet as LDS fp64
//    atomic adds in the y window, in wave-schedule order -- not bitwise
//    reproducible run to run (~1 ulp of the row's terms);
//  * DET = true (deterministic mode, arpack_hip_set_deterministic): they become
//    64-bit FIXED-POINT integers, and integer addition is exact, so their sum
//    is the same in any order:
//      q = rint(a_ij x_i 2^(B-E))      (one fma onto 1.5 * 2^52: the low mantissa
//                                       bits of the result are q, |q| < 2^B <= 2^51)
//      y_j = (row sum) + (double)(sum of the q) * 2^(E-B)
//    with 2^E >= amax * (largest |x| the chain has staged so far): a running
//    maximum, so E only grows, and a partial sum carried into the next window
//    is rescaled by an arithmetic shift when it does; B = min(51, 62 - bits(L))
//    for columns that receive at most L transposed terms, so no sum can
//    overflow.  Each term is rounded to 2^(E-B) -- at most 2^-51 of the
//    window's largest product.  The row sums (one lane's sequential sum, as in
//    the default) wait in registers (at most MAXQ slices a wave) until the
//    window's x is spent, then meet the integer sums in the x window.  One LDS
//    word past every window (span <= kSymWin - 1) holds the running maximum.
// Everything else -- chunk pipeline, window carry, slots, the chain-head
// hand-off and the carried finalize -- is the same code for both.
//
// FUSE (one GPU; AHIP_SPMV_FUSE=0 turns it off): the chain-head combine
// y = lo + hi happens here instead of in k_ssell_combine.  Each chain's head
// rows pair two workgroups (the previous chain's, whose last spill is lo, and
// this chain's, whose first superblock's head rows are hi); both publish their
// part and add to the pair's counter; the one whose add returns 1 arrived
// second and combines.  No workgroup ever waits on another.  Two orderings
// (handoff_store / handoff_arrive / handoff_load below):
//  * FUSE = 1 (measured form, MI355X_MICROARCH.md's hand-off row for one
//    workgroup a CU): agent-scope (sc1) slot stores drained by a vmcnt(0)
//    wait, a relaxed counter add, agent-scope (sc1) slot loads;
//  * FUSE = 2 (the memory model's form): plain slot stores, the workgroup
//    barrier, ONE acq_rel agent-scope counter add (release: the barrier-ordered
//    stores of every wave; acquire: the partner's), the barrier, plain loads --
//    the idiom of a grid barrier.  AHIP_HANDOFF=2 selects it (A/B).
// The deferred finalize of the step (fa, kernels.hip) then runs in workgroup 0
// over its spent x window.
template <int FUSE>
__device__ __forceinline__ void handoff_store(double* p, double v) {
    if constexpr (FUSE == 1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
template <int FUSE>
__device__ __forceinline__ double handoff_load(const double* p) {
    if constexpr (FUSE == 1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <int FUSE>
__device__ __forceinline__ int handoff_arrive(int* p) {
    if constexpr (FUSE == 1) return __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_fetch_add(p, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
}

template <int U, bool NT, bool YNT = false, int FUSE = 0, bool DET = false, int MAXQ = 1>
__global__ __launch_bounds__(kSymThreads) void k_csr_ssell(
    const int64_t* __restrict__ sb_r0, const int32_t* __restrict__ sb_span,
    const int32_t* __restrict__ sb_pre, const int64_t* __restrict__ sb_off,
    const int64_t* __restrict__ sb_slice0, const int64_t* __restrict__ sptr,
    const int32_t* __restrict__ srow, const uint16_t* __restrict__ scolw,
    const double* __restrict__ sval, const double* __restrict__ x, double* __restrict__ y,
    double* __restrict__ slot_lo, double* __restrict__ slot_hi, int64_t coff, int chain,
    int64_t nsb, int* __restrict__ pair, FinArgs fa, double amax, int bits) {
    // the y window: fp64 sums, or (DET) two's-complement fixed-point sums
    using Word = std::conditional_t<DET, unsigned long long, double>;
    __shared__ double xw[kSymWin];
    __shared__ Word yw[kSymWin];
    constexpr int NW = kSymThreads / 64;
    constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t ch = xcd_block(blockIdx.x, gridDim.x);
    const int64_t b0 = ch * chain, b1 = min(b0 + (int64_t)chain, nsb);
    struct Chunk {
        double v[U];
        int c[U];
    };
    auto load = [&](Chunk& c, int64_t base, int w, int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k0 + u < w;
            c.v[u] = in ? ldg<double, NT>(sval + base + (int64_t)(k0 + u) * 64 + lane) : 0.0;
            c.c[u] = in ? (int)ldg<uint16_t, NT>(scolw + base + (int64_t)(k0 + u) * 64 + lane) : -1;
        }
    };
    auto geom = [&](int64_t sl, int64_t& base, int& w) {
        base = sptr[sl];
        w = (int)((sptr[sl + 1] - base) >> 6);
    };
    Chunk cur, nxt;
    int64_t cur_s = -1;  // slice whose first chunk is in `cur`
    {
        const int64_t s = sb_slice0[b0] + wave;
        if (s < sb_slice0[b0 + 1]) {
            int64_t base;
            int w;
            geom(s, base, w);
            load(cur, base, w, 0);
            cur_s = s;
        }
    }
    // DET: the fixed-point scale 2^(B-E) (inv) and its inverse (sc)
    [[maybe_unused]] unsigned long long* xmax = nullptr;  // bits of the running max |x|
    [[maybe_unused]] int ea = 0, E = INT_MIN;
    [[maybe_unused]] double inv = 1.0, sc = 0.0;
    if constexpr (DET) {
        xmax = reinterpret_cast<unsigned long long*>(&yw[kSymWin - 1]);
        (void)frexp(amax, &ea);  // amax < 2^ea
        if (t == 0) *xmax = 0ull;
        __syncthreads();  // before any wave's first atomicMax (LDS holds the last launch's words)
    }
    int R_prev = 0, span_prev = 0;
    for (int64_t b = b0; b < b1; ++b) {
        const int64_t r0 = sb_r0[b];
        const int R = (int)(sb_r0[b + 1] - r0);
        const int span = sb_span[b];
        const int64_t s1 = sb_slice0[b + 1];
        int carry = 0;
        if (b > b0) {  // the previous window's tail [R_prev, span_prev) becomes this head
            // (span <= 2R inside chains, so source and destination do not overlap)
            carry = span_prev - R_prev;
            __syncthreads();  // every wave has read its epilogue values
            for (int i = t; i < carry; i += kSymThreads) {
                xw[i] = xw[R_prev + i];
                yw[i] = yw[R_prev + i];
            }
            __syncthreads();  // the staging below overwrites the shift's source range
        }
        if constexpr (!DET) {
            for (int i = carry + t; i < span; i += kSymThreads) {
                xw[i] = x[coff + r0 + i];
                yw[i] = 0.0;
            }
            __syncthreads();
        } else {
            // stage the new columns; the max over their |x| (as bit patterns, so a
            // NaN wins and reaches every output of the chain) joins the running max
            unsigned long long mb = 0;
            for (int i = carry + t; i < span; i += kSymThreads) {
                const double v = x[coff + r0 + i];
                xw[i] = v;
                yw[i] = 0;
                mb = max(mb, (unsigned long long)__double_as_longlong(fabs(v)));
            }
            for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned long long)__shfl_xor(mb, o, 64));
            if (lane == 0) atomicMax(xmax, mb);
            __syncthreads();
            const double X = __longlong_as_double((long long)*xmax);
            int ex = 0;
            (void)frexp(X, &ex);  // X < 2^ex
            // (floor: 2^(B-E) <= 2^1000; with 2^-900 <= amax <= 2^900, the
            // plan's condition, x_i 2^(B-E) then stays finite and every |q| < 2^B)
            const int En = max(ea + ex, bits - 1000);
            if (En > E) {  // uniform: X came from LDS after the barrier
                if (carry > 0) {  // the carried sums were scaled by 2^(B-E): rescale
                    const int d = min(En - E, 63);
                    for (int i = t; i < carry; i += kSymThreads)
                        yw[i] = (unsigned long long)((long long)yw[i] >> d);
                    __syncthreads();
                }
                E = En;
                inv = ldexp(1.0, bits - E);
                sc = ldexp(1.0, E - bits);
            }
            if (!(X <= DBL_MAX)) sc = __longlong_as_double(0x7ff8000000000000ll);  // NaN / inf in x
        }
        [[maybe_unused]] double accq[MAXQ];
        [[maybe_unused]] uint32_t rlq[(MAXQ + 1) / 2];  // window rows, two 16-bit halves (0xffff: padding)
        int nq = 0;
        for (int64_t s = sb_slice0[b] + wave; s < s1; s += NW, ++nq) {
            int64_t base;
            int w;
            geom(s, base, w);
            if (cur_s != s) load(cur, base, w, 0);
            const int row = srow[s * 64 + lane];
            const int rl = row >= 0 ? row - (int)r0 : 0;
            const double xi = DET ? xw[rl] * inv : xw[rl];  // (DET: exact, a power-of-two scale)
            // this wave's next slice: in this superblock, else its first in the next one
            int64_t sn = s + NW;
            if (sn >= s1) sn = b + 1 < b1 ? sb_slice0[b + 1] + wave : -1;
            if (sn >= 0 && b + 1 < b1 && sn >= s1 && sn >= sb_slice0[b + 2]) sn = -1;
            int64_t nbase = 0;
            int nw = 0;
            if (sn >= 0) geom(sn, nbase, nw);
            double acc = 0.0;
            int k = 0;
            do {
                if (k + U < w) load(nxt, base, w, k + U);
                else if (sn >= 0) load(nxt, nbase, nw, 0);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int c = cur.c[u];
                    if (c >= 0) {
                        acc += cur.v[u] * xw[c];
                        if (c != rl) {
                            if constexpr (DET) {
                                const double f = fma(cur.v[u], xi, kMagic);
                                atomicAdd(&yw[c], (unsigned long long)__double_as_longlong(f) -
                                                      (unsigned long long)__double_as_longlong(kMagic));
                            } else {
                                atomicAdd(&yw[c], cur.v[u] * xi);
                            }
                        }
                    }
                }
                cur = nxt;
                k += U;
            } while (k < w);
            cur_s = sn;
            if constexpr (DET) {
                const uint32_t h = row >= 0 ? (uint32_t)rl : 0xffffu;
#pragma unroll
                for (int u = 0; u < MAXQ; ++u)
                    if (u == nq) {
                        accq[u] = acc;
                        if (u & 1) rlq[u >> 1] = (rlq[u >> 1] & 0xffffu) | (h << 16);
                        else rlq[u >> 1] = h;
                    }
            } else {
                if (row >= 0) atomicAdd(&yw[rl], acc);
            }
        }
        __syncthreads();  // (DET: x of the window spent, every integer sum complete)
        if constexpr (DET) {
#pragma unroll
            for (int u = 0; u < MAXQ; ++u) {
                const uint32_t h = (u & 1) ? rlq[u >> 1] >> 16 : rlq[u >> 1] & 0xffffu;
                if (u < nq && h != 0xffffu) xw[h] = accq[u];
            }
            __syncthreads();
        }
        // the window's word i as y: the row sum (+ the transposed terms)
        auto yrow = [&](int i) {
            if constexpr (DET) return xw[i] + (double)(long long)yw[i] * sc;
            else return yw[i];
        };
        auto yspill = [&](int i) {
            if constexpr (DET) return (double)(long long)yw[i] * sc;
            else return yw[i];
        };
        // head rows meet another chain's spill through the slots; the rest are final
        const int head = b == b0 ? sb_pre[b] : 0;
        const int64_t off = sb_off[b];
        for (int i = t; i < R; i += kSymThreads) {
            const double v = yrow(i);
            if (i < head) {
                handoff_store<FUSE>(slot_hi + off + i, v);
            } else if constexpr (YNT) {
                __builtin_nontemporal_store(v, y + r0 + i);
            } else {
                y[r0 + i] = v;
            }
        }
        if (b == b1 - 1) {  // the chain's last spill leaves through a slot
            const int64_t offn = sb_off[b + 1];
            for (int i = R + t; i < span; i += kSymThreads)
                handoff_store<FUSE>(slot_lo + offn + (i - R), yspill(i));
        }
        R_prev = R;
        span_prev = span;
    }
    if constexpr (FUSE != 0) {
        const int64_t nch = gridDim.x;
        int* flag = reinterpret_cast<int*>(xw);  // the x window is spent
        if constexpr (FUSE == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's slot stores
        __syncthreads();
        if (t == 0) {
            flag[0] = ch > 0 ? handoff_arrive<FUSE>(pair + ch) : 0;
            flag[1] = ch + 1 < nch ? handoff_arrive<FUSE>(pair + ch + 1) : 0;
        }
        // FUSE = 1 (the measured sc1 hand-off for one workgroup per CU, this
        // kernel's occupancy): every slot store above is an agent-scope (sc1)
        // store drained by the vmcnt(0) wait before the barrier, ONE lane adds
        // to the pair's unsharded counter, and the second arriver -- told by the
        // value its add returned -- reads both slots with agent-scope (sc1)
        // loads after the barrier below.  The barriers also keep the compiler
        // from moving the slot accesses across the counter (they are workgroup
        // fences).  FUSE = 2: the counter add is acq_rel at agent scope.  The
        // word-by-word check under uneven load is tests/test_gpu_symspmv_handoff.py.
        __syncthreads();
        for (int side = 0; side < 2; ++side) {
            if (flag[side] != 1) continue;  // first of its pair: the partner combines
            const int64_t c = ch + side;     // the chain whose head rows are combined
            const int64_t bh = c * chain;
            const int pre = sb_pre[bh];
            const int64_t off = sb_off[bh], rh = sb_r0[bh];
            for (int i = t; i < pre; i += kSymThreads)
                y[rh + i] = handoff_load<FUSE>(slot_lo + off + i) + handoff_load<FUSE>(slot_hi + off + i);
            if (t == 0) pair[c] = 0;  // both parties are done with it (next launch: kernel order)
        }
        if (fa.active && blockIdx.x == 0) {
            __syncthreads();  // flag[] read by every wave before the window is reused
            finalize_block<false>(fa, reinterpret_cast<FinLds*>(xw), nullptr);
        }
    }
}

// The same chained walk with the superblock's work cut evenly over its waves.
// Above, wave q takes slices q, q + 16, ...: a superblock of ~77 slices gives 13
// waves five slices and three waves four, and every wave then idles at the
// barrier until the five-slice waves finish.  Here the superblock's slices are
// flattened into their column steps (sptr / 64: a slice of width w is w steps)
// and wave q takes the contiguous steps [wg0[b*16+q], wg0[b*16+q+1]) -- equal
// counts to within one step, and one contiguous val / col stream per wave.  A
// range may start or end inside a slice, so a row can receive its upper-row
// sum from two waves (both LDS atomic adds, like the transposed terms).
template <int U, bool NT>
__global__ __launch_bounds__(kSymThreads) void k_csr_ssell_bal(
    const int64_t* __restrict__ sb_r0, const int32_t* __restrict__ sb_span,
    const int32_t* __restrict__ sb_pre, const int64_t* __restrict__ sb_off,
    const int64_t* __restrict__ wg0, const int32_t* __restrict__ wsl,
    const int64_t* __restrict__ sptr, const int32_t* __restrict__ srow,
    const uint16_t* __restrict__ scolw, const double* __restrict__ sval,
    const double* __restrict__ x, double* __restrict__ y, double* __restrict__ slot_lo,
    double* __restrict__ slot_hi, int64_t coff, int chain, int64_t nsb) {
    __shared__ double xw[kSymWin];
    __shared__ double yw[kSymWin];
    constexpr int NW = kSymThreads / 64;
    // wave-uniform: the unit bookkeeping below lives in scalar registers
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t ch = xcd_block(blockIdx.x, gridDim.x);
    const int64_t b0 = ch * chain, b1 = min(b0 + (int64_t)chain, nsb);
    struct Chunk {
        double v[U];
        int c[U];
    };
    // a unit: steps [k, khi) of slice s (element offset base); khi < 0 = none
    struct Unit {
        int64_t s, base, g1;
        int k, khi;
    };
    auto load = [&](Chunk& c, int64_t base, int khi, int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k0 + u < khi;
            c.v[u] = in ? ldg<double, NT>(sval + base + (int64_t)(k0 + u) * 64 + lane) : 0.0;
            c.c[u] = in ? (int)ldg<uint16_t, NT>(scolw + base + (int64_t)(k0 + u) * 64 + lane) : -1;
        }
    };
    auto first = [&](int64_t b, Unit& q) {  // this wave's first unit in superblock b
        const int64_t g0 = wg0[b * NW + wave];
        q.g1 = wg0[b * NW + wave + 1];
        q.s = wsl[b * NW + wave];
        q.base = sptr[q.s];
        const int64_t st = q.base >> 6, w = (sptr[q.s + 1] - q.base) >> 6;
        q.k = (int)(g0 - st);
        q.khi = g0 < q.g1 ? (int)min(w, q.g1 - st) : -1;
    };
    auto advance = [&](const Unit& q, Unit& nq) {  // the next slice of the same range
        if ((q.base >> 6) + q.khi >= q.g1) return false;
        nq.s = q.s + 1;
        nq.g1 = q.g1;
        nq.base = sptr[nq.s];
        const int64_t w = (sptr[nq.s + 1] - nq.base) >> 6;
        nq.k = 0;
        nq.khi = (int)min(w, q.g1 - (nq.base >> 6));
        return true;
    };
    Chunk cur, nxt;
    Unit u;
    first(b0, u);
    if (u.khi >= 0) load(cur, u.base, u.khi, u.k);
    int R_prev = 0, span_prev = 0;
    for (int64_t b = b0; b < b1; ++b) {
        const int64_t r0 = sb_r0[b];
        const int R = (int)(sb_r0[b + 1] - r0);
        const int span = sb_span[b];
        int carry = 0;
        if (b > b0) {  // the previous window's tail [R_prev, span_prev) becomes this head
            carry = span_prev - R_prev;
            __syncthreads();
            for (int i = t; i < carry; i += kSymThreads) {
                xw[i] = xw[R_prev + i];
                yw[i] = yw[R_prev + i];
            }
            __syncthreads();
        }
        for (int i = carry + t; i < span; i += kSymThreads) {
            xw[i] = x[coff + r0 + i];
            yw[i] = 0.0;
        }
        __syncthreads();
        // `u` (first chunk in `cur`) is this wave's first unit of superblock b
        if (u.khi >= 0) {
            bool more;
            do {
                const int row = srow[u.s * 64 + lane];
                const int rl = row >= 0 ? row - (int)r0 : 0;
                const double xi = xw[rl];
                Unit nu;
                more = advance(u, nu);
                if (!more) {
                    if (b + 1 < b1) first(b + 1, nu);
                    else nu.khi = -1;
                }
                double acc = 0.0;
                int k = u.k;
                do {
                    if (k + U < u.khi) load(nxt, u.base, u.khi, k + U);
                    else if (nu.khi >= 0) load(nxt, nu.base, nu.khi, nu.k);
#pragma unroll
                    for (int q = 0; q < U; ++q) {
                        const int c = cur.c[q];
                        if (c >= 0) {
                            acc += cur.v[q] * xw[c];
                            if (c != rl) atomicAdd(&yw[c], cur.v[q] * xi);
                        }
                    }
                    cur = nxt;
                    k += U;
                } while (k < u.khi);
                if (row >= 0) atomicAdd(&yw[rl], acc);
                u = nu;
            } while (more);
        } else if (b + 1 < b1) {  // empty range here: set up the next superblock's
            first(b + 1, u);
            if (u.khi >= 0) load(cur, u.base, u.khi, u.k);
        }
        __syncthreads();
        const int head = b == b0 ? sb_pre[b] : 0;
        const int64_t off = sb_off[b];
        for (int i = t; i < R; i += kSymThreads) {
            const double v = yw[i];
            if (i < head) slot_hi[off + i] = v;
            else y[r0 + i] = v;
        }
        if (b == b1 - 1) {
            const int64_t offn = sb_off[b + 1];
            for (int i = R + t; i < span; i += kSymThreads) slot_lo[offn + (i - R)] = yw[i];
        }
        R_prev = R;
        span_prev = span;
    }
}

// y(head rows of each chain's first superblock) = lo + hi (1024 threads: a
// head is ~4k rows, so every load of the block is in flight at once)
__global__ __launch_bounds__(1024) void k_ssell_combine(const int64_t* __restrict__ sb_r0,
                                                       const int32_t* __restrict__ sb_pre,
                                                       const int64_t* __restrict__ sb_off,
                                                       const double* __restrict__ lo,
                                                       const double* __restrict__ hi,
                                                       double* __restrict__ y, int chain) {
    const int64_t b = (int64_t)blockIdx.x * chain;
    const int pre = sb_pre[b];
    const int64_t off = sb_off[b], r0 = sb_r0[b];
    for (int i = threadIdx.x; i < pre; i += 1024) y[r0 + i] = lo[off + i] + hi[off + i];
}

// The same combine carrying a deferred finalize of the Lanczos step
// (kernels.hip finalize(..., defer)): workgroup 0 runs it after its rows.  It
// reads the partial sums of the pass before the SpMV and writes the step
// state the pass after it reads -- both across kernel boundaries -- and
// touches nothing of the SpMV, so the launch it saves (~6 us of a 60-500 us
// SpMV) costs no ordering.
template <bool HS>
__global__ __launch_bounds__(1024) void k_ssell_combine_fin(const int64_t* __restrict__ sb_r0,
                                                           const int32_t* __restrict__ sb_pre,
                                                           const int64_t* __restrict__ sb_off,
                                                           const double* __restrict__ lo,
                                                           const double* __restrict__ hi,
                                                           double* __restrict__ y, int chain,
                                                           FinArgs fa) {
    const int64_t b = (int64_t)blockIdx.x * chain;
    const int pre = sb_pre[b];
    const int64_t off = sb_off[b], r0 = sb_r0[b];
    for (int i = threadIdx.x; i < pre; i += 1024) y[r0 + i] = lo[off + i] + hi[off + i];
    if (blockIdx.x == 0) finalize_block_dyn<HS>(fa);
}

// Spill-free distributed combine (Csr::ss_lg): the rank's first pre[0] rows
// take their lower ghost terms (columns in the low halo, x_ext[0, coff)) from
// their own full CSR rows instead of the previous rank's spill -- the same
// products, since A is symmetric, with x from the two-sided halo.  Workgroups
// [0, nch) combine chains 1.. as above (workgroup 0 carries a deferred
// finalize); workgroups nch.. take 256 head rows each, four lanes a row, the
// lanes' partials summed in lane order.
template <bool HS>
__global__ __launch_bounds__(1024) void k_ssell_combine_lg(
    const int64_t* __restrict__ sb_r0, const int32_t* __restrict__ sb_pre,
    const int64_t* __restrict__ sb_off, const double* __restrict__ lo, const double* __restrict__ hi,
    double* __restrict__ y, int chain, int nch, const int64_t* __restrict__ rp,
    const int32_t* __restrict__ col, const double* __restrict__ val, const double* __restrict__ xe,
    int64_t coff, FinArgs fa) {
    if ((int)blockIdx.x < nch) {
        if (blockIdx.x > 0) {
            const int64_t b = (int64_t)blockIdx.x * chain;
            const int pre = sb_pre[b];
            const int64_t off = sb_off[b], r0 = sb_r0[b];
            for (int i = threadIdx.x; i < pre; i += 1024) y[r0 + i] = lo[off + i] + hi[off + i];
        } else if (fa.active) {
            finalize_block_dyn<HS>(fa);
        }
        return;
    }
    const int64_t i = (int64_t)(blockIdx.x - nch) * 256 + (threadIdx.x >> 2);
    const int q = threadIdx.x & 3;
    const int pre = sb_pre[0];
    double s = 0.0;
    if (i < pre) {
        for (int64_t k = rp[i] + q; k < rp[i + 1]; k += 4) {
            const int64_t c = col[k];
            if (c < coff) s += val[k] * xe[c];
        }
    }
    const double s1 = __shfl_down(s, 1, 4);
    const double s2 = __shfl_down(s, 2, 4);
    const double s3 = __shfl_down(s, 3, 4);
    if (i < pre && q == 0) y[i] = hi[sb_off[0] + i] + (((s + s1) + s2) + s3);
}

}  // namespace

// Superblock plan from the per-row largest upper column cmax[i] (>= i).
// Superblock b owns rows [r0s[b], r0s[b+1]); its window [r0, r0 + spans[b])
// covers every upper column of its rows (<= win columns); pre[b] = leading rows
// reached by superblock b-1's window (its spill), which must lie inside b, so
// every row has at most two partial sums; pre[0] = spill_in (the previous
// rank's spill); the last window may reach spill_out rows past the block.
// off = prefix sums of pre (the combine slots).
//
// Balanced first: with the largest reach m = max(cmax[i] - i), any block of
// <= win - m rows fits a window, and blocks of >= m rows hold the previous
// block's spill, so k equal blocks work whenever n/k lies in [m, win - m].
// k is rounded up to a multiple of kQuantum (the CU count: whole rounds of
// one workgroup per CU, no tail) when the rows allow.  Otherwise greedy
// blocks (widest windows), which suit the end of a matrix where reaches
// shrink.  -1 if neither satisfies the rules.
static bool plan_check(int64_t n, const int32_t* cmax, int win, std::vector<int64_t>& r0s,
                       std::vector<int32_t>& spans, std::vector<int32_t>& pre,
                       std::vector<int64_t>& off, int64_t spill_in, int64_t spill_out) {
    const int64_t nsb = (int64_t)r0s.size() - 1;
    spans.assign(nsb, 0);
    for (int64_t b = 0; b < nsb; ++b) {
        int64_t run = r0s[b + 1] - 1;
        for (int64_t i = r0s[b]; i < r0s[b + 1]; ++i) run = std::max<int64_t>(run, cmax[i]);
        if (run - r0s[b] + 1 > win) return false;
        spans[b] = (int32_t)(run - r0s[b] + 1);
    }
    pre.assign(nsb, 0);
    off.assign(nsb + 1, 0);
    pre[0] = (int32_t)spill_in;
    if (spill_in > r0s[1] - r0s[0]) return false;
    for (int64_t b = 1; b < nsb; ++b) {
        pre[b] = (int32_t)(spans[b - 1] - (r0s[b] - r0s[b - 1]));
        if (pre[b] > r0s[b + 1] - r0s[b]) return false;  // would reach two superblocks ahead
    }
    if (spans[nsb - 1] - (r0s[nsb] - r0s[nsb - 1]) > spill_out) return false;
    for (int64_t b = 0; b < nsb; ++b) off[b + 1] = off[b] + pre[b];
    return true;
}

int symsell_plan(int64_t n, const int32_t* cmax, int win, std::vector<int64_t>& r0s,
                 std::vector<int32_t>& spans, std::vector<int32_t>& pre, std::vector<int64_t>& off,
                 int64_t spill_in, int64_t spill_out, int64_t kQuantum) {
    if (n <= 0) return -1;
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c = std::max<int64_t>(cmax[i], i);
        if (c >= n + spill_out || c - i + 1 > win) return -1;
        m = std::max<int64_t>(m, c - i);
    }
    auto balanced = [&](int64_t k) {
        r0s.resize(k + 1);
        for (int64_t b = 0; b <= k; ++b) r0s[b] = b * n / k;
        return plan_check(n, cmax, win, r0s, spans, pre, off, spill_in, spill_out);
    };
    // k blocks with the first one lighter: workgroup 0 walks chain 0 and then
    // runs the step's deferred finalize (k_csr_ssell FUSE), so the finalize
    // overlaps the other chains instead of trailing them.  Superblock 0 (of R
    // rows) is shortened by d = 8% of R / chain -- at n = 1e7 (chain 4) 2% of R,
    // ~0.5% of chain 0's rows, about 1 us of its walk; AHIP_LIGHT_SB=2 takes
    // the larger d = 8% of the chain's rows (2 R chain / 25) for the
    // A/B.  Inside a chain the window shift needs span <= 2R, so the first
    // superblock keeps at least the reach m.
    auto light_first = [&](int64_t k) {
        if (!light_first_sb() || kQuantum <= 0 || k % kQuantum != 0 || k < 2) return false;
        const int64_t chain = k / kQuantum, R = n / k;
        int64_t d = light_sb_chain() ? (R * 2 * chain) / 25 : (R * 2) / (25 * chain);
        if (chain > 1 && R - d < m + 1) d = R - (m + 1);
        if (d <= 0) return false;
        r0s.resize(k + 1);
        r0s[0] = 0;
        r0s[1] = R - d;
        for (int64_t b = 2; b <= k; ++b) r0s[b] = r0s[1] + (b - 1) * (n - r0s[1]) / (k - 1);
        if (!plan_check(n, cmax, win, r0s, spans, pre, off, spill_in, spill_out)) return false;
        for (int64_t b = 0; b < k; ++b)  // keep the chained window shift possible
            if (chain > 1 && spans[b] > 2 * (r0s[b + 1] - r0s[b])) return false;
        return true;
    };
    const int64_t rmax = win - m;  // >= 1
    const int64_t k0 = (n + rmax - 1) / rmax;
    const int64_t kq = (k0 + kQuantum - 1) / kQuantum * kQuantum;
    if (kq <= n && (light_first(kq) || balanced(kq))) return 0;
    if (balanced(k0)) return 0;
    // greedy: extend each superblock while its window fits
    r0s.assign(1, 0);
    int64_t start = 0, run = -1;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c = std::max<int64_t>(cmax[i], i);
        const int64_t nrun = std::max(run, c);
        if (i > start && nrun - start + 1 > win) {
            r0s.push_back(i);
            start = i;
            run = c;
        } else {
            run = nrun;
        }
    }
    r0s.push_back(n);
    return plan_check(n, cmax, win, r0s, spans, pre, off, spill_in, spill_out) ? 0 : -1;
}

// Host analysis (once per matrix): greedy superblocks under the window, the
// spill-inside-the-next-superblock rule, SELL slices of the upper rows.
// -1 when the matrix does not fit the scheme (rectangular / distributed, a row
// wider than the window, or a spill reaching past the next superblock).
int csr_build_symsell(Csr& A, int64_t ncols, int64_t coff, int64_t spill_in, int64_t spill_out,
                      void** owned) {
    const int64_t n = A.n;
    if (ncols != coff + n + spill_out || n <= 0 || ncols >= (int64_t)INT32_MAX) return -1;
    const int64_t nc = n + spill_out;  // columns that receive transposed terms
    int32_t *dcnt = nullptr, *dcm = nullptr, *dcc = nullptr;
    unsigned long long* dst = nullptr;  // amax, amin bits
    auto free_all = [&]() {
        (void)hipFree(dcnt);
        (void)hipFree(dcm);
        (void)hipFree(dcc);
        (void)hipFree(dst);
    };
    if (fault_filter(hipMalloc(&dcnt, sizeof(int32_t) * n)) != hipSuccess ||
        fault_filter(hipMalloc(&dcm, sizeof(int32_t) * n)) != hipSuccess ||
        fault_filter(hipMalloc(&dcc, sizeof(int32_t) * nc)) != hipSuccess ||
        fault_filter(hipMalloc(&dst, 2 * sizeof(unsigned long long))) != hipSuccess) {
        free_all();
        return -2;
    }
    int64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    const unsigned long long init[2] = {0ull, (unsigned long long)0x7fefffffffffffffll};  // 0, DBL_MAX
    bool got = fault_filter(hipMemcpy(dst, init, sizeof(init), hipMemcpyHostToDevice)) == hipSuccess &&
               fault_filter(hipMemset(dcc, 0, sizeof(int32_t) * nc)) == hipSuccess;
    if (got)
        AHIP_LAUNCH(k_upper_stats, dim3((unsigned)g), dim3(256), 0, nullptr, n, coff, A.rowptr, A.col,
                    A.val, dcnt, dcm, dst, dcc);
    std::vector<int32_t> cnt(n), cm(n), ccol(nc);
    unsigned long long hst[2] = {0, 0}, hmin = 0;
    got = got &&
          fault_filter(hipMemcpy(cnt.data(), dcnt, sizeof(int32_t) * n, hipMemcpyDeviceToHost)) == hipSuccess &&
          fault_filter(hipMemcpy(cm.data(), dcm, sizeof(int32_t) * n, hipMemcpyDeviceToHost)) == hipSuccess &&
          fault_filter(hipMemcpy(ccol.data(), dcc, sizeof(int32_t) * nc, hipMemcpyDeviceToHost)) == hipSuccess &&
          fault_filter(hipMemcpy(hst, dst, sizeof(unsigned long long), hipMemcpyDeviceToHost)) == hipSuccess &&
          fault_filter(hipMemcpy(&hmin, dst + 1, sizeof(unsigned long long), hipMemcpyDeviceToHost)) == hipSuccess;
    free_all();
    if (!got) return -2;
    // the most transposed terms one word sums (per column, not the
    // row's lower count, which equals it only for a structurally symmetric
    // pattern and never sees the spill columns)
    for (int64_t j = 0; j < nc; ++j) hst[1] = std::max<unsigned long long>(hst[1], (unsigned long long)ccol[j]);
    // rows with columns before the block (a distributed block's low halo): the
    // spill-free exchange computes their lower ghost terms locally
    int64_t lg_rows = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (cnt[i] >> 30) lg_rows = i + 1;
        cnt[i] &= (1 << 30) - 1;
    }
    std::vector<int64_t> r0s, off;
    std::vector<int32_t> spans, pre;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || ncu < 1)
        ncu = 256;
    if (symsell_plan(n, cm.data(), kSymWin, r0s, spans, pre, off, spill_in, spill_out, ncu) != 0)
        return -1;
    const int64_t nsb = (int64_t)spans.size();
    // SELL-64 slices of the upper rows, longest first (stable)
    std::vector<int64_t> slice0{0}, sptr{0}, slice_r0;
    std::vector<int32_t> srow, order;
    int64_t nnz_u = 0;
    for (int64_t b = 0; b < nsb; ++b) {
        const int64_t R0 = r0s[b], R1 = r0s[b + 1];
        order.resize((size_t)(R1 - R0));
        for (int64_t r = R0; r < R1; ++r) {
            order[r - R0] = (int32_t)r;
            nnz_u += cnt[r];
        }
        std::stable_sort(order.begin(), order.end(),
                         [&](int32_t a, int32_t c) { return cnt[a] > cnt[c]; });
        for (size_t q = 0; q < order.size(); q += 64) {
            const int64_t w = cnt[order[q]];
            for (size_t l = 0; l < 64; ++l) srow.push_back(q + l < order.size() ? order[q + l] : -1);
            sptr.push_back(sptr.back() + 64 * w);
            slice_r0.push_back(R0);
        }
        slice0.push_back((int64_t)sptr.size() - 1);
    }
    // balanced walk (k_csr_ssell_bal): wave q of superblock b takes the column
    // steps [wg0[b*NW+q], wg0[b*NW+q+1]) of the superblock's flattened slices,
    // starting in slice wsl[b*NW+q] (the non-empty slice holding its first step)
    constexpr int NW = kSymThreads / 64;
    std::vector<int64_t> wg0((size_t)nsb * NW + 1);
    std::vector<int32_t> wsl((size_t)nsb * NW);
    for (int64_t b = 0; b < nsb; ++b) {
        const int64_t sa = slice0[b], sz = slice0[b + 1];
        const int64_t G0 = sptr[sa] >> 6, T = (sptr[sz] >> 6) - G0;
        for (int q = 0; q < NW; ++q) {
            const int64_t g0 = G0 + T * q / NW;
            const int64_t s = std::upper_bound(sptr.begin() + sa, sptr.begin() + sz, g0 << 6) - sptr.begin() - 1;
            wg0[(size_t)b * NW + q] = g0;
            wsl[(size_t)b * NW + q] = (int32_t)std::max<int64_t>(s, sa);
        }
    }
    wg0[(size_t)nsb * NW] = sptr.back() >> 6;
    // slots: off[nsb] combined rows, then the outgoing spill (spill_out)
    const int64_t ns = (int64_t)sptr.size() - 1, padded = sptr.back(), ncomb = off[nsb];
    const int64_t nslot = ncomb + spill_out;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t b_r0 = sizeof(int64_t) * (nsb + 1), b_sp = sizeof(int32_t) * nsb,
                 b_pre = sizeof(int32_t) * nsb, b_off = sizeof(int64_t) * (nsb + 1),
                 b_s0 = sizeof(int64_t) * (nsb + 1), b_ptr = sizeof(int64_t) * (ns + 1),
                 b_row = sizeof(int32_t) * srow.size(),
                 b_val = sizeof(double) * (size_t)std::max<int64_t>(padded, 1),
                 b_cw = sizeof(uint16_t) * (size_t)std::max<int64_t>(padded, 1),
                 b_slot = sizeof(double) * (size_t)std::max<int64_t>(nslot, 1),
                 b_wg0 = sizeof(int64_t) * wg0.size(), b_wsl = sizeof(int32_t) * wsl.size(),
                 b_pair = sizeof(int32_t) * (nsb + 2);
    char* d = nullptr;
    if (fault_filter(hipMalloc(&d, up(b_r0) + up(b_sp) + up(b_pre) + up(b_off) + up(b_s0) + up(b_ptr) +
                                       up(b_row) + up(b_val) + up(b_cw) + 2 * up(b_slot) + up(b_wg0) +
                                       up(b_wsl) + up(b_pair))) != hipSuccess)
        return -2;
    char* p = d;
    auto take = [&](size_t bytes) {
        char* r = p;
        p += up(bytes);
        return r;
    };
    auto* d_r0 = (int64_t*)take(b_r0);
    auto* d_sp = (int32_t*)take(b_sp);
    auto* d_pre = (int32_t*)take(b_pre);
    auto* d_off = (int64_t*)take(b_off);
    auto* d_s0 = (int64_t*)take(b_s0);
    auto* d_ptr = (int64_t*)take(b_ptr);
    auto* d_row = (int32_t*)take(b_row);
    auto* d_val = (double*)take(b_val);
    auto* d_cw = (uint16_t*)take(b_cw);
    auto* d_lo = (double*)take(b_slot);
    auto* d_hi = (double*)take(b_slot);
    auto* d_wg0 = (int64_t*)take(b_wg0);
    auto* d_wsl = (int32_t*)take(b_wsl);
    auto* d_pair = (int*)take(b_pair);
    auto h2d = [](void* dst, const void* src, size_t bytes) {
        return fault_filter(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)) == hipSuccess;
    };
    bool ok = h2d(d_wg0, wg0.data(), b_wg0) && h2d(d_wsl, wsl.data(), b_wsl) &&
              h2d(d_r0, r0s.data(), b_r0) && h2d(d_sp, spans.data(), b_sp) &&
              h2d(d_pre, pre.data(), b_pre) && h2d(d_off, off.data(), b_off) &&
              h2d(d_s0, slice0.data(), b_s0) && h2d(d_ptr, sptr.data(), b_ptr) &&
              h2d(d_row, srow.data(), b_row);
    int64_t* d_sr0 = nullptr;
    if (ok && ns > 0) {
        ok = fault_filter(hipMalloc(&d_sr0, sizeof(int64_t) * ns)) == hipSuccess &&
             h2d(d_sr0, slice_r0.data(), sizeof(int64_t) * ns);
        if (ok)
            AHIP_LAUNCH(k_symsell_fill, dim3((unsigned)ns), dim3(64), 0, nullptr, coff, d_ptr, d_row,
                        d_sr0, A.rowptr, A.col, A.val, d_cw, d_val);
    }
    // the outgoing spill's tail past the last window is never written: zero it once
    ok = ok && fault_filter(hipMemset(d_lo, 0, b_slot)) == hipSuccess;
    ok = ok && fault_filter(hipMemset(d_pair, 0, b_pair)) == hipSuccess;  // (FUSE pair counters)
    ok = ok && fault_filter(hipDeviceSynchronize()) == hipSuccess;
    if (d_sr0) (void)hipFree(d_sr0);
    if (!ok) {
        (void)hipFree(d);
        return -2;
    }
    A.ss_sb_r0 = d_r0;
    A.ss_sb_span = d_sp;
    A.ss_sb_pre = d_pre;
    A.ss_sb_off = d_off;
    A.ss_slice0 = d_s0;
    A.ss_ptr = d_ptr;
    A.ss_row = d_row;
    A.ss_val = d_val;
    A.ss_colw = d_cw;
    A.ss_lo = d_lo;
    A.ss_hi = d_hi;
    A.ss_wg0 = d_wg0;
    A.ss_wsl = d_wsl;
    A.ss_pair = d_pair;
    A.ss_nsb = nsb;
    // chains of consecutive superblocks, one workgroup per CU (k_csr_ssell);
    // the in-LDS window shift needs span <= 2R (true for the balanced plan)
    bool shift_ok = true;
    for (int64_t b = 0; b < nsb; ++b) shift_ok = shift_ok && spans[b] <= 2 * (r0s[b + 1] - r0s[b]);
    A.ss_chain = (shift_ok && nsb >= ncu && nsb % ncu == 0) ? (int)(nsb / ncu) : 1;
    A.ss_nnz = nnz_u;
    A.ss_padded = padded;
    A.ss_ncomb = ncomb;
    A.ss_coff = coff;
    A.ss_spill_out = spill_out;
    A.ss_lg_rows = lg_rows;
    A.ss_pre0 = pre[0];
    A.ss_lg = 0;  // (set by arpack_hip_csr_set_symmetric when every rank can)
    // the fixed-point form (k_csr_ssell_det): a free LDS word past every
    // window, >= 40 bits a term after the headroom for the most transposed
    // terms a row receives (L < 2^hb), a finite scale
    {
        double amax;
        std::memcpy(&amax, &hst[0], sizeof amax);
        const int L = (int)(uint32_t)hst[1];
        int hb = 0;
        while (hb < 31 && (1ll << hb) <= (long long)L) ++hb;
        int maxspan = 0;
        for (int64_t b = 0; b < nsb; ++b) maxspan = std::max(maxspan, (int)spans[b]);
        A.ss_amax = amax;
        A.ss_bits = std::min(51, 62 - hb);
        const bool scaled = amax == 0.0 || (amax >= 0x1p-900 && amax <= 0x1p900);  // (NaN: no)
        A.ss_det = (maxspan <= kSymWin - 1 && A.ss_bits >= 40 && scaled) ? 1 : 0;
        // the DEFAULT accumulator takes the fixed-point form only where the
        // off-diagonal magnitudes span <= 2^20: every term is then rounded to
        // <= 2^-31 of the smallest entry's product with the window's max|x|
        // (a graded operator's small entries keep the fp64 form's
        // relative accuracy; deterministic mode takes the form regardless)
        double amin;
        std::memcpy(&amin, &hmin, sizeof amin);
        A.ss_fx_ok = A.ss_det && (amax == 0.0 || amax <= 0x1p20 * amin) ? 1 : 0;
        int64_t ms = 0;
        for (int64_t b = 0; b < nsb; ++b) ms = std::max<int64_t>(ms, slice0[b + 1] - slice0[b]);
        A.ss_detq = (int)((ms + NW - 1) / NW);
    }
    *owned = d;
    return 0;
}

// variant 7: no chaining (one superblock per workgroup launch), for A/B
static int sym_chain(const Csr& A) { return A.ss_variant == 7 ? 1 : A.ss_chain; }
// AHIP_SPMV_YNT=1: the default kernel stores y with non-temporal stores (A/B knob)
static bool spmv_ynt() {
    static const bool on = [] {
        const char* e = getenv("AHIP_SPMV_YNT");
        return e && e[0] == '1';
    }();
    return on;
}

// the fixed-point form wherever it serves the operator on every rank: by
// default, or always in deterministic mode (an operator outside the form runs
// the LDS fp64 form by default, the full-storage kernel in deterministic mode)
static bool sym_det(const Csr& A) {
    return A.ss_det_all && ((A.ss_acc == 0 && A.ss_fx_all) || deterministic());
}
// AHIP_HANDOFF=2: the fused chain-head hand-off in the memory model's acq_rel
// form instead of the measured sc1 form (k_csr_ssell FUSE = 2 vs 1, A/B)
static int handoff_form() {
    static const int f = [] {
        const char* e = getenv("AHIP_HANDOFF");
        return e && e[0] == '2' ? 2 : 1;
    }();
    return f;
}
// MAXQ: slices a wave walks in one superblock -- at most 10 (rows <= span <=
// kSymWin - 1); 6 (superblocks of <= 96 slices, the NS operator's 88) keeps
// the kernel inside 128 VGPRs without spilling
template <int FUSE>
static void launch_det(hipStream_t s, const Csr& A, const double* x, double* y, int* pair,
                       const FinArgs& fa) {
    const int chain = sym_chain(A);
    const int64_t nch = (A.ss_nsb + chain - 1) / chain;
    auto* kern = A.ss_detq <= 6 ? &k_csr_ssell<8, true, false, FUSE, true, 6>
                                : &k_csr_ssell<8, true, false, FUSE, true, 10>;
    AHIP_LAUNCH(kern, dim3((unsigned)nch), dim3(kSymThreads), 0, s, A.ss_sb_r0, A.ss_sb_span, A.ss_sb_pre,
                A.ss_sb_off, A.ss_slice0, A.ss_ptr, A.ss_row, A.ss_colw, A.ss_val, x, y, A.ss_lo,
                A.ss_hi, A.ss_coff, chain, A.ss_nsb, pair, fa, A.ss_amax, A.ss_bits);
}

void csr_spmv_sym_main(hipStream_t s, const Csr& A, const double* x, double* y) {
    if (sym_det(A)) {
        launch_det<0>(s, A, x, y, nullptr, FinArgs{});
        return;
    }
    auto go = [&](auto kern) {
        const int chain = sym_chain(A);
        const int64_t nch = (A.ss_nsb + chain - 1) / chain;
        AHIP_LAUNCH(kern, dim3((unsigned)nch), dim3(kSymThreads), 0, s, A.ss_sb_r0,
                           A.ss_sb_span, A.ss_sb_pre, A.ss_sb_off, A.ss_slice0, A.ss_ptr, A.ss_row,
                           A.ss_colw, A.ss_val, x, y, A.ss_lo, A.ss_hi, A.ss_coff, chain, A.ss_nsb,
                           (int*)nullptr, FinArgs{}, 0.0, 0);
    };
    // measured on the NS operator (tools/spmv_sym_time.py, one process, before
    // chaining): U = 8 with non-temporal val/col loads 0.594 ms incl. the
    // combine; U = 8 plain 0.611, U = 12 0.611, U = 6 0.626, U = 4 0.652,
    // U = 2 0.671, U = 16 spills.  Diagnostic builds (wrong y, not kept):
    // without the transposed LDS adds 0.611 (U = 4), without any LDS traffic
    // 0.559 -- the slice stream, not the atomics, bounds it.
    auto go_bal = [&](auto kern) {
        const int chain = A.ss_chain;
        const int64_t nch = (A.ss_nsb + chain - 1) / chain;
        AHIP_LAUNCH(kern, dim3((unsigned)nch), dim3(kSymThreads), 0, s, A.ss_sb_r0,
                           A.ss_sb_span, A.ss_sb_pre, A.ss_sb_off, A.ss_wg0, A.ss_wsl, A.ss_ptr,
                           A.ss_row, A.ss_colw, A.ss_val, x, y, A.ss_lo, A.ss_hi, A.ss_coff, chain,
                           A.ss_nsb);
    };
    switch (A.ss_variant) {  // alternative unrolls for tools/spmv_sym_time.py
        case 8: go_bal(k_csr_ssell_bal<8, true>); break;
        case 9: go_bal(k_csr_ssell_bal<6, true>); break;
        case 10: go_bal(k_csr_ssell_bal<12, true>); break;
        case 3: go(k_csr_ssell<8, false>); break;
        case 4: go(k_csr_ssell<4, false>); break;
        case 5: go(k_csr_ssell<6, true>); break;
        case 6: go(k_csr_ssell<12, true>); break;
        case 11: go(k_csr_ssell<8, true, true>); break;  // y stored non-temporally
        default:  // 7: the same without chaining
            if (spmv_ynt()) go(k_csr_ssell<8, true, true>);
            else go(k_csr_ssell<8, true>);
            break;
    }
}

void csr_spmv_sym_combine(hipStream_t s, const Csr& A, double* y, const double* x_ext, FinQueue* q) {
    const int chain = sym_chain(A);
    const int64_t nch = (A.ss_nsb + chain - 1) / chain;
    if (x_ext && A.ss_lg) {  // spill-free form: the head rows' lower ghost terms here
        FinArgs fa{};
        size_t lds = 0;
        if (!take_deferred_finalize(q, &fa, &lds, 64 * 1024)) {
            flush_deferred_finalize(q, s);
            fa = FinArgs{};
            lds = 0;
        }
        const int64_t nlg = (A.ss_pre0 + 255) / 256;  // (ss_lg: lg_rows <= pre[0])
        AHIP_LAUNCH(fa.hs ? k_ssell_combine_lg<true> : k_ssell_combine_lg<false>,
                    dim3((unsigned)(nch + nlg)), dim3(1024), lds, s, A.ss_sb_r0, A.ss_sb_pre,
                    A.ss_sb_off, A.ss_lo, A.ss_hi, y, chain, (int)nch, A.rowptr, A.col, A.val,
                    x_ext, A.ss_coff, fa);
        return;
    }
    if (A.ss_ncomb <= 0) {
        flush_deferred_finalize(q, s);
        return;
    }
    FinArgs fa{};
    size_t lds = 0;
    if (!take_deferred_finalize(q, &fa, &lds, 64 * 1024)) {
        flush_deferred_finalize(q, s);  // (one too large for this launch's LDS)
        AHIP_LAUNCH(k_ssell_combine, dim3((unsigned)nch), dim3(1024), 0, s, A.ss_sb_r0,
                    A.ss_sb_pre, A.ss_sb_off, A.ss_lo, A.ss_hi, y, chain);
        return;
    }
    // the step's deferred finalize rides in this launch (workgroup 0)
    AHIP_LAUNCH(fa.hs ? k_ssell_combine_fin<true> : k_ssell_combine_fin<false>, dim3((unsigned)nch),
                dim3(1024), lds, s, A.ss_sb_r0, A.ss_sb_pre, A.ss_sb_off, A.ss_lo, A.ss_hi, y, chain,
                fa);
}

// AHIP_SPMV_FUSE=0: the combine (and a deferred finalize) as a launch of its own
static bool spmv_fuse() {
    static const bool on = [] {
        const char* e = getenv("AHIP_SPMV_FUSE");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool csr_spmv_sym_fusable(const Csr& A) {
    // one GPU (coff = spill = 0), the default kernel, counters allocated
    return A.ss_pair && A.ss_coff == 0 && A.ss_spill_out == 0 &&
           (A.ss_variant == 0 || A.ss_variant == 7) && !spmv_ynt();
}

void csr_spmv_sym(hipStream_t s, const Csr& A, const double* x, double* y, FinQueue* q) {
    csr_spmv_sym_as(s, A, x, y, spmv_fuse(), q);
}

void csr_spmv_sym_as(hipStream_t s, const Csr& A, const double* x, double* y, bool want_fuse,
                     FinQueue* q) {
    const bool fuse = want_fuse && csr_spmv_sym_fusable(A);
    if (!fuse) {
        csr_spmv_sym_main(s, A, x, y);
        csr_spmv_sym_combine(s, A, y, nullptr, q);
        return;
    }
    // the step's deferred finalize rides along when it fits the spent x window
    // (without the H-column staging: k_finalize<false>'s form)
    FinArgs fa{};
    size_t lds = 0;
    if (!take_deferred_finalize(q, &fa, &lds, sizeof(double) * kSymWin, false)) {
        flush_deferred_finalize(q, s);
        fa = FinArgs{};
    }
    const int chain = sym_chain(A);
    const int64_t nch = (A.ss_nsb + chain - 1) / chain;
    if (sym_det(A)) {
        if (handoff_form() == 2) launch_det<2>(s, A, x, y, A.ss_pair, fa);
        else launch_det<1>(s, A, x, y, A.ss_pair, fa);
        return;
    }
    auto go = [&](auto kern) {
        AHIP_LAUNCH(kern, dim3((unsigned)nch), dim3(kSymThreads), 0, s, A.ss_sb_r0, A.ss_sb_span,
                    A.ss_sb_pre, A.ss_sb_off, A.ss_slice0, A.ss_ptr, A.ss_row, A.ss_colw, A.ss_val, x, y,
                    A.ss_lo, A.ss_hi, A.ss_coff, chain, A.ss_nsb, A.ss_pair, fa, 0.0, 0);
    };
    if (handoff_form() == 2) go(k_csr_ssell<8, true, false, 2>);
    else go(k_csr_ssell<8, true, false, 1>);
}

}  // namespace ahip::dev

// Host-only view of the plan (CPU-tested, tests/test_symsell_plan.py): writes
// nsb, then r0s[0..nsb], spans[0..nsb), pre[0..nsb) (caller sizes them n + 1).
extern "C" int arpack_hip_kit_symsell_plan(int64_t n, const int32_t* cmax, int win, int64_t spill_in,
                                           int64_t spill_out, int64_t* nsb, int64_t* r0s, int32_t* spans,
                                           int32_t* pre) {
    std::vector<int64_t> r, o;
    std::vector<int32_t> sp, pr;
    const int rc = ahip::dev::symsell_plan(n, cmax, win, r, sp, pr, o, spill_in, spill_out, 256);
    *nsb = rc == 0 ? (int64_t)sp.size() : 0;
    if (rc != 0) return rc;
    std::copy(r.begin(), r.end(), r0s);
    std::copy(sp.begin(), sp.end(), spans);
    std::copy(pr.begin(), pr.end(), pre);
    return 0;
}
