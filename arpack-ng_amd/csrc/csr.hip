// Device CSR operator (the `ido = +-1` user OP served on the GPU) and the
// synthetic-operator generators used by the benchmarks and parity tests.
//
// Generators build the matrices directly in HBM (count -> exclusive scan ->
// fill), deterministically from a counter-based hash, so the CPU baseline and
// every GPU count see bit-identical operators (BASELINE.md §3 "Inputs").
//
//  laplace2d   5-pt 2-D Laplacian, m x m grid (EXAMPLES/SIMPLE/dssimp.f:484-538
//              operator shape; `scale` = 1/h^2 = (m+1)^2 reproduces dssimp)
//  laplace3d   7-pt 3-D Laplacian, m^3 (BASELINE config 4)
//  anderson    Laplacian + W*u_i on the diagonal (SURVEY.md §8c G3 "3-D Anderson"):
//              breaks the Laplacian's exact eigenvalue multiplicities
//  banded_sym  the north-star symmetric CSR: pairs (i, i+d), 1 <= d < B, are
//              present with probability per_row/4096 (~2*per_row nnz/row),
//              off-diagonal values -k/4096 (k in 1..4096), diagonal
//              -sum(offdiag) + U[0,16) on a 2^-8 grid.  All values are on
//              power-of-two grids, so row sums are exact in any order and a
//              row-block of the matrix generated on one GPU is bit-identical
//              to the same rows generated anywhere else.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstring>
#include <vector>

#include "device.hpp"
#include "../../include/arpack_hip.h"

#include "csr_internal.hpp"
#include "dist.hpp"

namespace ahip::gen {

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__host__ __device__ __forceinline__ uint32_t pair_hash(uint32_t seedmix, uint32_t a, uint32_t d) {
    return mix32(mix32(a ^ seedmix) + d * 0x9E3779B9u);
}
__host__ __device__ __forceinline__ double offdiag_value(uint32_t h) {
    return -(double)((mix32(h ^ 0x68e31da4u) >> 20) + 1u) * 0x1p-12;
}
__host__ __device__ __forceinline__ double diag_shift(uint32_t seed, uint32_t i) {
    return (double)(mix32(i ^ mix32(seed ^ 0x5bd1e995u)) >> 20) * 0x1p-8;
}

// ---- banded symmetric (north star) -----------------------------------------
__global__ void k_band_count(int64_t n, int64_t r0, int64_t r1, uint32_t seed, int B, int per_row,
                             int64_t* __restrict__ cnt) {
    const uint32_t sm = mix32(seed);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < r1 - r0; li += stride) {
        const int64_t i = r0 + li;
        int64_t c = 1;
        for (int d = 1; d < B; ++d) {
            if (i - d >= 0 && (pair_hash(sm, (uint32_t)(i - d), (uint32_t)d) >> 20) < (uint32_t)per_row) ++c;
            if (i + d < n && (pair_hash(sm, (uint32_t)i, (uint32_t)d) >> 20) < (uint32_t)per_row) ++c;
        }
        cnt[li] = c;
    }
}

__global__ void k_band_fill(int64_t n, int64_t r0, int64_t r1, uint32_t seed, int B, int per_row,
                            const int64_t* __restrict__ rp, int32_t* __restrict__ col,
                            double* __restrict__ val) {
    const uint32_t sm = mix32(seed);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < r1 - r0; li += stride) {
        const int64_t i = r0 + li;
        int64_t k = rp[li];
        double sum = 0.0;
        for (int d = B - 1; d >= 1; --d) {  // lower part, increasing column
            if (i - d < 0) continue;
            const uint32_t h = pair_hash(sm, (uint32_t)(i - d), (uint32_t)d);
            if ((h >> 20) < (uint32_t)per_row) {
                const double v = offdiag_value(h);
                col[k] = (int32_t)(i - d);
                val[k] = v;
                sum += v;
                ++k;
            }
        }
        const int64_t kd = k++;
        for (int d = 1; d < B; ++d) {
            if (i + d >= n) break;
            const uint32_t h = pair_hash(sm, (uint32_t)i, (uint32_t)d);
            if ((h >> 20) < (uint32_t)per_row) {
                const double v = offdiag_value(h);
                col[k] = (int32_t)(i + d);
                val[k] = v;
                sum += v;
                ++k;
            }
        }
        col[kd] = (int32_t)i;
        val[kd] = -sum + diag_shift(seed, (uint32_t)i);
    }
}

// ---- Laplacians -----------------------------------------------------------------
// rows [r0, r0 + rows) of the m^dim grid operator (a row block for the
// distributed engine: PARPACK/EXAMPLES/MPI/pdsdrv1.f's slab decomposition; the
// whole operator is r0 = 0, rows = n), columns global
__global__ void k_lap_count(int64_t m, int dim, int64_t r0, int64_t rows, int64_t* __restrict__ cnt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < rows; li += stride) {
        const int64_t i = r0 + li;
        const int64_t x = i % m, y = (i / m) % m, z = dim == 3 ? i / (m * m) : 0;
        int64_t c = 1 + (x > 0) + (x < m - 1) + (y > 0) + (y < m - 1);
        if (dim == 3) c += (z > 0) + (z < m - 1);
        cnt[li] = c;
    }
}

__global__ void k_lap_fill(int64_t m, int dim, int64_t r0, int64_t rows, double scale, double disorder,
                           uint32_t seed, const int64_t* __restrict__ rp, int32_t* __restrict__ col,
                           double* __restrict__ val) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const double off = -1.0 * scale, dg = (dim == 2 ? 4.0 : 6.0) * scale;
    for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < rows; li += stride) {
        const int64_t i = r0 + li;
        const int64_t x = i % m, y = (i / m) % m, z = dim == 3 ? i / (m * m) : 0;
        int64_t k = rp[li];
        auto put = [&](int64_t j, double v) { col[k] = (int32_t)j; val[k] = v; ++k; };
        if (dim == 3 && z > 0) put(i - m * m, off);
        if (y > 0) put(i - m, off);
        if (x > 0) put(i - 1, off);
        // Anderson disorder: + W * u_i, u_i on a 2^-12 grid in [0,1) (exact sums)
        const double u = disorder != 0.0
                             ? (double)(mix32((uint32_t)i ^ mix32(seed ^ 0x2545f491u)) >> 20) * 0x1p-12
                             : 0.0;
        put(i, dg + disorder * u);
        if (x < m - 1) put(i + 1, off);
        if (y < m - 1) put(i + m, off);
        if (dim == 3 && z < m - 1) put(i + m * m, off);
    }
}

// 2-D convection-diffusion -Lap u + rho du/dx on the unit square (the dndrv1 /
// dnsimp operator, EXAMPLES/NONSYM/dndrv1.f:397-475): x-neighbours dl/du,
// y-neighbours offy, diagonal dd (coefficients computed on the host).
__global__ void k_cd_fill(int64_t m, double dd, double dl, double du, double offy,
                          const int64_t* __restrict__ rp, int32_t* __restrict__ col,
                          double* __restrict__ val) {
    const int64_t n = m * m;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t x = i % m, y = i / m;
        int64_t k = rp[i];
        auto put = [&](int64_t j, double v) { col[k] = (int32_t)j; val[k] = v; ++k; };
        if (y > 0) put(i - m, offy);
        if (x > 0) put(i - 1, dl);
        put(i, dd);
        if (x < m - 1) put(i + 1, du);
        if (y < m - 1) put(i + m, offy);
    }
}

}  // namespace ahip::gen

namespace {

int pick_group(int64_t n, int64_t nnz) {
    const double avg = n > 0 ? (double)nnz / (double)n : 1.0;
    if (avg <= 6) return 4;
    if (avg <= 14) return 8;
    if (avg <= 48) return 16;
    if (avg <= 100) return 32;
    return 64;
}

int grid_of(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    return (int)(g < 1 ? 1 : g);
}

// counts[0..rows) -> rowptr[0..rows] (exclusive scan, rowptr[rows] = nnz).
// Returns nnz, or -2 when the scan's scratch cannot be allocated / any HIP call
// fails (the caller frees its buffers and reports the error).
int64_t scan_counts(int64_t rows, int64_t* counts_then_rowptr_tmp, int64_t* rowptr) {
    void* tmp = nullptr;
    size_t bytes = 0;
    if (hipMemset(counts_then_rowptr_tmp + rows, 0, sizeof(int64_t)) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(tmp, bytes, counts_then_rowptr_tmp, rowptr, rows + 1) !=
            hipSuccess ||
        hipMalloc(&tmp, bytes) != hipSuccess)
        return -2;
    const bool ok =
        hipcub::DeviceScan::ExclusiveSum(tmp, bytes, counts_then_rowptr_tmp, rowptr, rows + 1) ==
            hipSuccess &&
        hipDeviceSynchronize() == hipSuccess;
    (void)hipFree(tmp);
    int64_t nnz = 0;
    if (!ok || hipMemcpy(&nnz, rowptr + rows, sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return -2;
    return nnz;
}

// Count -> scan -> fill of a generated operator: `count(cnt)` writes the row
// counts, `fill(rp, col, val)` the entries.  Every allocation and launch is
// checked; on failure nothing leaks and -2 is returned.
template <class Count, class Fill>
int build_generated(int64_t rows, Count count, Fill fill, int64_t** rp_out, int32_t** col_out,
                    double** val_out, int64_t* nnz_out) {
    int64_t *cnt = nullptr, *rp = nullptr;
    int32_t* col = nullptr;
    double* val = nullptr;
    auto fail = [&]() {
        (void)hipFree(cnt);
        (void)hipFree(rp);
        (void)hipFree(col);
        (void)hipFree(val);
        return -2;
    };
    if (hipMalloc(&cnt, sizeof(int64_t) * (rows + 1)) != hipSuccess ||
        hipMalloc(&rp, sizeof(int64_t) * (rows + 1)) != hipSuccess)
        return fail();
    count(cnt);
    if (hipGetLastError() != hipSuccess) return fail();
    const int64_t nnz = scan_counts(rows, cnt, rp);
    (void)hipFree(cnt);
    cnt = nullptr;
    if (nnz < 0) return fail();
    if (hipMalloc(&col, sizeof(int32_t) * (nnz > 0 ? nnz : 1)) != hipSuccess ||
        hipMalloc(&val, sizeof(double) * (nnz > 0 ? nnz : 1)) != hipSuccess)
        return fail();
    fill(rp, col, val);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return fail();
    *rp_out = rp;
    *col_out = col;
    *val_out = val;
    *nnz_out = nnz;
    return 0;
}

// LDS x-window tables, then the SELL-64 layout over them (default kernel);
// matrices whose rows span more than a window keep the CSR-stream kernel.
// -2 if a HIP call of the analysis failed (-1 from a builder: the layout does
// not fit this matrix, and the next form is tried).
int analyse_window_sell(arpack_hip_csr* A, int64_t ncols) {
    int rc = ahip::dev::csr_analyse_window(A->A, ncols, &A->win);
    if (rc == -2) return -2;
    if (rc != 0) {
        // rows spanning several distant column bands (a 3-D stencil in natural
        // order): multi-range windows, read by the SELL kernel only
        rc = ahip::dev::csr_analyse_ranges(A->A, ncols, &A->win);
        if (rc != 0) return rc == -2 ? -2 : 0;
    } else {
        A->A.kernel = ahip::dev::kCsrWVecX;
    }
    rc = ahip::dev::csr_build_sell(A->A, &A->sell);
    if (rc == -2) return -2;
    if (rc == 0) {
        A->A.kernel = ahip::dev::kCsrSell;
        A->A.s_unroll = 10;  // U = 4 with non-temporal val/col loads (tools/spmv_full_time.py)
    }
    return 0;
}

// The operator object over device arrays rp/col/val (ownership taken) and its
// SpMV plans.  0, or -2 if a HIP call of the plan builders failed: then
// everything, rp/col/val included, is released and *out is untouched.
int finish(arpack_hip_csr** out, int64_t rows, int64_t ncols, int64_t nnz, int64_t* rp, int32_t* col,
           double* val) {
    auto* A = new arpack_hip_csr;
    A->rowptr = rp;
    A->col = col;
    A->val = val;
    A->ncols = ncols;
    A->A.n = rows;
    A->A.nnz = nnz;
    A->A.rowptr = rp;
    A->A.col = col;
    A->A.val = val;
    A->A.group = pick_group(rows, nnz);
    int rc = ahip::dev::csr_analyse(A->A, 4096, &A->rblk);
    if (rc == 0) A->A.kernel = ahip::dev::kCsrStream;
    if (rc != -2) rc = analyse_window_sell(A, ncols);
    if (rc == -2) {
        arpack_hip_csr_destroy(A);
        return -2;
    }
    *out = A;
    return 0;
}

}  // namespace

extern "C" {

int arpack_hip_csr_create(arpack_hip_csr** out, int64_t n, int64_t nnz, const int64_t* rowptr,
                          const int32_t* col, const double* val) {
    int64_t* rp = nullptr;
    int32_t* c = nullptr;
    double* v = nullptr;
    bool ok = hipMalloc(&rp, sizeof(int64_t) * (n + 1)) == hipSuccess &&
              hipMalloc(&c, sizeof(int32_t) * (nnz > 0 ? nnz : 1)) == hipSuccess &&
              hipMalloc(&v, sizeof(double) * (nnz > 0 ? nnz : 1)) == hipSuccess &&
              hipMemcpy(rp, rowptr, sizeof(int64_t) * (n + 1), hipMemcpyDefault) == hipSuccess;
    if (ok && nnz > 0)
        ok = hipMemcpy(c, col, sizeof(int32_t) * nnz, hipMemcpyDefault) == hipSuccess &&
             hipMemcpy(v, val, sizeof(double) * nnz, hipMemcpyDefault) == hipSuccess;
    if (!ok) {
        (void)hipFree(rp);
        (void)hipFree(c);
        (void)hipFree(v);
        return -1;
    }
    return finish(out, n, n, nnz, rp, c, v);
}

void arpack_hip_csr_destroy(arpack_hip_csr* A) {
    if (!A) return;
    ahip_dist_detach_csr(A->dist);
    (void)hipFree(A->rowptr);
    (void)hipFree(A->col);
    (void)hipFree(A->val);
    if (A->rblk) (void)hipFree(A->rblk);
    if (A->win) (void)hipFree(A->win);
    if (A->sell) (void)hipFree(A->sell);
    if (A->symsell) (void)hipFree(A->symsell);
    if (A->A.w_colw) (void)hipFree((void*)A->A.w_colw);
    A->A.w_colw = nullptr;
    delete A;
}

// SELL-64 layout statistics (0 slices if it was never built)
int arpack_hip_csr_sell_info(const arpack_hip_csr* A, int64_t* nslices, int64_t* padded) {
    *nslices = A->A.s_nslices;
    *padded = A->A.s_padded;
    return A->sell ? 0 : -1;
}

int arpack_hip_csr_info(const arpack_hip_csr* A, int64_t* n, int64_t* nnz) {
    *n = A->A.n;
    *nnz = A->A.nnz;
    return 0;
}

int arpack_hip_csr_download(const arpack_hip_csr* A, int64_t* rowptr, int32_t* col, double* val) {
    const bool ok =
        hipMemcpy(rowptr, A->rowptr, sizeof(int64_t) * (A->A.n + 1), hipMemcpyDeviceToHost) == hipSuccess &&
        (A->A.nnz == 0 ||
         (hipMemcpy(col, A->col, sizeof(int32_t) * A->A.nnz, hipMemcpyDeviceToHost) == hipSuccess &&
          hipMemcpy(val, A->val, sizeof(double) * A->A.nnz, hipMemcpyDeviceToHost) == hipSuccess));
    return ok ? 0 : -1;
}

int arpack_hip_csr_spmv(const arpack_hip_csr* A, const double* x, double* y) {
    // x may come from the caller's own GPU work on a non-blocking stream, which
    // the null stream does not order against: complete it first
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    ahip::dev::csr_spmv(nullptr, A->A, x, y);
    // synchronous like the reference callers' OP: y is complete on return
    return hipStreamSynchronize(nullptr) == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -1;
}

static void csr_full_storage(arpack_hip_csr* A) {
    if (A->A.kernel == ahip::dev::kCsrSymSell)
        A->A.kernel = A->sell ? ahip::dev::kCsrSell
                              : (A->rblk ? ahip::dev::kCsrStream : ahip::dev::kCsrVector);
}

int arpack_hip_csr_set_symmetric(arpack_hip_csr* A, int on) {
    // one rank's block of a distributed operator: the symmetric SpMV changes the
    // exchange pattern (hi-only halo + forward spill), so the switch -- either
    // way -- is collective, and every rank falls back to full storage if any
    // rank's plan failed
    bool stale = false;
    const ahip::Comm* c = ahip_csr_dist_comm(A, &stale);
    if (stale) return -3;  // its communicator was destroyed: no agreement possible
    if (!on) {
        if (c && !ahip::dist_all_ok(c, 1)) return -2;
        csr_full_storage(A);
        return 0;
    }
    // a general operator's block (ghost lists / all-gather) has no spill
    // exchange for the transposed terms: full storage stays, reported as kept
    // (1, as in deterministic mode) -- the mode is the same on every rank, so no
    // agreement is needed.  (A banded block declared symmetric before
    // arpack_hip_dist_create keeps the neighbour halo and symmetric storage.)
    if (A->dist && ahip_dist_mode(A->dist) != 0) {
        csr_full_storage(A);
        return 1;
    }
    int rc = 0;
    if (!A->symsell)
        rc = ahip::dev::csr_build_symsell(A->A, A->ncols, A->sym_coff, A->sym_spill_in,
                                          A->sym_spill_out, &A->symsell);
    if (c && !ahip::dist_all_ok(c, rc == 0)) {
        csr_full_storage(A);
        return rc != 0 ? rc : -2;
    }
    if (rc != 0) return rc;
    // whether the fixed-point form (k_csr_ssell_det) serves every rank (a
    // second agreement, made in either mode, so that deterministic mode turned
    // on later finds it agreed); in deterministic mode without it the
    // fixed-order full-storage SpMV stays, reported as kept (1) on every rank
    const bool det = A->A.ss_det != 0;
    A->A.ss_det_all = (c ? ahip::dist_all_ok(c, det) : det) ? 1 : 0;
    const bool fx = A->A.ss_fx_ok != 0;
    A->A.ss_fx_all = (c ? ahip::dist_all_ok(c, fx) : fx) ? 1 : 0;
    if (ahip::deterministic() && !A->A.ss_det_all) {
        csr_full_storage(A);
        return 1;
    }
    A->A.kernel = ahip::dev::kCsrSymSell;
    // a distributed block: the spill-free exchange when every rank's lower ghost
    // rows lie inside its incoming spill's rows (structurally symmetric
    // coupling); AHIP_DIST_SPILL=1 keeps the spill
    if (A->dist) {
        const char* e = std::getenv("AHIP_DIST_SPILL");
        const bool want = !(e && e[0] == '1');
        A->A.ss_lg = ahip::dist_all_ok(c, want && A->A.ss_lg_rows <= A->A.ss_pre0) ? 1 : 0;
    }
    return 0;
}

int arpack_hip_csr_set_sym_accumulator(arpack_hip_csr* A, int acc) {
    if (!A || (acc != 0 && acc != 1)) return -1;
    A->A.ss_acc = acc;
    return 0;
}

int arpack_hip_csr_sym_form(const arpack_hip_csr* A) {
    const ahip::dev::Csr& M = A->A;
    if (M.kernel != ahip::dev::kCsrSymSell || !M.ss_val || ahip::dev::csr_sym_det_fallback(M)) return 0;
    return M.ss_det_all && ((M.ss_acc == 0 && M.ss_fx_all) || ahip::deterministic()) ? 2 : 1;
}

int arpack_hip_csr_set_kernel(arpack_hip_csr* A, int kernel, int tile) {
    if (kernel == ahip::dev::kCsrSymSell) {  // tile selects the variant
        const int rc = arpack_hip_csr_set_symmetric(A, 1);
        if (rc == 0) A->A.ss_variant = tile >= 0 && tile <= 16 ? tile : 0;
        return rc;
    }
    if (kernel == ahip::dev::kCsrVector) {
        A->A.kernel = kernel;
        return 0;
    }
    if (kernel == ahip::dev::kCsrSell) {  // tile selects the unroll (4, 8, 16)
        if (!A->sell && ahip::dev::csr_build_sell(A->A, &A->sell) != 0) return -1;
        A->A.kernel = kernel;
        A->A.s_unroll = (tile >= 2 && tile <= 11) ? tile : 4;  // 5, 7: two slices per wave; 9-11 NT
        return 0;
    }
    if (kernel >= ahip::dev::kCsrWindow && kernel <= ahip::dev::kCsrWVecP4) {
        if (!A->win || A->A.w_rng) return -1;  // multi-range windows: SELL only
        A->A.kernel = kernel;
        return 0;
    }
    if (tile != 2048 && tile != 4096) return -1;
    if (A->A.tile != tile || !A->rblk) {
        if (A->rblk) (void)hipFree(A->rblk);
        A->rblk = nullptr;
        A->A.rblk = nullptr;
        if (ahip::dev::csr_analyse(A->A, tile, &A->rblk) != 0) return -1;
    }
    A->A.kernel = kernel;
    return 0;
}

double arpack_hip_csr_time(const arpack_hip_csr* A, const double* x, double* y, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    ahip::dev::csr_spmv(nullptr, A->A, x, y);  // warm
    (void)hipEventRecord(a, nullptr);
    for (int r = 0; r < reps; ++r) ahip::dev::csr_spmv(nullptr, A->A, x, y);
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return (double)ms / reps;
}

static int gen_lap(arpack_hip_csr** out, int64_t m, int dim, double scale, double disorder = 0.0,
                   uint32_t seed = 0, int64_t r0 = 0, int64_t r1 = -1) {
    const int64_t n = dim == 2 ? m * m : m * m * m;
    if (r1 < 0) r1 = n;
    if (m < 1 || r0 < 0 || r1 <= r0 || r1 > n) return -1;
    const int64_t rows = r1 - r0;
    int64_t *rp = nullptr, nnz = 0;
    int32_t* col = nullptr;
    double* val = nullptr;
    const int rc = build_generated(
        rows,
        [&](int64_t* cnt) {
            hipLaunchKernelGGL(ahip::gen::k_lap_count, dim3(grid_of(rows)), dim3(256), 0, nullptr, m, dim,
                               r0, rows, cnt);
        },
        [&](int64_t* rp_, int32_t* col_, double* val_) {
            hipLaunchKernelGGL(ahip::gen::k_lap_fill, dim3(grid_of(rows)), dim3(256), 0, nullptr, m, dim,
                               r0, rows, scale, disorder, seed, rp_, col_, val_);
        },
        &rp, &col, &val, &nnz);
    if (rc != 0) return rc;
    if (finish(out, rows, n, nnz, rp, col, val) != 0) return -2;
    (*out)->row_begin = r0;
    return 0;
}

int arpack_hip_gen_laplace2d(arpack_hip_csr** A, int64_t m, double scale) { return gen_lap(A, m, 2, scale); }

int arpack_hip_gen_convdiff2d(arpack_hip_csr** out, int64_t m, double rho) {
    const int64_t n = m * m;
    // coefficients exactly as EXAMPLES/NONSYM/dndrv1.f:425,458-462 compute them
    const double h = 1.0 / (double)(m + 1), h2 = h * h;
    const double dd = 4.0 / h2, dl = -1.0 / h2 - 0.5 * rho / h, du = -1.0 / h2 + 0.5 * rho / h;
    const double offy = -1.0 / (1.0 / (double)((m + 1) * (m + 1)));
    int64_t *rp = nullptr, nnz = 0;
    int32_t* col = nullptr;
    double* val = nullptr;
    const int rc = build_generated(
        n,
        [&](int64_t* cnt) {
            hipLaunchKernelGGL(ahip::gen::k_lap_count, dim3(grid_of(n)), dim3(256), 0, nullptr, m, 2,
                               (int64_t)0, n, cnt);
        },
        [&](int64_t* rp_, int32_t* col_, double* val_) {
            hipLaunchKernelGGL(ahip::gen::k_cd_fill, dim3(grid_of(n)), dim3(256), 0, nullptr, m, dd, dl,
                               du, offy, rp_, col_, val_);
        },
        &rp, &col, &val, &nnz);
    if (rc != 0) return rc;
    return finish(out, n, n, nnz, rp, col, val);
}
int arpack_hip_gen_laplace3d(arpack_hip_csr** A, int64_t m, double scale) { return gen_lap(A, m, 3, scale); }
int arpack_hip_gen_laplace3d_rows(arpack_hip_csr** A, int64_t m, int64_t r0, int64_t r1, double scale) {
    return gen_lap(A, m, 3, scale, 0.0, 0, r0, r1);
}
int arpack_hip_gen_anderson(arpack_hip_csr** A, int64_t m, int dim, double disorder, uint32_t seed) {
    return gen_lap(A, m, dim, 1.0, disorder, seed);
}

int arpack_hip_gen_banded_sym(arpack_hip_csr** out, int64_t n, int64_t r0, int64_t r1, uint32_t seed,
                              int bandwidth, int per_row) {
    if (r1 <= r0 || r1 > n || bandwidth < 2) return -1;
    const int64_t rows = r1 - r0;
    int64_t *rp = nullptr, nnz = 0;
    int32_t* col = nullptr;
    double* val = nullptr;
    const int rc = build_generated(
        rows,
        [&](int64_t* cnt) {
            hipLaunchKernelGGL(ahip::gen::k_band_count, dim3(grid_of(rows)), dim3(256), 0, nullptr, n,
                               r0, r1, seed, bandwidth, per_row, cnt);
        },
        [&](int64_t* rp_, int32_t* col_, double* val_) {
            hipLaunchKernelGGL(ahip::gen::k_band_fill, dim3(grid_of(rows)), dim3(256), 0, nullptr, n,
                               r0, r1, seed, bandwidth, per_row, rp_, col_, val_);
        },
        &rp, &col, &val, &nnz);
    if (rc != 0) return rc;
    if (finish(out, rows, n, nnz, rp, col, val) != 0) return -2;
    (*out)->row_begin = r0;
    return 0;
}

}  // extern "C"

const ahip::dev::Csr* ahip_csr_view(const arpack_hip_csr* A) { return &A->A; }

// ------------------------------------------------------------ remap helpers --
namespace {
__global__ void k_shift_cols(int64_t nnz, int32_t* col, int64_t shift) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += stride)
        col[k] = (int32_t)((int64_t)col[k] - shift);
}
// ghost-list remap of a general operator's block (dist.hip ghost plan): own
// columns [row0, row0 + nloc) -> c - row0, others -> nloc + their index in the
// sorted ghost list (binary search; every off-block column is in the list)
__global__ void k_remap_ghost(int64_t nnz, int32_t* col, int64_t row0, int64_t nloc,
                              const int64_t* __restrict__ ghosts, int64_t nghost) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += stride) {
        const int64_t c = col[k];
        if (c >= row0 && c < row0 + nloc) {
            col[k] = (int32_t)(c - row0);
            continue;
        }
        int64_t lo = 0, hi = nghost;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (ghosts[mid] < c) lo = mid + 1;
            else hi = mid;
        }
        col[k] = (int32_t)(nloc + lo);
    }
}
__global__ void k_col_span(int64_t nnz, const int32_t* col, int* mn, int* mx) {
    int a = 0x7fffffff, b = -1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += stride) {
        a = min(a, col[k]);
        b = max(b, col[k]);
    }
    atomicMin(mn, a);
    atomicMax(mx, b);
}
}  // namespace

int ahip_csr_col_span(const arpack_hip_csr* A, int64_t* cmin, int64_t* cmax) {
    int* d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(int)) != hipSuccess) return -1;
    const int init[2] = {0x7fffffff, -1};
    int h[2];
    bool ok = hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice) == hipSuccess;
    if (ok && A->A.nnz > 0) {
        hipLaunchKernelGGL(k_col_span, dim3(grid_of(A->A.nnz)), dim3(256), 0, nullptr, A->A.nnz, A->col, d,
                           d + 1);
        ok = hipGetLastError() == hipSuccess;
    }
    ok = ok && hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d);
    if (!ok) return -1;
    *cmin = h[0];
    *cmax = h[1];
    return 0;
}

static int reanalyse(arpack_hip_csr* A, int64_t ncols);

int ahip_csr_remap_cols(arpack_hip_csr* A, int64_t shift, int64_t ncols) {
    if (A->A.nnz > 0 && shift != 0)
        hipLaunchKernelGGL(k_shift_cols, dim3(grid_of(A->A.nnz)), dim3(256), 0, nullptr, A->A.nnz, A->col, shift);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return reanalyse(A, ncols);
}

int ahip_csr_remap_ghost(arpack_hip_csr* A, int64_t row0, int64_t nloc, const int64_t* ghosts,
                         int64_t nghost) {
    if (A->A.nnz > 0)
        hipLaunchKernelGGL(k_remap_ghost, dim3(grid_of(A->A.nnz)), dim3(256), 0, nullptr, A->A.nnz,
                           A->col, row0, nloc, ghosts, nghost);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return reanalyse(A, nloc + nghost);
}

// the SpMV analysis again for new column indices over an x of ncols entries
static int reanalyse(arpack_hip_csr* A, int64_t ncols) {
    A->ncols = ncols;
    if (A->win) (void)hipFree(A->win);
    if (A->sell) (void)hipFree(A->sell);
    if (A->symsell) (void)hipFree(A->symsell);
    A->symsell = nullptr;
    A->A.ss_val = nullptr;
    A->A.ss_pair = nullptr;
    if (A->A.w_colw) (void)hipFree((void*)A->A.w_colw);
    A->A.w_colw = nullptr;
    A->win = nullptr;
    A->sell = nullptr;
    A->A.s_val = nullptr;
    A->A.w_nsb = 0;
    A->A.w_rng = nullptr;  // (inside the freed window allocation)
    A->A.kernel = A->rblk ? ahip::dev::kCsrStream : ahip::dev::kCsrVector;
    if (analyse_window_sell(A, ncols) == -2) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- test hook: the fused symmetric SpMV's hand-off under uneven load ---------
namespace {
__global__ void k_load_stream(double* __restrict__ a, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
        a[k] = a[k] * 0.5 + 1.0;
}
}  // namespace

extern "C" int arpack_hip_test_symspmv_handoff(const arpack_hip_csr* A, const double* x, double* y,
                                               int fuse, double* load, int64_t load_n, int64_t* heads,
                                               int64_t cap, double* lo_out) {
    using namespace ahip::dev;
    const Csr& M = A->A;
    if (M.kernel != kCsrSymSell || !M.ss_val) return -1;
    if (fuse && !csr_spmv_sym_fusable(M)) return -2;
    static hipStream_t ls = nullptr;  // the competing stream (never destroyed)
    if (!ls && hipStreamCreateWithFlags(&ls, hipStreamNonBlocking) != hipSuccess) return -3;
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    // the competing read / write stream is issued first, so the SpMV's
    // workgroups land on CUs it already occupies (uneven arrival at the pairs)
    if (load && load_n > 0) hipLaunchKernelGGL(k_load_stream, dim3(4096), dim3(256), 0, ls, load, load_n);
    csr_spmv_sym_as(nullptr, M, x, y, fuse != 0);
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    // chain-head rows (combined through the slots) and the slot_lo halves they read
    const int chain = M.ss_chain;
    const int64_t nch = (M.ss_nsb + chain - 1) / chain;
    std::vector<int64_t> r0((size_t)M.ss_nsb + 1), off((size_t)M.ss_nsb + 1);
    std::vector<int32_t> pre((size_t)M.ss_nsb);
    if (hipMemcpy(r0.data(), M.ss_sb_r0, sizeof(int64_t) * r0.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(off.data(), M.ss_sb_off, sizeof(int64_t) * off.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(pre.data(), M.ss_sb_pre, sizeof(int32_t) * pre.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return -3;
    int64_t k = 0;
    for (int64_t c = 0; c < nch && k < cap; ++c) {
        const int64_t b = c * chain;
        heads[2 * k] = r0[b];
        heads[2 * k + 1] = pre[b];
        if (lo_out && pre[b] > 0 &&
            hipMemcpy(lo_out + r0[b], M.ss_lo + off[b], sizeof(double) * pre[b], hipMemcpyDeviceToHost) !=
                hipSuccess)
            return -3;
        ++k;
    }
    return (int)k;
}
