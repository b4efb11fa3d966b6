// Definition of the opaque arpack_hip_csr handle (shared by csr.hip / dist.hip).
#pragma once
#include <cstdint>

#include "device.hpp"

namespace ahip {
struct Comm;
}
struct arpack_hip_dist;

struct arpack_hip_csr {
    ahip::dev::Csr A;
    int64_t* rowptr = nullptr;
    int32_t* col = nullptr;
    double* val = nullptr;
    int64_t row_begin = 0;  // global index of local row 0 (sharded generators)
    int64_t ncols = 0;
    int64_t* rblk = nullptr;  // CSR-stream row blocks (owned)
    void* win = nullptr;      // LDS-window superblock tables (owned)
    void* sell = nullptr;     // SELL-64 slices + values (owned, built on demand)
    void* symsell = nullptr;  // symmetric-storage layout (owned, arpack_hip_csr_set_symmetric)
    // row distribution seen by the symmetric layout (arpack_hip_dist_create):
    // x = [sym_coff | local rows | sym_spill_out], sym_spill_in leading rows
    // receive the previous rank's transposed terms
    int64_t sym_coff = 0, sym_spill_in = 0, sym_spill_out = 0;
    // set by arpack_hip_dist_create: the CSR is one rank's block of a row-
    // distributed operator, so a storage-mode switch must be agreed by all ranks
    // (cleared by arpack_hip_dist_destroy)
    arpack_hip_dist* dist = nullptr;
};


// the live communicator of A's distribution (nullptr if A is not distributed
// or, with *stale = true, if that communicator has been destroyed)
const ahip::Comm* ahip_csr_dist_comm(const arpack_hip_csr* A, bool* stale);
void ahip_dist_detach_csr(arpack_hip_dist* D);
// the exchange form of a distribution (DistOp::Mode; 0 for the neighbour halo)
int ahip_dist_mode(const arpack_hip_dist* D);

// remap every column index c -> c - shift (int32) and rebuild the SpMV
// analysis for an x vector of length ncols; 0 on success
int ahip_csr_remap_cols(arpack_hip_csr* A, int64_t shift, int64_t ncols);
// ghost-list form (general operators): own columns [row0, row0 + nloc) ->
// c - row0, any other -> nloc + its index in `ghosts` (device, sorted, nghost);
// x is then [nloc local | nghost ghosts]
int ahip_csr_remap_ghost(arpack_hip_csr* A, int64_t row0, int64_t nloc, const int64_t* ghosts,
                         int64_t nghost);
// per-matrix [min col, max col] over all rows (device reduction)
int ahip_csr_col_span(const arpack_hip_csr* A, int64_t* cmin, int64_t* cmax);
