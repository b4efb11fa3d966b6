// Row-block distribution over GPUs (PARPACK's decomposition,
// PARPACK/SRC/MPI/pdsaitr.f): one process per GPU, rank r owns rows
// [row0, row0 + nloc) of V, resid, workd and of the operator.  Every inner
// product is a local partial + one RCCL allreduce of <= ncv+1 doubles (fused:
// [V'w ; w'w] in one collective where PARPACK issues 2-3 MPI_ALLREDUCEs); V*Q
// is row-local (pdsapps.f has no communication).  The SpMV needs the x entries
// of the neighbouring ranks inside its column span: a halo exchanged with
// ncclSend/ncclRecv into an extended x buffer [halo_lo | local | halo_hi].
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "device.hpp"

namespace ahip {

struct Comm;  // RCCL communicator (comm.cpp)
struct DistOp;
Comm* comm_get();
int comm_rank(const Comm*);
int comm_size(const Comm*);
// in-place SUM allreduce of `count` doubles on `stream`; 0, or -1 after an
// RCCL / HIP / transport error (also recorded: comm_failed).  timed: the
// collective is a marker span of the profiler's allreduce class (the engine's
// data path: the Gram-Schmidt sums); the control plane's flag agreements and
// plan tables pass false
int comm_allreduce_sum(const Comm*, double* dev, int count, hipStream_t stream, bool timed = true);
// nonzero once a collective of c failed (sticky; also polls RCCL's async error)
int comm_failed(const Comm* c);
// generation of a communicator and whether (c, gen) is still the live one
uint64_t comm_gen(const Comm* c);
bool comm_alive(const Comm* c, uint64_t gen);
// one device double owned by the communicator (dist_all_ok's scratch)
double* comm_flag(const Comm* c);
// the communicator has its separate point-to-point communicator (RCCL, > 1 rank)
bool comm_has_p2p(const Comm* c);
// the host-staged transport (arpack_hip_comm_init_host) rather than RCCL
bool comm_is_host(const Comm* c);
// exchanges of the general distributed SpMV (one group of send / recv, on
// RCCL or the host-staged transport):
// kGhostLists -- D.send_buf slices to each peer, ghosts into x_ext after the
// local rows; kAllGather -- x_mid to every peer, every peer's block into x_ext
void comm_ghosts(const Comm* c, const DistOp& D, hipStream_t s, bool p2p);
// collective over the ranks of c: 1 if every rank passes ok_local != 0
int dist_all_ok(const Comm* c, int ok_local);

// Distributed operator: the local CSR (columns relative to the start of x_ext)
// plus the halo plan.
struct DistOp {
    int64_t n_global = 0, row0 = 0, nloc = 0;
    int64_t halo_lo = 0, halo_hi = 0;   // x_ext = [halo_lo | nloc | halo_hi]
    int64_t send_lo = 0, send_hi = 0;   // my first rows -> rank-1, my last rows -> rank+1
    double* x_ext = nullptr;            // device, halo_lo + nloc + halo_hi
    const dev::Csr* A = nullptr;        // local rows, local (x_ext) column indices
    const Comm* comm = nullptr;
    uint64_t comm_gen = 0;              // generation of comm at creation
    // info = 0 start vector: 0 = one dlarnv stream sliced at the rank's global
    // row offset (the same iterates for every rank count); 1 = PARPACK's
    // per-rank stream (PARPACK/SRC/MPI/pdgetv0.f:234-245)
    int seed_mode = 0;
    // exchange form: kHaloNeighbour -- banded operators whose
    // columns reach at most the neighbouring ranks' rows (the slab exchange of
    // PARPACK/EXAMPLES/MPI/pdsdrv1.f); kGhostLists -- any other operator: x_ext =
    // [nloc local | halo_hi ghosts sorted by global column], each peer sends
    // exactly the rows on its precomputed list (grouped send / recv);
    // kAllGather -- ghost sets too dense to pay for lists: x_ext is the whole
    // x (halo_lo = row0), every rank's block goes to every rank
    enum Mode : int { kHaloNeighbour = 0, kGhostLists = 1, kAllGather = 2 };
    int mode = kHaloNeighbour;
    std::vector<int64_t> peer_row0, peer_nloc;        // every rank's block
    std::vector<int64_t> send_cnt, send_off;          // kGhostLists: rows for each peer
    std::vector<int64_t> recv_cnt, recv_off;          // ... and ghosts from each peer
    int32_t* send_idx = nullptr;   // device: local rows packed for the peers, in rank order
    double* send_buf = nullptr;    // device: the packed values
    int64_t nsend = 0;
    int64_t* ghost_glob = nullptr; // device: global column of each ghost (the column remap)
    double* x_mid() const { return x_ext + halo_lo; }
};

// y = A_loc * x for the distributed operator: copy x into x_ext (skipped when
// the engine already placed it there), halo exchange, local SpMV.
// p2p: run the halo / spill exchanges on the communicator's separate
// point-to-point communicator (the SpMV then may run on a stream of its own,
// concurrently with the engine stream's allreduces)
// q: the solve's deferred finalize (carried by the SpMV where it can be)
void dist_spmv(const DistOp& D, hipStream_t s, const double* x, double* y, bool p2p = false,
               dev::FinQueue* q = nullptr);

}  // namespace ahip
