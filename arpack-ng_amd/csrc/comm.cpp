// RCCL communicator of the multi-GPU (row-block) engine.  One process per GPU;
// the 128-byte unique id is created by rank 0 and handed to the other ranks by
// the launcher's control plane (bench.py: torch.distributed over gloo).
#include <rccl/rccl.h>

#include <cstring>

#include "../../include/arpack_hip.h"
#include "dist.hpp"

namespace ahip {

struct Comm {
    ncclComm_t nccl = nullptr;
    int rank = 0, nranks = 1, device = 0;
};

static Comm* g_comm = nullptr;

Comm* comm_get() { return g_comm; }
int comm_rank(const Comm* c) { return c ? c->rank : 0; }
int comm_size(const Comm* c) { return c ? c->nranks : 1; }

void comm_allreduce_sum(const Comm* c, double* dev, int count, hipStream_t stream) {
    if (!c || !c->nccl) return;
    (void)ncclAllReduce(dev, dev, (size_t)count, ncclDouble, ncclSum, c->nccl, stream);
}

}  // namespace ahip

extern "C" {

int arpack_hip_comm_unique_id(char* out) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

int arpack_hip_comm_init(int nranks, int rank, const char* id, int device) {
    if (hipSetDevice(device) != hipSuccess) return -2;
    auto* c = new ahip::Comm;
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    {   // a 1-rank communicator is real too, so the distributed path runs on one GPU
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
        if (ncclCommInitRank(&c->nccl, nranks, uid, rank) != ncclSuccess) {
            delete c;
            return -1;
        }
    }
    if (ahip::g_comm) arpack_hip_comm_destroy();
    ahip::g_comm = c;
    return 0;
}

void arpack_hip_comm_destroy(void) {
    if (!ahip::g_comm) return;
    if (ahip::g_comm->nccl) (void)ncclCommDestroy(ahip::g_comm->nccl);
    delete ahip::g_comm;
    ahip::g_comm = nullptr;
}

int arpack_hip_comm_rank(void) { return ahip::comm_rank(ahip::g_comm); }
int arpack_hip_comm_size(void) { return ahip::comm_size(ahip::g_comm); }

// In-place SUM allreduce of a device buffer (test hook for the RCCL plumbing).
int arpack_hip_comm_allreduce(double* dev, int count) {
    ahip::comm_allreduce_sum(ahip::g_comm, dev, count, nullptr);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

}  // extern "C"

namespace ahip {

// Halo exchange of the distributed SpMV (grouped point-to-point over xGMI).
void comm_halo(const Comm* c, const DistOp& D, hipStream_t s) {
    if (!c || c->nranks == 1) return;
    const int r = c->rank, P = c->nranks;
    (void)ncclGroupStart();
    if (r > 0) {
        if (D.send_lo) (void)ncclSend(D.x_mid(), (size_t)D.send_lo, ncclDouble, r - 1, c->nccl, s);
        if (D.halo_lo) (void)ncclRecv(D.x_ext, (size_t)D.halo_lo, ncclDouble, r - 1, c->nccl, s);
    }
    if (r < P - 1) {
        if (D.send_hi)
            (void)ncclSend(D.x_mid() + D.nloc - D.send_hi, (size_t)D.send_hi, ncclDouble, r + 1, c->nccl, s);
        if (D.halo_hi) (void)ncclRecv(D.x_mid() + D.nloc, (size_t)D.halo_hi, ncclDouble, r + 1, c->nccl, s);
    }
    (void)ncclGroupEnd();
}

}  // namespace ahip
