// RCCL communicator of the multi-GPU (row-block) engine.  One process per GPU;
// the 128-byte unique id is created by rank 0 and handed to the other ranks by
// the launcher's control plane (bench.py: torch.distributed over gloo).
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/arpack_hip.h"
#include "dist.hpp"

namespace ahip {

struct Comm {
    ncclComm_t nccl = nullptr;
    // a second communicator (ncclCommSplit of nccl, same ranks) for the SpMV's
    // point-to-point halo / spill exchange on its own stream, so it can run
    // while the Gram-Schmidt allreduce of the same step is in flight on the
    // engine's stream (operations of ONE communicator must not be issued to two
    // streams concurrently); nullptr: everything on nccl, serialised
    ncclComm_t nccl_p2p = nullptr;
    int rank = 0, nranks = 1, device = 0;
    uint64_t gen = 0;          // distinguishes communicators created at the same address
    double* d_flag = nullptr;  // device scratch of dist_all_ok (allocated at init)
    int failed = 0;            // sticky: a collective or the transport reported an error
    // host-staged transport (arpack_hip_comm_init_host): the launcher's own
    // collectives move the scalars and halos through host memory
    arpack_hip_host_allreduce_fn h_allreduce = nullptr;
    arpack_hip_host_halo_fn h_halo = nullptr;
    void* h_ctx = nullptr;
    std::vector<double> h_buf;
};

static Comm* g_comm = nullptr;
static uint64_t g_gen = 0;

Comm* comm_get() { return g_comm; }
int comm_rank(const Comm* c) { return c ? c->rank : 0; }
int comm_size(const Comm* c) { return c ? c->nranks : 1; }
uint64_t comm_gen(const Comm* c) { return c ? c->gen : 0; }
bool comm_alive(const Comm* c, uint64_t gen) { return c && c == g_comm && c->gen == gen; }
double* comm_flag(const Comm* c) { return c ? c->d_flag : nullptr; }
bool comm_has_p2p(const Comm* c) { return c && c->nccl_p2p; }
bool comm_is_host(const Comm* c) { return c && c->h_halo; }

// Record an RCCL / HIP failure of a collective: the communicator is marked
// failed and the engine's drivers turn that into info = -9999 at their next
// return (a failed collective leaves the ranks' sums inconsistent, so the solve
// cannot continue).
static void note(const Comm* c, bool ok) {
    if (!ok) const_cast<Comm*>(c)->failed = 1;
}

int comm_failed(const Comm* c) {
    if (!c) return 0;
    for (ncclComm_t cm : {c->nccl, c->nccl_p2p}) {  // both communicators' async errors
        if (c->failed || !cm) continue;
        ncclResult_t a = ncclSuccess;
        if (ncclCommGetAsyncError(cm, &a) != ncclSuccess || (a != ncclSuccess && a != ncclInProgress))
            const_cast<Comm*>(c)->failed = 1;
    }
    return c->failed;
}

int comm_allreduce_sum(const Comm* c, double* dev, int count, hipStream_t stream) {
    if (!c) return 0;
    if (c->h_allreduce) {
        auto* m = const_cast<Comm*>(c);
        m->h_buf.resize((size_t)count);
        bool ok = hipMemcpyAsync(m->h_buf.data(), dev, sizeof(double) * count,
                                 hipMemcpyDeviceToHost, stream) == hipSuccess &&
                  hipStreamSynchronize(stream) == hipSuccess;
        // the transport is collective: call it even after a local failure so the
        // other ranks are not left waiting; the failure is recorded
        c->h_allreduce(m->h_buf.data(), count, c->h_ctx);
        ok = ok &&
             hipMemcpyAsync(dev, m->h_buf.data(), sizeof(double) * count, hipMemcpyHostToDevice,
                            stream) == hipSuccess &&
             hipStreamSynchronize(stream) == hipSuccess;
        note(c, ok);
        return ok ? 0 : -1;
    }
    if (!c->nccl) return 0;
    const bool ok =
        ncclAllReduce(dev, dev, (size_t)count, ncclDouble, ncclSum, c->nccl, stream) == ncclSuccess;
    note(c, ok);
    return ok ? 0 : -1;
}

static Comm* comm_new(int nranks, int rank, int device) {
    auto* c = new Comm;
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    c->gen = ++g_gen;
    if (hipMalloc(&c->d_flag, sizeof(double)) != hipSuccess) {
        delete c;
        return nullptr;
    }
    return c;
}

static void comm_free(Comm* c) {
    if (c->nccl_p2p) (void)ncclCommDestroy(c->nccl_p2p);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->d_flag) (void)hipFree(c->d_flag);
    delete c;
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
    if (nranks < 1 || rank < 0 || rank >= nranks) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    auto* c = ahip::comm_new(nranks, rank, device);
    if (!c) return -2;
    {   // a 1-rank communicator is real too, so the distributed path runs on one GPU
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
        if (ncclCommInitRank(&c->nccl, nranks, uid, rank) != ncclSuccess) {
            c->nccl = nullptr;
            ahip::comm_free(c);
            return -1;
        }
        // only for the opt-in overlapped SpMV (AHIP_DIST_OVERLAP=1; the variable
        // must be the same on every rank): collective on every rank, right here;
        // a failure leaves the serialised path (also split for one rank, where it
        // carries no traffic, so the 1-rank rehearsal runs that stream schedule)
        const char* ov = std::getenv("AHIP_DIST_OVERLAP");
        if (ov && ov[0] == '1' &&
            ncclCommSplit(c->nccl, 0, rank, &c->nccl_p2p, nullptr) != ncclSuccess)
            c->nccl_p2p = nullptr;
    }
    if (ahip::g_comm) arpack_hip_comm_destroy();
    ahip::g_comm = c;
    return 0;
}

int arpack_hip_comm_init_host(int nranks, int rank, arpack_hip_host_allreduce_fn allreduce,
                              arpack_hip_host_halo_fn halo, void* ctx, int device) {
    if (!allreduce || !halo || nranks < 1 || rank < 0 || rank >= nranks) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    auto* c = ahip::comm_new(nranks, rank, device);
    if (!c) return -2;
    c->h_allreduce = allreduce;
    c->h_halo = halo;
    c->h_ctx = ctx;
    if (ahip::g_comm) arpack_hip_comm_destroy();
    ahip::g_comm = c;
    return 0;
}

void arpack_hip_comm_destroy(void) {
    if (!ahip::g_comm) return;
    ahip::comm_free(ahip::g_comm);
    ahip::g_comm = nullptr;
}

int arpack_hip_comm_failed(void) { return ahip::comm_failed(ahip::g_comm); }

int arpack_hip_comm_rank(void) { return ahip::comm_rank(ahip::g_comm); }
int arpack_hip_comm_size(void) { return ahip::comm_size(ahip::g_comm); }

// In-place SUM allreduce of a device buffer (test hook for the RCCL plumbing).
int arpack_hip_comm_allreduce(double* dev, int count) {
    const int rc = ahip::comm_allreduce_sum(ahip::g_comm, dev, count, nullptr);
    return rc == 0 && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

}  // extern "C"

namespace ahip {

// Halo exchange of the distributed SpMV (grouped point-to-point over xGMI).
static void comm_halo_host(const Comm* c, const DistOp& D, hipStream_t s, bool hi_only) {
    const int r = c->rank, P = c->nranks;
    const int64_t slo = r > 0 ? D.send_lo : 0, shi = r < P - 1 && !hi_only ? D.send_hi : 0;
    const int64_t hlo = r > 0 && !hi_only ? D.halo_lo : 0, hhi = r < P - 1 ? D.halo_hi : 0;
    std::vector<double> b((size_t)(slo + shi + hlo + hhi));
    double *bsl = b.data(), *bsh = bsl + slo, *brl = bsh + shi, *brh = brl + hlo;
    bool ok = true;
    if (slo) ok = ok && hipMemcpyAsync(bsl, D.x_mid(), 8 * slo, hipMemcpyDeviceToHost, s) == hipSuccess;
    if (shi)
        ok = ok && hipMemcpyAsync(bsh, D.x_mid() + D.nloc - shi, 8 * shi, hipMemcpyDeviceToHost, s) ==
                       hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    c->h_halo(bsl, slo, brl, hlo, bsh, shi, brh, hhi, c->h_ctx);  // collective: always joined
    if (hlo) ok = ok && hipMemcpyAsync(D.x_ext, brl, 8 * hlo, hipMemcpyHostToDevice, s) == hipSuccess;
    if (hhi)
        ok = ok && hipMemcpyAsync(D.x_mid() + D.nloc, brh, 8 * hhi, hipMemcpyHostToDevice, s) ==
                       hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    note(c, ok);
}

// Forward "spill" of the symmetric-storage SpMV: send nsend doubles to rank+1,
// receive nrecv from rank-1 (the reverse of the x halo's hi side).
void comm_spill(const Comm* c, const double* send, int64_t nsend, double* recv, int64_t nrecv,
                hipStream_t s, bool p2p) {
    if (!c || c->nranks == 1) return;
    const int r = c->rank, P = c->nranks;
    const int64_t ns = r < P - 1 ? nsend : 0, nr = r > 0 ? nrecv : 0;
    if (c->h_halo) {
        std::vector<double> b((size_t)(ns + nr));
        bool ok = true;
        if (ns) ok = hipMemcpyAsync(b.data(), send, 8 * ns, hipMemcpyDeviceToHost, s) == hipSuccess;
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        c->h_halo(nullptr, 0, b.data() + ns, nr, b.data(), ns, nullptr, 0, c->h_ctx);
        if (nr)
            ok = ok && hipMemcpyAsync(recv, b.data() + ns, 8 * nr, hipMemcpyHostToDevice, s) == hipSuccess;
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        note(c, ok);
        return;
    }
    ncclComm_t cm = p2p && c->nccl_p2p ? c->nccl_p2p : c->nccl;
    bool ok = ncclGroupStart() == ncclSuccess;
    if (ns) ok = ncclSend(send, (size_t)ns, ncclDouble, r + 1, cm, s) == ncclSuccess && ok;
    if (nr) ok = ncclRecv(recv, (size_t)nr, ncclDouble, r - 1, cm, s) == ncclSuccess && ok;
    ok = ncclGroupEnd() == ncclSuccess && ok;
    note(c, ok);
}

// hi_only: the symmetric-storage SpMV reads x only at and above its own rows,
// so only the hi halo travels (my first rows to rank-1, rank+1's to me).
void comm_halo(const Comm* c, const DistOp& D, hipStream_t s, bool hi_only, bool p2p) {
    if (!c || c->nranks == 1) return;
    if (c->h_halo) return comm_halo_host(c, D, s, hi_only);
    const int r = c->rank, P = c->nranks;
    ncclComm_t cm = p2p && c->nccl_p2p ? c->nccl_p2p : c->nccl;
    bool ok = ncclGroupStart() == ncclSuccess;
    auto chk = [&](ncclResult_t e) { ok = ok && e == ncclSuccess; };
    if (r > 0) {
        if (D.send_lo) chk(ncclSend(D.x_mid(), (size_t)D.send_lo, ncclDouble, r - 1, cm, s));
        if (D.halo_lo && !hi_only) chk(ncclRecv(D.x_ext, (size_t)D.halo_lo, ncclDouble, r - 1, cm, s));
    }
    if (r < P - 1) {
        if (D.send_hi && !hi_only)
            chk(ncclSend(D.x_mid() + D.nloc - D.send_hi, (size_t)D.send_hi, ncclDouble, r + 1, cm, s));
        if (D.halo_hi) chk(ncclRecv(D.x_mid() + D.nloc, (size_t)D.halo_hi, ncclDouble, r + 1, cm, s));
    }
    chk(ncclGroupEnd());
    note(c, ok);
}

// The general distributed SpMV's exchange over RCCL: one group of point-to-
// point transfers, every peer pair only in the direction it has data for.
void comm_ghosts(const Comm* c, const DistOp& D, hipStream_t s, bool p2p) {
    if (!c || c->nranks == 1 || !c->nccl) return;
    const int r = c->rank, P = c->nranks;
    ncclComm_t cm = p2p && c->nccl_p2p ? c->nccl_p2p : c->nccl;
    bool ok = ncclGroupStart() == ncclSuccess;
    auto chk = [&](ncclResult_t e) { ok = ok && e == ncclSuccess; };
    for (int q = 0; q < P; ++q) {
        if (q == r) continue;
        if (D.mode == DistOp::kGhostLists) {
            if (D.send_cnt[q])
                chk(ncclSend(D.send_buf + D.send_off[q], (size_t)D.send_cnt[q], ncclDouble, q, cm, s));
            if (D.recv_cnt[q])
                chk(ncclRecv(D.x_ext + D.nloc + D.recv_off[q], (size_t)D.recv_cnt[q], ncclDouble, q,
                             cm, s));
        } else {  // kAllGather
            if (D.nloc) chk(ncclSend(D.x_mid(), (size_t)D.nloc, ncclDouble, q, cm, s));
            if (D.peer_nloc[q])
                chk(ncclRecv(D.x_ext + D.peer_row0[q], (size_t)D.peer_nloc[q], ncclDouble, q, cm, s));
        }
    }
    chk(ncclGroupEnd());
    note(c, ok);
}

}  // namespace ahip
