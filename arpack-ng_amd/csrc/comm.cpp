// RCCL communicator of the multi-GPU (row-block) engine.  One process per GPU;
// the 128-byte unique id is created by rank 0 and handed to the other ranks by
// the launcher's control plane (bench.py: torch.distributed over gloo).
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/arpack_hip.h"
#include "device.hpp"
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
    // collectives move the scalars and the SpMV's exchanges through host memory
    arpack_hip_host_allreduce_fn h_allreduce = nullptr;
    arpack_hip_host_p2p_fn h_p2p = nullptr;
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
bool comm_is_host(const Comm* c) { return c && c->h_p2p; }

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

static int comm_allreduce_raw(const Comm* c, double* dev, int count, hipStream_t stream);

int comm_allreduce_sum(const Comm* c, double* dev, int count, hipStream_t stream, bool timed) {
    if (!c) return 0;
    if (timed) dev::prof_begin(dev::kProfAllreduce, stream);
    const int rc = comm_allreduce_raw(c, dev, count, stream);
    if (timed) dev::prof_end(dev::kProfAllreduce, stream, 8.0 * count);
    return rc;
}

static int comm_allreduce_raw(const Comm* c, double* dev, int count, hipStream_t stream) {
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
                              arpack_hip_host_p2p_fn p2p, void* ctx, int device) {
    if (!allreduce || !p2p || nranks < 1 || rank < 0 || rank >= nranks) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    auto* c = ahip::comm_new(nranks, rank, device);
    if (!c) return -2;
    c->h_allreduce = allreduce;
    c->h_p2p = p2p;
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

// One group of point-to-point transfers: every exchange of the distributed
// SpMV (the neighbour halo, the symmetric form's forward spill, the ghost
// lists, the all-gather) is built as such a list by the functions below and run
// by either transport -- RCCL (ncclSend / ncclRecv between ncclGroupStart and
// ncclGroupEnd, on the stream) or the host-staged one (the send slices copied
// to host memory, the launcher's per-peer send / recv, the received slices
// copied back).  So the host rehearsal moves exactly the device slices, counts
// and offsets the RCCL path moves; only the wire differs.
struct P2pOp {
    int peer;
    int send;      // 1: send `count` doubles from buf to peer; 0: receive into buf
    double* buf;   // device
    int64_t count;
};

static void comm_group(const Comm* c, const std::vector<P2pOp>& ops, hipStream_t s, bool p2p) {
    if (c->h_p2p) {
        int64_t tot = 0;
        for (const P2pOp& o : ops) tot += o.count;
        std::vector<double> h((size_t)tot);
        std::vector<int> peer, kind;
        std::vector<double*> hb;
        std::vector<int64_t> cnt;
        bool ok = true;
        int64_t at = 0;
        for (const P2pOp& o : ops) {
            double* hp = h.data() + at;
            at += o.count;
            if (o.send)
                ok = ok && hipMemcpyAsync(hp, o.buf, sizeof(double) * o.count, hipMemcpyDeviceToHost, s) ==
                               hipSuccess;
            peer.push_back(o.peer);
            kind.push_back(o.send);
            hb.push_back(hp);
            cnt.push_back(o.count);
        }
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        // the transport is joined even after a local copy failure, so the peers
        // are not left waiting; the failure is recorded
        c->h_p2p((int)ops.size(), peer.data(), kind.data(), hb.data(), cnt.data(), c->h_ctx);
        for (size_t k = 0; k < ops.size(); ++k)
            if (!ops[k].send)
                ok = ok && hipMemcpyAsync(ops[k].buf, hb[k], sizeof(double) * ops[k].count,
                                          hipMemcpyHostToDevice, s) == hipSuccess;
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        note(c, ok);
        return;
    }
    if (!c->nccl) return;
    ncclComm_t cm = p2p && c->nccl_p2p ? c->nccl_p2p : c->nccl;
    bool ok = ncclGroupStart() == ncclSuccess;
    for (const P2pOp& o : ops) {
        const ncclResult_t e = o.send ? ncclSend(o.buf, (size_t)o.count, ncclDouble, o.peer, cm, s)
                                      : ncclRecv(o.buf, (size_t)o.count, ncclDouble, o.peer, cm, s);
        ok = ok && e == ncclSuccess;
    }
    ok = ncclGroupEnd() == ncclSuccess && ok;
    note(c, ok);
}

// Forward "spill" of the symmetric-storage SpMV: send nsend doubles to rank+1,
// receive nrecv from rank-1 (the reverse of the x halo's hi side).
void comm_spill(const Comm* c, const double* send, int64_t nsend, double* recv, int64_t nrecv,
                hipStream_t s, bool p2p) {
    if (!c || c->nranks == 1) return;
    const int r = c->rank, P = c->nranks;
    std::vector<P2pOp> ops;
    if (r < P - 1 && nsend) ops.push_back({r + 1, 1, const_cast<double*>(send), nsend});
    if (r > 0 && nrecv) ops.push_back({r - 1, 0, recv, nrecv});
    comm_group(c, ops, s, p2p);
}

// Halo exchange of the banded distributed SpMV: my first send_lo rows to
// rank-1 and my last send_hi rows to rank+1; halo_lo rows from rank-1 into the
// head of x_ext, halo_hi rows from rank+1 after my rows.  hi_only: the
// symmetric-storage SpMV with the spill reads x only at and above its own rows,
// so only the hi halo travels (my first rows to rank-1, rank+1's to me).
void comm_halo(const Comm* c, const DistOp& D, hipStream_t s, bool hi_only, bool p2p) {
    if (!c || c->nranks == 1) return;
    const int r = c->rank, P = c->nranks;
    std::vector<P2pOp> ops;
    if (r > 0) {
        if (D.send_lo) ops.push_back({r - 1, 1, D.x_mid(), D.send_lo});
        if (D.halo_lo && !hi_only) ops.push_back({r - 1, 0, D.x_ext, D.halo_lo});
    }
    if (r < P - 1) {
        if (D.send_hi && !hi_only) ops.push_back({r + 1, 1, D.x_mid() + D.nloc - D.send_hi, D.send_hi});
        if (D.halo_hi) ops.push_back({r + 1, 0, D.x_mid() + D.nloc, D.halo_hi});
    }
    comm_group(c, ops, s, p2p);
}

// The general distributed SpMV's exchange: one group of point-to-point
// transfers, every peer pair only in the direction it has data for.
void comm_ghosts(const Comm* c, const DistOp& D, hipStream_t s, bool p2p) {
    if (!c || c->nranks == 1) return;
    const int r = c->rank, P = c->nranks;
    std::vector<P2pOp> ops;
    for (int q = 0; q < P; ++q) {
        if (q == r) continue;
        if (D.mode == DistOp::kGhostLists) {
            if (D.send_cnt[q]) ops.push_back({q, 1, D.send_buf + D.send_off[q], D.send_cnt[q]});
            if (D.recv_cnt[q]) ops.push_back({q, 0, D.x_ext + D.nloc + D.recv_off[q], D.recv_cnt[q]});
        } else {  // kAllGather
            if (D.nloc) ops.push_back({q, 1, D.x_mid(), D.nloc});
            if (D.peer_nloc[q]) ops.push_back({q, 0, D.x_ext + D.peer_row0[q], D.peer_nloc[q]});
        }
    }
    comm_group(c, ops, s, p2p);
}

}  // namespace ahip
