// Distributed operator setup (halo plan) and the distributed SpMV.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../../include/arpack_hip.h"
#include "csr_internal.hpp"
#include "dist.hpp"

namespace ahip {
void comm_halo(const Comm* c, const DistOp& D, hipStream_t s, bool hi_only, bool p2p);
void comm_spill(const Comm* c, const double* send, int64_t nsend, double* recv, int64_t nrecv,
                hipStream_t s, bool p2p);

namespace {
__global__ void k_pack(int64_t m, const int32_t* __restrict__ idx, const double* __restrict__ x,
                       double* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride)
        out[k] = x[idx[k]];
}
inline unsigned grid_for_rows(int64_t m) {
    const int64_t g = (m + 255) / 256;
    return (unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}
}  // namespace

// The general operator's exchange (kGhostLists / kAllGather): the requested
// rows packed into send_buf (k_pack over send_idx), then one group of
// point-to-point transfers -- the same group on RCCL and on the host-staged
// rehearsal transport (comm_ghosts).
static void exchange_general(const DistOp& D, hipStream_t s, bool p2p) {
    if (D.mode == DistOp::kGhostLists && D.nsend > 0)
        hipLaunchKernelGGL(k_pack, dim3(grid_for_rows(D.nsend)), dim3(256), 0, s, D.nsend, D.send_idx,
                           D.x_mid(), D.send_buf);
    dev::prof_begin(dev::kProfHalo, s);
    comm_ghosts(D.comm, D, s, p2p);
    dev::prof_end(dev::kProfHalo, s, 0.0);
}

void dist_spmv(const DistOp& D, hipStream_t s, const double* x, double* y, bool p2p, dev::FinQueue* q) {
    if (x != D.x_mid()) dev::copy(s, D.nloc, x, D.x_mid());
    if (D.mode != DistOp::kHaloNeighbour) {
        exchange_general(D, s, p2p);
        dev::csr_spmv(s, *D.A, D.x_ext, y, q);
        return;
    }
    const dev::Csr& A = *D.A;
    // (deterministic mode without the fixed-point form on every rank: every
    // rank takes the full-storage exchange and SpMV, csr_spmv's fallback)
    const bool sym = A.kernel == dev::kCsrSymSell && A.ss_val && !dev::csr_sym_det_fallback(A);
    // spill-free symmetric form (A.ss_lg, agreed by every rank): one two-sided
    // halo, and the leading rows' lower ghost terms from the rank's own rows
    // the halo group is a marker span of its own (profiler class halo; empty
    // at one rank), inside the SpMV's span
    dev::prof_begin(dev::kProfHalo, s);
    comm_halo(D.comm, D, s, sym && !A.ss_lg, p2p);
    dev::prof_end(dev::kProfHalo, s, 0.0);
    if (sym) {
        dev::csr_spmv_sym_main(s, A, D.x_ext, y);
        // otherwise my rows' upper entries reach the next rank's first rows --
        // those transposed terms (the spill) travel forward and are combined
        // into the receiver's leading rows (a reverse halo)
        if (!A.ss_lg) {
            dev::prof_begin(dev::kProfHalo, s);
            comm_spill(D.comm, A.ss_lo + A.ss_ncomb, A.ss_spill_out, A.ss_lo, D.send_lo, s, p2p);
            dev::prof_end(dev::kProfHalo, s, 0.0);
        }
        dev::csr_spmv_sym_combine(s, A, y, D.x_ext, q);
        return;
    }
    dev::csr_spmv(s, A, D.x_ext, y, q);
}

int dist_all_ok(const Comm* c, int ok_local) {
    if (!c || comm_size(c) == 1) return ok_local != 0;
    // the communicator's own device double: no allocation that could fail on
    // one rank only, so every rank always joins the collective
    double h = ok_local ? 0.0 : 1.0, *d = comm_flag(c);  // SUM of failures
    bool ok = hipMemcpy(d, &h, sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    if (comm_allreduce_sum(c, d, 1, nullptr, false) != 0) ok = false;
    ok = ok && hipMemcpy(&h, d, sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
    return ok && h == 0.0;
}
}  // namespace ahip

struct arpack_hip_dist {
    ahip::DistOp D;
    arpack_hip_csr* csr = nullptr;  // the operator block it remapped (cleared if freed first)
};

extern "C" {

// Halo plan of rank r from every rank's [row0, nloc, min col, max col] (global
// indices).  out = {halo_lo, halo_hi, send_lo, send_hi}: rank r receives
// halo_lo rows from r-1 and halo_hi rows from r+1 and sends its first send_lo
// rows to r-1 and its last send_hi rows to r+1 (the slab exchange of
// PARPACK/EXAMPLES/MPI/pdsdrv1.f:429-480, generalised to any banded CSR).
int arpack_hip_kit_halo_plan(int P, int r, const double* tab, int64_t* out) {
    auto R0 = [&](int q) { return (int64_t)tab[4 * q]; };
    auto NL = [&](int q) { return (int64_t)tab[4 * q + 1]; };
    auto HLO = [&](int q) { return std::max<int64_t>(0, R0(q) - (int64_t)tab[4 * q + 2]); };
    auto HHI = [&](int q) {
        return std::max<int64_t>(0, (int64_t)tab[4 * q + 3] - (R0(q) + NL(q) - 1));
    };
    if (P < 1 || r < 0 || r >= P) return -1;
    // contiguous blocks in rank order, checked for every rank before any reach
    // (a -4 sends the caller to the general plan, which needs this layout)
    if (R0(0) != 0) return -3;
    for (int q = 1; q < P; ++q)
        if (R0(q) != R0(q - 1) + NL(q - 1)) return -3;
    for (int q = 0; q < P; ++q) {  // halos only from the neighbours
        if (q > 0 && HLO(q) > NL(q - 1)) return -4;
        if (q < P - 1 && HHI(q) > NL(q + 1)) return -4;
        if ((q == 0 && HLO(q) > 0) || (q == P - 1 && HHI(q) > 0)) return -4;
    }
    out[0] = HLO(r);
    out[1] = HHI(r);
    out[2] = r > 0 ? HHI(r - 1) : 0;
    out[3] = r < P - 1 ? HLO(r + 1) : 0;
    return 0;
}

}  // extern "C"

namespace {
using namespace ahip;

void free_general(DistOp& o) {
    for (void* p : {(void*)o.x_ext, (void*)o.send_idx, (void*)o.send_buf, (void*)o.ghost_glob})
        if (p) (void)hipFree(p);
    o.x_ext = o.send_buf = nullptr;
    o.send_idx = nullptr;
    o.ghost_glob = nullptr;
}

// in-place SUM allreduce of a host vector through the engine's communicator
// (plan setup only); collective, agreed: false on every rank if any failed
bool host_allreduce(const Comm* c, std::vector<double>& h) {
    double* d = nullptr;
    const size_t bytes = sizeof(double) * (h.empty() ? 1 : h.size());
    bool ok = hipMalloc(&d, bytes) == hipSuccess;
    if (!dist_all_ok(c, ok)) {
        if (d) (void)hipFree(d);
        return false;
    }
    ok = h.empty() || hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice) == hipSuccess;
    if (!h.empty() && comm_allreduce_sum(c, d, (int)h.size(), nullptr, false) != 0) ok = false;
    ok = ok && (h.empty() || hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost) == hipSuccess);
    (void)hipFree(d);
    return dist_all_ok(c, ok);
}

template <class T>
bool upload(T** dst, const std::vector<T>& h) {
    if (hipMalloc(dst, sizeof(T) * (h.empty() ? 1 : h.size())) != hipSuccess) {
        *dst = nullptr;
        return false;
    }
    return h.empty() || hipMemcpy(*dst, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice) == hipSuccess;
}

// Ghost plan of a general operator's row block (collective; SURVEY §8(e) "SpMV
// exchange"): the sorted set of off-block columns this rank's rows read
// (its ghosts), their owners, and -- through one allreduce of every rank's
// ghost list -- the rows each peer needs from this rank.  Where the ghosts are
// more than half of all off-block rows (a dense coupling, e.g. config 5's
// random operator at small P) the lists do not pay and every rank gathers the
// whole x (kAllGather; AHIP_DIST_ALLGATHER=1 forces it).
// The sorted distinct off-block columns of a block's rows (its ghosts; global
// indices).  false if the columns could not be read.
bool ghost_cols(const arpack_hip_csr* A, int64_t row0, int64_t nloc, std::vector<int64_t>& g) {
    const int64_t nnz = A->A.nnz;
    std::vector<int32_t> hc((size_t)nnz);
    g.clear();
    if (nnz > 0 && hipMemcpy(hc.data(), A->col, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost) != hipSuccess)
        return false;
    for (int32_t v : hc)
        if (v < row0 || v >= row0 + nloc) g.push_back(v);
    std::sort(g.begin(), g.end());
    g.erase(std::unique(g.begin(), g.end()), g.end());
    return true;
}

int ghost_plan(arpack_hip_csr* A, DistOp& o, const Comm* c, int P, int r) {
    const int64_t nloc = o.nloc, row0 = o.row0;
    std::vector<int64_t> g;
    const bool ok0 = ghost_cols(A, row0, nloc, g);
    if (!dist_all_ok(c, ok0)) return -1;
    bool ok = true;
    auto owner = [&](int64_t col) {
        return (int)(std::upper_bound(o.peer_row0.begin(), o.peer_row0.end(), col) - o.peer_row0.begin()) - 1;
    };
    // C[q * P + p]: ghosts of rank q owned by rank p
    std::vector<double> C((size_t)P * P, 0.0);
    for (int64_t v : g) C[(size_t)r * P + owner(v)] += 1.0;
    if (!host_allreduce(c, C)) return -1;
    double total = 0.0, possible = 0.0;
    std::vector<int64_t> nghost(P, 0), seg(P + 1, 0);
    for (int q = 0; q < P; ++q) {
        for (int p = 0; p < P; ++p) nghost[q] += (int64_t)C[(size_t)q * P + p];
        seg[q + 1] = seg[q] + nghost[q];
        total += (double)nghost[q];
        possible += (double)(o.n_global - o.peer_nloc[q]);
    }
    const char* fe = std::getenv("AHIP_DIST_ALLGATHER");
    const bool want_ag = (fe && fe[0] == '1') || total > 0.5 * possible;
    const bool all_gather = !dist_all_ok(c, !want_ag);  // any rank's wish, every rank's mode
    if (all_gather) {
        o.mode = DistOp::kAllGather;
        o.halo_lo = row0;
        o.halo_hi = o.n_global - row0 - nloc;
        ok = hipMalloc(&o.x_ext, sizeof(double) * o.n_global) == hipSuccess &&
             hipMemset(o.x_ext, 0, sizeof(double) * o.n_global) == hipSuccess;
        // global column indices stay: x_ext is the whole x
        ok = ok && ahip_csr_remap_cols(A, 0, o.n_global) == 0;
        return dist_all_ok(c, ok) ? 0 : -1;
    }
    o.mode = DistOp::kGhostLists;
    // every rank's sorted ghost list, back to back (rank q's at seg[q])
    std::vector<double> lists((size_t)seg[P], 0.0);
    for (size_t k = 0; k < g.size(); ++k) lists[(size_t)seg[r] + k] = (double)g[k];
    if (!host_allreduce(c, lists)) return -1;
    o.send_cnt.assign(P, 0);
    o.send_off.assign(P, 0);
    o.recv_cnt.assign(P, 0);
    o.recv_off.assign(P, 0);
    std::vector<int32_t> sidx;
    for (int q = 0; q < P; ++q) {
        // q's ghosts owned by me: a contiguous run of q's sorted list
        int64_t at = seg[q];
        for (int p = 0; p < r; ++p) at += (int64_t)C[(size_t)q * P + p];
        const int64_t cnt = q == r ? 0 : (int64_t)C[(size_t)q * P + r];
        o.send_off[q] = (int64_t)sidx.size();
        o.send_cnt[q] = cnt;
        for (int64_t k = 0; k < cnt; ++k) sidx.push_back((int32_t)((int64_t)lists[(size_t)(at + k)] - row0));
    }
    for (int q = 0, acc = 0; q < P; ++q) {
        o.recv_off[q] = acc;
        o.recv_cnt[q] = q == r ? 0 : (int64_t)C[(size_t)r * P + q];
        acc += (int)o.recv_cnt[q];
    }
    lists = std::vector<double>();
    o.nsend = (int64_t)sidx.size();
    o.halo_lo = 0;
    o.halo_hi = (int64_t)g.size();
    const int64_t next = nloc + o.halo_hi;
    ok = hipMalloc(&o.x_ext, sizeof(double) * (next > 0 ? next : 1)) == hipSuccess &&
         hipMemset(o.x_ext, 0, sizeof(double) * (next > 0 ? next : 1)) == hipSuccess &&
         upload(&o.send_idx, sidx) &&
         hipMalloc(&o.send_buf, sizeof(double) * (o.nsend > 0 ? o.nsend : 1)) == hipSuccess &&
         upload(&o.ghost_glob, g);
    ok = ok && ahip_csr_remap_ghost(A, row0, nloc, o.ghost_glob, o.halo_hi) == 0;
    return dist_all_ok(c, ok) ? 0 : -1;
}
}  // namespace

int ahip_dist_mode(const arpack_hip_dist* D) { return D ? D->D.mode : 0; }

extern "C" {

int arpack_hip_dist_create(arpack_hip_dist** out, arpack_hip_csr* A, int64_t n_global,
                           int64_t row0) {
    using namespace ahip;
    const Comm* c = comm_get();
    const int P = comm_size(c), r = comm_rank(c);
    const int64_t nloc = A->A.n;
    int64_t cmin = 0, cmax = -1;
    if (!dist_all_ok(c, ahip_csr_col_span(A, &cmin, &cmax) == 0)) return -1;
    if (cmax < 0) cmin = cmax = row0;  // empty operator block
    // share [row0, nloc, cmin, cmax] of every rank (allreduce of a one-hot table)
    std::vector<double> tab(4 * (size_t)P, 0.0);
    tab[4 * r + 0] = (double)row0;
    tab[4 * r + 1] = (double)nloc;
    tab[4 * r + 2] = (double)cmin;
    tab[4 * r + 3] = (double)cmax;
    double* d = nullptr;
    int ok_tab = hipMalloc(&d, sizeof(double) * tab.size()) == hipSuccess;
    if (!dist_all_ok(c, ok_tab)) {
        if (d) (void)hipFree(d);
        return -1;
    }
    ok_tab = hipMemcpy(d, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice) == hipSuccess;
    if (comm_allreduce_sum(c, d, (int)tab.size(), nullptr, false) != 0) ok_tab = 0;
    if (hipMemcpy(tab.data(), d, sizeof(double) * tab.size(), hipMemcpyDeviceToHost) != hipSuccess)
        ok_tab = 0;
    (void)hipFree(d);
    if (!dist_all_ok(c, ok_tab)) return -1;
    // the layout every plan needs, agreed from the shared table (so every rank
    // returns the same code): blocks contiguous from row 0 covering
    // [0, n_global), and every rank's columns inside [0, n_global) -- the
    // general plan's owner lookup and the remap assume both
    int64_t plan[4];
    {
        int64_t tot = 0;
        for (int q = 0; q < P; ++q) tot += (int64_t)tab[4 * q + 1];
        if (tot != n_global || (P > 0 && (int64_t)tab[0] != 0)) return -3;
        for (int q = 0; q < P; ++q) {
            if (q > 0 && (int64_t)tab[4 * q] != (int64_t)tab[4 * (q - 1)] + (int64_t)tab[4 * (q - 1) + 1])
                return -3;
            if ((int64_t)tab[4 * q + 1] > 0 &&
                ((int64_t)tab[4 * q + 2] < 0 || (int64_t)tab[4 * q + 3] >= n_global))
                return -1;
        }
    }
    int rc = arpack_hip_kit_halo_plan(P, r, tab.data(), plan);
    // -4: some rank's columns reach past its neighbours' rows (a general
    // operator): ghost lists or the all-gather instead of the slab halo.  A
    // valid slab halo wider than half the block (a few long-range entries
    // stretch the column span of a sparse coupling; a band is far narrower:
    // the north star's 4096 rows against a 1.25e6-row share) goes to the
    // general plan too, on every rank if on any.
    // (AHIP_DIST_GHOSTS=0: a valid slab halo is always kept)
    // A block declared symmetric on every rank keeps a valid slab halo whatever
    // its width: the upper-triangle SpMV it enables halves the matrix stream,
    // which no saving in halo rows repays, and a ghost-list block could only
    // run full storage (a wide band at small nloc lost symmetric
    // storage to the pricing).
    // A slab is "wide" when its halo rows exceed half of the block; a wide slab
    // goes to ghost lists only where the block's distinct ghost columns are
    // fewer than half of the slab's rows (a sparse long-range coupling) -- a
    // band or stencil reads nearly every slab row anyway (a 3-D stencil at 8
    // ranks: ghosts = halo planes), and keeps the slab, the symmetric-storage
    // form and its one neighbour exchange.
    const char* gv = std::getenv("AHIP_DIST_GHOSTS");
    const bool was_sym0 = A->A.kernel == ahip::dev::kCsrSymSell;
    const bool all_sym = dist_all_ok(c, was_sym0) != 0;  // collective: every rank calls it
    const bool price = !(gv && gv[0] == '0') && !all_sym;
    if (rc == 0 && P > 1 && price) {
        const bool wide = 2 * (plan[0] + plan[1]) > nloc;
        if (!dist_all_ok(c, !wide)) {  // some rank's slab is wide: count the ghosts
            std::vector<int64_t> g;
            bool sparse = false, gok = true;
            if (wide) {
                gok = ghost_cols(A, row0, nloc, g);
                sparse = 2 * (int64_t)g.size() < plan[0] + plan[1];
            }
            if (!dist_all_ok(c, gok)) return -1;
            if (!dist_all_ok(c, !sparse)) rc = -4;
        }
    }
    if (rc != 0 && rc != -4) return rc;
    auto* D = new arpack_hip_dist;
    DistOp& o = D->D;
    for (int q = 0; q < P; ++q) {
        o.peer_row0.push_back((int64_t)tab[4 * q]);
        o.peer_nloc.push_back((int64_t)tab[4 * q + 1]);
    }
    if (rc == -4) {
        o.n_global = n_global;
        o.row0 = row0;
        o.nloc = nloc;
        o.comm = c;
        o.comm_gen = comm_gen(c);
        const int grc = ghost_plan(A, o, c, P, r);
        if (grc != 0) {
            free_general(o);
            delete D;
            return grc;
        }
        o.A = &A->A;
        D->csr = A;
        if (A->dist) A->dist->csr = nullptr;
        A->dist = D;
        *out = D;
        return 0;
    }
    o.n_global = n_global;
    o.row0 = row0;
    o.nloc = nloc;
    o.halo_lo = plan[0];
    o.halo_hi = plan[1];
    o.send_lo = plan[2];
    o.send_hi = plan[3];
    o.comm = c;
    o.comm_gen = comm_gen(c);
    const int64_t next = o.halo_lo + nloc + o.halo_hi;
    // local column indices relative to x_ext; a failure on any rank fails the
    // call on every rank (the later collectives would otherwise mismatch)
    const bool was_sym = A->A.kernel == ahip::dev::kCsrSymSell;
    int ok = hipMalloc(&o.x_ext, sizeof(double) * (next > 0 ? next : 1)) == hipSuccess;
    if (ok) {
        (void)hipMemset(o.x_ext, 0, sizeof(double) * (next > 0 ? next : 1));
        A->sym_coff = o.halo_lo;
        A->sym_spill_in = o.send_lo;
        A->sym_spill_out = o.halo_hi;
        ok = ahip_csr_remap_cols(A, row0 - o.halo_lo, next) == 0;
    }
    if (!dist_all_ok(c, ok)) {
        if (o.x_ext) (void)hipFree(o.x_ext);
        delete D;
        return -1;
    }
    // storage mode agreed by all ranks: symmetric only if every rank declared it
    // and every rank's plan succeeds (arpack_hip_csr_set_symmetric is collective
    // from here on); otherwise every rank runs the full-storage SpMV (the remap
    // above already reset the kernel)
    o.A = &A->A;
    D->csr = A;
    if (A->dist) A->dist->csr = nullptr;  // a re-distributed block: the old handle lets go
    A->dist = D;
    if (dist_all_ok(c, was_sym)) (void)arpack_hip_csr_set_symmetric(A, 1);
    *out = D;
    return 0;
}

// Row-block decomposition without an operator (PARPACK's RCI use: the caller
// applies OP to its local rows and does its own halo exchange).
int arpack_hip_dist_rows(arpack_hip_dist** out, int64_t nloc, int64_t row0, int64_t n_global) {
    using namespace ahip;
    const Comm* c = comm_get();
    if (!c || nloc <= 0 || row0 < 0 || row0 + nloc > n_global) return -1;
    auto* D = new arpack_hip_dist;
    D->D.n_global = n_global;
    D->D.row0 = row0;
    D->D.nloc = nloc;
    D->D.comm = c;
    D->D.comm_gen = comm_gen(c);
    *out = D;
    return 0;
}

// y = A x over the row distribution (collective): x, y are this rank's rows
// in device memory.  The halo (and, for symmetric storage, the spill) exchange
// runs on the null stream.
int arpack_hip_dist_spmv(const arpack_hip_dist* D, const double* x, double* y) {
    if (!D || !D->D.A) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;  // the caller's x (see csr_spmv)
    ahip::dist_spmv(D->D, nullptr, x, y);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

void arpack_hip_dist_destroy(arpack_hip_dist* D) {
    if (!D) return;
    if (D->csr) D->csr->dist = nullptr;  // the CSR is a plain (unsharded) operator again
    free_general(D->D);
    delete D;
}

int arpack_hip_dist_mode(const arpack_hip_dist* D) { return D ? D->D.mode : -1; }

int arpack_hip_dist_info(const arpack_hip_dist* D, int64_t* halo_lo, int64_t* halo_hi,
                         int64_t* send_lo, int64_t* send_hi) {
    *halo_lo = D->D.halo_lo;
    *halo_hi = D->D.halo_hi;
    *send_lo = D->D.send_lo;
    *send_hi = D->D.send_hi;
    return 0;
}

int arpack_hip_dist_spill(const arpack_hip_dist* D) {
    if (!D || !D->csr || !D->D.A) return -1;
    const ahip::dev::Csr& A = *D->D.A;
    const bool sym = D->D.mode == ahip::DistOp::kHaloNeighbour && A.kernel == ahip::dev::kCsrSymSell &&
                     A.ss_val && !ahip::dev::csr_sym_det_fallback(A);
    return sym && !A.ss_lg ? 1 : 0;
}

}  // extern "C"

const ahip::DistOp* ahip_dist_view(const arpack_hip_dist* D) { return &D->D; }

// Called by arpack_hip_csr_destroy: the distribution loses its operator.
void ahip_dist_detach_csr(arpack_hip_dist* D) {
    if (!D) return;
    D->csr = nullptr;
    D->D.A = nullptr;
}

// The communicator of the distribution A belongs to, if that communicator is
// still the live one; stale (comm destroyed) -> *stale = true.
const ahip::Comm* ahip_csr_dist_comm(const arpack_hip_csr* A, bool* stale) {
    *stale = false;
    if (!A->dist) return nullptr;
    const ahip::DistOp& o = A->dist->D;
    if (!ahip::comm_alive(o.comm, o.comm_gen)) {
        *stale = true;
        return nullptr;
    }
    return o.comm;
}

