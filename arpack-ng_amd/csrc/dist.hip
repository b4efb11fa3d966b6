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

void dist_spmv(const DistOp& D, hipStream_t s, const double* x, double* y, bool p2p) {
    if (x != D.x_mid()) dev::copy(s, D.nloc, x, D.x_mid());
    const dev::Csr& A = *D.A;
    const bool sym = A.kernel == dev::kCsrSymSell && A.ss_val;
    comm_halo(D.comm, D, s, sym, p2p);
    if (sym) {
        // symmetric storage: my rows' upper entries reach the next rank's first
        // rows -- those transposed terms (the spill) travel forward and are
        // combined into the receiver's leading rows (a reverse halo)
        dev::csr_spmv_sym_main(s, A, D.x_ext, y);
        comm_spill(D.comm, A.ss_lo + A.ss_ncomb, A.ss_spill_out, A.ss_lo, D.send_lo, s, p2p);
        dev::csr_spmv_sym_combine(s, A, y);
        return;
    }
    dev::csr_spmv(s, A, D.x_ext, y);
}

int dist_all_ok(const Comm* c, int ok_local) {
    if (!c || comm_size(c) == 1) return ok_local != 0;
    // the communicator's own device double: no allocation that could fail on
    // one rank only, so every rank always joins the collective
    double h = ok_local ? 0.0 : 1.0, *d = comm_flag(c);  // SUM of failures
    bool ok = hipMemcpy(d, &h, sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    if (comm_allreduce_sum(c, d, 1, nullptr) != 0) ok = false;
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
    for (int q = 0; q < P; ++q) {  // contiguous blocks, halos only from the neighbours
        if (q > 0 && R0(q) != R0(q - 1) + NL(q - 1)) return -3;
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
    if (comm_allreduce_sum(c, d, (int)tab.size(), nullptr) != 0) ok_tab = 0;
    if (hipMemcpy(tab.data(), d, sizeof(double) * tab.size(), hipMemcpyDeviceToHost) != hipSuccess)
        ok_tab = 0;
    (void)hipFree(d);
    if (!dist_all_ok(c, ok_tab)) return -1;
    int64_t plan[4];
    const int rc = arpack_hip_kit_halo_plan(P, r, tab.data(), plan);
    if (rc != 0) return rc;
    auto* D = new arpack_hip_dist;
    DistOp& o = D->D;
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
    ahip::dist_spmv(D->D, nullptr, x, y);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

void arpack_hip_dist_destroy(arpack_hip_dist* D) {
    if (!D) return;
    if (D->csr) D->csr->dist = nullptr;  // the CSR is a plain (unsharded) operator again
    (void)hipFree(D->D.x_ext);
    delete D;
}

int arpack_hip_dist_info(const arpack_hip_dist* D, int64_t* halo_lo, int64_t* halo_hi,
                         int64_t* send_lo, int64_t* send_hi) {
    *halo_lo = D->D.halo_lo;
    *halo_hi = D->D.halo_hi;
    *send_lo = D->D.send_lo;
    *send_hi = D->D.send_hi;
    return 0;
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

